"""One resident grid (stencil_rolling_*): the job stencil_iterate runs on two
ping-pong grids (the reference's two owner buffers, stencil.cpp:14-21,
88-92), run in place with D spare planes, bitwise against the oracle and
against the two-grid path -- up to BASELINE config 3 itself, 4096^3 fp32 on
one GPU, where two grids do not fit."""
import numpy as np
import pytest

from oracle import binding as ob

pytestmark = pytest.mark.gpu


def same_bits(a, b):
    return a.shape == b.shape and np.array_equal(np.ascontiguousarray(a).view(np.uint8),
                                                 np.ascontiguousarray(b).view(np.uint8))


def spec(dtype, shape="star", r=1, kernel="auto"):
    from stencil_amd.engine import StencilSpec
    return StencilSpec(dims=3, dtype=dtype, shape=shape, radius=r, order="naive", kernel=kernel)


@pytest.mark.parametrize("dtype,shape,r,dims3", [
    ("fp64", "star", 1, (131, 61, 29)),   # K = 4
    ("fp32", "star", 1, (200, 90, 23)),   # K = 4 (small planes)
    ("fp32", "star", 1, (1024, 1024, 9)), # K = 5 (fp32 planes >= 1024^2: C3's kernel)
    ("fp64", "box", 1, (77, 40, 19)),     # K = 3
    ("fp64", "box", 1, (700, 650, 11)),   # K = 4 (box planes >= 384^2)
    ("fp64", "star", 2, (45, 23, 17)),    # single sweeps (direct kernel)
])
def test_rolling_matches_oracle(gpu, dtype, shape, r, dims3):
    """Every shift from the minimum (K + 1: one-plane launches) to more than
    the grid (one launch per pass), iteration counts with remainder passes,
    zero iterations, repeated calls continuing from the returned position."""
    from stencil_amd.engine import RollingGrid
    nx, ny, nz = dims3
    sp = spec(dtype, shape, r)
    p = ob.problem(3, dtype, shape, r, "naive", nx, ny, nz)
    probe = RollingGrid(sp, nx, ny, 1, 64, device=gpu)  # (the pass depth of this problem)
    k = probe.sweeps_per_pass
    del probe
    iters = sorted({0, 1, 2, k, k + 1, 2 * k + 3})
    for shift in (k * r + 1, k * r + 3, nz + k * r + 5):  # the minimum (one-plane launches) .. one launch per pass
        g = RollingGrid(sp, nx, ny, nz, shift, device=gpu)
        for it in iters:
            g.reset("random", 90 + it)
            g.iterate(it)
            assert same_bits(g.to_numpy(), ob.run(p, it, "random", 90 + it, threads=16)), (shift, it)
        # continuing: 3 then 4 more sweeps == 7 sweeps
        g.reset("random", 5)
        g.iterate(3)
        g.iterate(4)
        assert same_bits(g.to_numpy(), ob.run(p, 7, "random", 5, threads=16)), shift


def test_rolling_equals_two_grids_c3_planes(gpu):
    """4096^2 x 1024 fp32 7-point (C3's planes, a quarter of its depth), 40
    sweeps from the reference initial condition: the rolling job with the
    shift bench.py picks for C3 and the two-grid stencil_iterate, bitwise."""
    import gc
    import torch
    from stencil_amd.engine import JacobiEngine, RollingGrid
    gc.collect()
    torch.cuda.empty_cache()  # earlier tests' cached blocks: this test needs ~210 GB
    nx = ny = 4096
    nz, it = 1024, 40
    sp = spec("fp32")
    e = JacobiEngine(sp, nx, ny, nz, device=gpu)
    e.reset()
    fin, _ = e.iterate(it)
    want = e.interior(fin).clone()
    del e, fin
    torch.cuda.empty_cache()
    g = RollingGrid(sp, nx, ny, nz, 395, device=gpu)
    assert g.sweeps_per_pass == 5
    g.reset()
    _, _, launches = g.iterate(it)
    assert launches == 8 * 3  # 8 passes of ceil(1024 / 390) launches
    assert torch.equal(g.interior(), want)
    del g, want
    torch.cuda.empty_cache()


@pytest.mark.parametrize("case", ["C3", "C4"])
def test_full_size_on_one_gpu(gpu, case):
    """BASELINE configs 3 and 4 at their stated sizes on ONE GPU -- C3 4096^3
    fp32 (two grids would need 2 x 279 GB), C4 2048^2 x 4096 fp64 (2 x 138 GB)
    -- `it` sweeps of the rolling job from the reference initial condition
    (C3 10: two K = 5 passes; C4 8: two K = 4 passes).  Size-independent
    checks against the two-grid path on an nx x ny x 64 grid: after t sweeps
    plane z depends on planes z-t .. z+t only, so the deep grid's bottom 64-t
    planes equal the shallow grid's bottom 64-t, its top 64-t the shallow
    grid's top 64-t, and every plane in [t, nz - t) the shallow grid's plane
    32 -- bit for bit (whole planes compared on the GPU); plus the bitwise
    x-mirror symmetry of the reference initial condition."""
    import gc
    import torch
    from stencil_amd.engine import JacobiEngine, RollingGrid
    gc.collect()
    torch.cuda.empty_cache()  # earlier tests' cached blocks: this test needs the whole HBM
    dtype, nx, ny, nz, it = {"C3": ("fp32", 4096, 4096, 4096, 10), "C4": ("fp64", 2048, 2048, 4096, 8)}[case]
    sp = spec(dtype)
    e = JacobiEngine(sp, nx, ny, 64, device=gpu)
    e.reset()
    fin, _ = e.iterate(it)
    ref = e.interior(fin).clone()  # 64 planes, 4.3 GB (C3) / 2.1 GB (C4)
    del e, fin
    torch.cuda.empty_cache()
    free = torch.cuda.mem_get_info(gpu)[0]
    lay_plane = RollingGrid.bytes_needed(sp, nx, ny, 1, 64) - RollingGrid.bytes_needed(sp, nx, ny, 1, 63)
    grid_bytes = RollingGrid.bytes_needed(sp, nx, ny, nz, 6)
    shift = int(min(400, (free - grid_bytes - (2 << 30)) // lay_plane + 6))
    assert shift >= 40, f"free {free / 2**30:.1f} GiB leaves no room for the rolling margin"
    g = RollingGrid(sp, nx, ny, nz, shift, device=gpu)
    assert g.sweeps_per_pass == it // 2
    g.reset()
    g.iterate(it)
    got = g.interior()
    keep = 64 - it
    assert torch.equal(got[:keep], ref[:keep])
    assert torch.equal(got[nz - keep:], ref[64 - keep:])
    mid = ref[32]
    for z in range(it, nz - it, 1):
        assert torch.equal(got[z], mid), z
    assert torch.equal(got[100], torch.flip(got[100], dims=[1]))
    # values in [0, 1] (every plane of `got` is bitwise one of `ref`'s, checked above)
    assert float(ref.min()) >= 0.0 and float(ref.max()) <= 1.0
    del g, got, ref
    torch.cuda.empty_cache()


def test_fill_initial_beyond_2_32_elements(gpu):
    """The initial-condition fill of a grid of more than 2^32 elements
    (4096^2 x 300 fp32: 5.1e9 with ghosts and padding): every plane gets the
    reference condition and the random interior matches the splitmix64 rule
    at sampled cells of the last planes.  (A one-work-item-per-element
    dispatch is truncated modulo 2^32 work-items: before round 3 the fill
    left every plane past the first ~2^32 elements unset -- caught by the
    rolling tests at C3 size.)"""
    import torch
    from stencil_amd.engine import JacobiEngine
    nx, ny, nz = 4096, 4096, 300
    e = JacobiEngine(spec("fp32"), nx, ny, nz, device=gpu, allocate=False)
    assert int(e.layout.elems) > 2 ** 32
    e.a = torch.full((int(e.layout.elems) + 64,), 7.0, dtype=torch.float32, device=torch.device("cuda", gpu))
    e.fill_initial(e.a, "reference")
    g = e.with_ghosts(e.a)
    assert bool((g[:, :, 0] == 1).all()) and bool((g[:, :, -1] == 1).all())  # x-ghost faces, every plane
    assert float(e.interior(e.a).abs().max()) == 0.0
    assert float(g[:, 0, 1:-1].abs().max()) == 0.0 and float(g[-1, 1:-1, 1:-1].abs().max()) == 0.0
    e.fill_initial(e.a, "random", 5)
    inner = e.interior(e.a)
    m64 = (1 << 64) - 1

    def splitmix(x):
        z = (x + 0x9E3779B97F4A7C15) & m64
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & m64
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & m64
        return z ^ (z >> 31)
    for z, y, x in ((nz - 1, ny - 1, nx - 1), (nz - 1, 17, 4000), (299, 2048, 0), (150, 3, 5)):
        want = float(np.float32((splitmix(5 + (z * ny + y) * nx + x) >> 40) * 2.0 ** -24))
        assert float(inner[z, y, x]) == want, (z, y, x)
    del e, g, inner
    torch.cuda.empty_cache()
