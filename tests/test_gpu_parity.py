"""GPU parity: the HIP kernels (through the C-ABI) against the CPU oracle.

Bit-exact everywhere: every kernel performs the reference's additions and
multiply in the reference's order (naive = check_result, stencil.cpp:104-125;
dma = stencil_dma.cpp:431-444 / 636-650), compiled without FMA contraction and
without denormal flushing.
"""
import ctypes
import os
import subprocess

import numpy as np
import pytest

from oracle import binding as ob

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def engine(gpu, dims, dtype, shape, r, order, kernel, nx, ny, nz):
    from stencil_amd.engine import JacobiEngine, StencilSpec
    return JacobiEngine(StencilSpec(dims=dims, dtype=dtype, shape=shape, radius=r, order=order, kernel=kernel),
                        nx, ny, nz, device=gpu)


def gpu_run(gpu, dims, dtype, shape, r, order, kernel, nx, ny, nz, it, init="reference", seed=0):
    e = engine(gpu, dims, dtype, shape, r, order, kernel, nx, ny, nz)
    e.reset(init, seed)
    fin, _ = e.iterate(it)
    return e, e.to_numpy(fin)


def same_bits(a, b):
    return a.shape == b.shape and np.array_equal(a.view(np.uint8), b.view(np.uint8))


# ---------------------------------------------------------------- fixtures
def _fixture_cases():
    fx = np.load(os.path.join(GOLD, "oracle_fixtures.npz"))
    return [k for k in fx.files if not k.endswith("__meta")]


@pytest.mark.parametrize("name", _fixture_cases())
@pytest.mark.parametrize("kernel", ["direct", "auto"])
def test_golden_fixtures(gpu, name, kernel):
    fx = np.load(os.path.join(GOLD, "oracle_fixtures.npz"))
    dims, f64, box, r, dma, nx, ny, nz, it, rnd, seed = (int(x) for x in fx[name + "__meta"])
    e, g = gpu_run(gpu, dims, "fp64" if f64 else "fp32", "box" if box else "star", r, "dma" if dma else "naive",
                   kernel, nx, ny, nz, it, "random" if rnd else "reference", seed)
    p = ob.problem(dims, "fp64" if f64 else "fp32", "box" if box else "star", r, "dma" if dma else "naive", nx, ny, nz)
    assert same_bits(np.ascontiguousarray(ob.interior(p, g)), fx[name])


def _ref_fixture_cases():
    return sorted(np.load(os.path.join(GOLD, "ref_fixtures.npz")).files)


@pytest.mark.parametrize("name", _ref_fixture_cases())
@pytest.mark.parametrize("kernel", ["direct", "auto"])
def test_reference_build_fixtures(gpu, name, kernel):
    """Outputs of the reference's OWN compiled naive loop (oracle/ref/build.sh,
    tests/golden/make_ref_golden.py) -- the HIP kernels bit for bit."""
    a = np.load(os.path.join(GOLD, "ref_fixtures.npz"))[name]
    n, it, r, dt = name.split("_")
    n, it, r = int(n[1:]), int(it[1:]), int(r[1:])
    dtype = "fp64" if dt == "f64" else "fp32"
    e, g = gpu_run(gpu, 2, dtype, "star", r, "naive", kernel, n, n, 1, it)
    p = ob.problem(2, dtype, "star", r, "naive", n, n)
    assert same_bits(np.ascontiguousarray(ob.interior(p, g)), np.ascontiguousarray(a))


@pytest.mark.parametrize("name", [c for c in _ref_fixture_cases() if c.endswith("f32") and "_r1_" in c])
def test_reference_build_fixtures_static_unroll_abi(gpu, name):
    """The drop-in entry point stencil_iterate_dma_static_unroll (the reference
    variant whose sum order is the naive loop's), host buffers,
    parity-selected output -- equal to the reference build's bytes."""
    from stencil_amd import _lib
    lib = _lib.load()
    want = np.load(os.path.join(GOLD, "ref_fixtures.npz"))[name]
    n, it = int(name.split("_")[0][1:]), int(name.split("_")[1][1:])
    p = ob.problem(2, "fp32", "star", 1, "naive", n, n)
    a = ob.init(p)
    b = a.copy()

    def view(arr):
        return _lib.MatrixView(n + 2, n + 2, 1, 1, n + 2, arr.ctypes.data_as(ctypes.POINTER(ctypes.c_float)))
    args = _lib.Arguments(max(1, (n + 7) // 8), it, view(a), view(b))
    lib.stencil_iterate_dma_static_unroll(ctypes.byref(args))
    assert lib.stencil_last_error() == 0, lib.stencil_last_error_message()
    got = np.ascontiguousarray(ob.interior(p, b if it % 2 else a))
    assert same_bits(got, np.ascontiguousarray(want))


# ------------------------------------------------ reference configs (2D)
@pytest.mark.parametrize("dtype", ["fp32", "fp64"])
@pytest.mark.parametrize("order", ["naive", "dma"])
def test_c1_1024_100_iterations(gpu, dtype, order):
    """BASELINE config 1 (2D 5-point, 1024^2, 100 iterations)."""
    p = ob.problem(2, dtype, "star", 1, order, 1024, 1024)
    want = ob.run(p, 100, threads=8)
    _, got = gpu_run(gpu, 2, dtype, "star", 1, order, "auto", 1024, 1024, 1, 100)
    assert same_bits(got, want)
    if order == "naive":
        sums = {"fp32": 10520.714292108827, "fp64": 10520.714308906061}
        assert ob.interior_sum(p, got) == pytest.approx(sums[dtype], rel=1e-15, abs=0)


@pytest.mark.parametrize("r", [1, 2, 3, 5])
@pytest.mark.parametrize("order", ["naive", "dma"])
def test_2d_radius_random(gpu, r, order):
    p = ob.problem(2, "fp32", "star", r, order, 131, 77)
    want = ob.run(p, 9, "random", 42)
    _, got = gpu_run(gpu, 2, "fp32", "star", r, order, "auto", 131, 77, 1, 9, "random", 42)
    assert same_bits(got, want)


@pytest.mark.parametrize("k", ["1", "3", "8", "12"])
@pytest.mark.parametrize("r,order", [(1, "naive"), (1, "dma"), (2, "naive"), (2, "dma"), (3, "dma"), (4, "naive")])
@pytest.mark.parametrize("dtype", ["fp32", "fp64"])
@pytest.mark.parametrize("cfg", ["default", "8064", "4032", "16128", "12096", "8128", "92808", "92816", "92408",
                                 "94808", "92416", "92216", "192808", "192416"])
def test_2d_tile_resident_multistep(gpu, monkeypatch, k, r, order, dtype, cfg):
    """kernels_tb2d.hip: K sweeps per launch, every region shape of the LDS
    kernel and of the register-strip kernel (cfg 9xxxx, r <= 2; 19xxxx the
    same strip shape with branch-free ghost selects), ragged grids spanning
    several tiles, iteration counts that leave a partial last launch."""
    monkeypatch.setenv("STENCIL_TB2D_K", k)
    monkeypatch.setenv("STENCIL_TB2D_SINGLE", "0")  # the K-step launches even where one workgroup fits
    if cfg != "default":
        monkeypatch.setenv("STENCIL_TB2D_CFG", cfg)
    shape = cfg[1:] if len(cfg) == 6 else cfg
    strip = shape.startswith("9") and r <= 2
    rw = 64 * int(shape[1]) if strip else 64
    rh = {"default": 64, "8064": 64, "4032": 32, "16128": 128, "12096": 96, "8128": 128, "92808": 64, "92816": 128,
          "92408": 32, "94808": 64, "92416": 64, "92216": 32}[shape] if (strip or not shape.startswith("9")) else 64
    if min(rw, rh) - 2 * min(int(k), 24 // r) * r < 4:
        pytest.skip("no tile left in this region for K sweeps")
    for nx, ny, it in ((301, 170, 11), (5, 3, 4), (64, 200, 9)):
        p = ob.problem(2, dtype, "star", r, order, nx, ny)
        want = ob.run(p, it, "random", 8 + r)
        _, got = gpu_run(gpu, 2, dtype, "star", r, order, "temporal2", nx, ny, 1, it, "random", 8 + r)
        assert same_bits(got, want), (nx, ny, it)


@pytest.mark.parametrize("r,order", [(1, "naive"), (1, "dma"), (2, "naive"), (2, "dma"), (3, "dma"), (4, "naive")])
@pytest.mark.parametrize("dtype", ["fp32", "fp64"])
def test_2d_single_workgroup(gpu, r, order, dtype):
    """Grids that fit one workgroup's LDS run every sweep in one launch
    (kernels_tb2d.hip tb2d1): odd and even iteration counts (the result lands
    where the ping-pong would leave it), ragged, one-cell and one-row grids,
    the largest grids that take the path and the first that do not."""
    esz = 4 if dtype == "fp32" else 8
    for nx, ny, it in ((32, 32, 3), (64, 64, 100), (1, 1, 2), (77, 13, 7), (5120, 1, 5), (80, 64, 5), (71, 72, 4),
                       (40, 40, 0)):
        p = ob.problem(2, dtype, "star", r, order, nx, ny)
        want = ob.run(p, it, "random", 3 + r)
        e, got = gpu_run(gpu, 2, dtype, "star", r, order, "auto", nx, ny, 1, it, "random", 3 + r)
        assert same_bits(got, want), (nx, ny, it)
        single = nx * ny <= 5120 and 2 * (nx + 2 * r) * (ny + 2 * r) * esz <= 160 * 1024
        if it and single:
            assert e.plan(it)[0] == 1, (nx, ny, it)


@pytest.mark.parametrize("k", ["1", "3", "8", "12"])
@pytest.mark.parametrize("r,order", [(1, "naive"), (1, "dma"), (2, "naive"), (2, "dma")])
@pytest.mark.parametrize("dtype", ["fp32", "fp64"])
def test_2d_persistent(gpu, monkeypatch, k, r, order, dtype):
    """kernels_tb2dp.hip: the whole job in one cooperative launch, K-sweep
    blocks between neighbour-flag waits; ragged grids, iteration counts below,
    at and between multiples of K, zero iterations; a K whose ring does not fit
    the region falls back to the K-step launches."""
    from stencil_amd import _lib
    monkeypatch.setenv("STENCIL_TB2DP_K", k)
    kk = min(int(k), 24 // r)
    fits_region = 128 - 2 * kk * r >= max(4, kk * r) and 64 - 2 * kk * r >= max(4, kk * r)
    for nx, ny, it in ((301, 170, 11), (5, 3, 4), (64, 200, 9), (257, 129, 1), (130, 66, 2 * kk), (40, 40, 0)):
        p = ob.problem(2, dtype, "star", r, order, nx, ny)
        want = ob.run(p, it, "random", 8 + r)
        e, got = gpu_run(gpu, 2, dtype, "star", r, order, "persistent", nx, ny, 1, it, "random", 8 + r)
        assert same_bits(got, want), (nx, ny, it)
        launches, kernel = e.plan(it)
        if fits_region and it:
            assert (launches, kernel) == (1, _lib.KERNEL_PERSISTENT)
        else:
            assert kernel != _lib.KERNEL_PERSISTENT or it == 0


@pytest.mark.parametrize("dtype", ["fp32", "fp64"])
@pytest.mark.parametrize("order", ["naive", "dma"])
def test_c1_persistent(gpu, dtype, order):
    """BASELINE config 1 through the persistent kernel: one launch, bitwise the
    oracle (and the probe's golden sum for the naive order)."""
    from stencil_amd import _lib
    p = ob.problem(2, dtype, "star", 1, order, 1024, 1024)
    want = ob.run(p, 100, threads=8)
    e, got = gpu_run(gpu, 2, dtype, "star", 1, order, "persistent", 1024, 1024, 1, 100)
    assert e.plan(100) == (1, _lib.KERNEL_PERSISTENT)
    assert same_bits(got, want)
    if order == "naive":
        sums = {"fp32": 10520.714292108827, "fp64": 10520.714308906061}
        assert ob.interior_sum(p, got) == pytest.approx(sums[dtype], rel=1e-15, abs=0)


def test_persistent_too_large_falls_back(gpu):
    """More tiles than resident workgroups: the K-step launches run instead."""
    from stencil_amd import _lib
    p = ob.problem(2, "fp64", "star", 1, "naive", 8000, 6000)
    want = ob.run(p, 3, "random", 3, threads=8)
    e, got = gpu_run(gpu, 2, "fp64", "star", 1, "naive", "persistent", 8000, 6000, 1, 3, "random", 3)
    assert e.plan(3)[1] != _lib.KERNEL_PERSISTENT
    assert same_bits(got, want)


# ------------------------------------------------------- 3D hot kernels
@pytest.mark.parametrize("stencil", ["star", "box"])
@pytest.mark.parametrize("dtype", ["fp32", "fp64"])
@pytest.mark.parametrize("kernel", ["direct", "zmarch", "temporal2", "temporalk"])
@pytest.mark.parametrize("shape3", [(64, 16, 8), (130, 37, 29), (1, 1, 1), (65, 17, 3), (200, 3, 70), (124, 28, 2),
                                    (249, 57, 11)])
def test_3d_r1_random_ragged(gpu, stencil, dtype, kernel, shape3):
    """7-point star and 27-point box, r = 1, every kernel family."""
    if kernel == "temporalk" and stencil == "box":
        pytest.skip("TEMPORALK is the 7-point star family")
    nx, ny, nz = shape3
    p = ob.problem(3, dtype, stencil, 1, "naive", nx, ny, nz)
    for it in (1, 2, 5, 7):
        want = ob.run(p, it, "random", 1234 + it)
        _, got = gpu_run(gpu, 3, dtype, stencil, 1, "naive", kernel, nx, ny, nz, it, "random", 1234 + it)
        assert same_bits(got, want), (it, shape3)


@pytest.mark.parametrize("t2cfg", ["default", "216", "1312"])
@pytest.mark.parametrize("zchunk", ["8", "9", "16"])
@pytest.mark.parametrize("dtype", ["fp32", "fp64"])
@pytest.mark.parametrize("stencil", ["star", "box"])
def test_temporal2_chunking(gpu, monkeypatch, zchunk, dtype, stencil, t2cfg):
    """Fused two-step launches with forced z-chunk sizes (chunk seams,
    remainder chunks), odd iteration counts (a trailing single sweep), for the
    default LDS-centre kernel and the register-ring shapes kept for A/B."""
    if t2cfg != "default":
        monkeypatch.setenv("STENCIL_T2_CFG", t2cfg)
    monkeypatch.setenv("STENCIL_T2_ZCHUNK", zchunk)
    monkeypatch.setenv("STENCIL_BOX_ZCHUNK", zchunk)
    nx, ny, nz = 131, 61, 29
    p = ob.problem(3, dtype, stencil, 1, "naive", nx, ny, nz)
    for it in (2, 3, 6):
        want = ob.run(p, it, "random", 99 + it)
        _, got = gpu_run(gpu, 3, dtype, stencil, 1, "naive", "temporal2", nx, ny, nz, it, "random", 99 + it)
        assert same_bits(got, want), it


@pytest.mark.parametrize("steps,cfg", [("3", "default"), ("3", "312"), ("3", "608"), ("3", "216"), ("3", "20312"), ("3", "30216"), ("3", "40216"), ("4", "default"),
                                       ("4", "408")])
@pytest.mark.parametrize("zchunk", ["0", "4", "7", "16"])
@pytest.mark.parametrize("dtype", ["fp32", "fp64"])
def test_temporalk_chunking(gpu, monkeypatch, steps, cfg, zchunk, dtype):
    """K = 3 / 4 fused sweeps per launch: every workgroup shape, forced z-chunk
    sizes (seams, remainder chunks, chunks shorter than the 2K-plane halo) and
    iteration counts leaving a remainder pair / single sweep."""
    monkeypatch.setenv("STENCIL_TK_STEPS", steps)
    monkeypatch.setenv("STENCIL_TK_ZCHUNK", zchunk)
    monkeypatch.setenv("STENCIL_TK_STRIP", "0")  # the interleaved-row layout (kernels_temporalk.hip)
    if cfg != "default":
        monkeypatch.setenv("STENCIL_TK_CFG", cfg)
    nx, ny, nz = 131, 61, 29
    p = ob.problem(3, dtype, "star", 1, "naive", nx, ny, nz)
    for it in (3, 4, 5, 9):
        want = ob.run(p, it, "random", 7 + it)
        e, got = gpu_run(gpu, 3, dtype, "star", 1, "naive", "temporalk", nx, ny, nz, it, "random", 7 + it)
        assert same_bits(got, want), it
    k = int(steps)
    assert e.plan(9) == (9 // k + (9 % k) // 2 + (9 % k) % 2, 4)


@pytest.mark.parametrize("steps,strip", [("3", "1"), ("3", "416"), ("3", "10408"), ("3", "216"), ("3", "10808"),
                                         ("3", "20808"), ("4", "1"), ("4", "10708"), ("4", "10608"), ("4", "20708"),
                                         ("5", "1"), ("5", "10608"), ("5", "20608"),
                                         # stage 1's history in LDS (HL)
                                         ("4", "810808"), ("4", "810708"), ("5", "810708"), ("5", "810608"),
                                         ("4", "820908"), ("5", "830708"), ("5", "820608"),
                                         # the default shape without the interior fast path
                                         ("4", "710708"),
                                         # the default shapes from kernels_strip.hip's own build ("1": AUTO, the
                                         # max-ILP build kernels_strip_ilp.hip on these small grids)
                                         ("5", "20508"),
                                         # SPLIT: two strips per wave, 16-B lane vectors (fp32 4 / fp64 2 cells
                                         # per lane; each cfg is one dtype's shape, the other dtype runs AUTO)
                                         ("5", "1040208"), ("5", "1030308"), ("5", "1830308"), ("5", "1030212"),
                                         ("4", "1020408"), ("4", "1020308"), ("4", "1820408")])
@pytest.mark.parametrize("zchunk", ["0", "4", "7", "16"])
@pytest.mark.parametrize("dtype", ["fp32", "fp64"])
@pytest.mark.parametrize("shape3", [(131, 61, 29), (64, 7, 9), (250, 100, 12)])
def test_tkstrip_chunking(gpu, monkeypatch, steps, strip, zchunk, dtype, shape3):
    """The strip layout of the K-step kernel (kernels_strip.hip: consecutive
    rows per wave, boundary rows through LDS): every shape, forced z-chunks,
    remainders, grids shorter than one strip region."""
    monkeypatch.setenv("STENCIL_TK_STEPS", steps)
    monkeypatch.setenv("STENCIL_TK_ZCHUNK", zchunk)
    monkeypatch.setenv("STENCIL_TK_STRIP", strip)
    nx, ny, nz = shape3
    p = ob.problem(3, dtype, "star", 1, "naive", nx, ny, nz)
    for it in (3, 4, 7):
        want = ob.run(p, it, "random", 17 + it)
        _, got = gpu_run(gpu, 3, dtype, "star", 1, "naive", "temporalk", nx, ny, nz, it, "random", 17 + it)
        assert same_bits(got, want), it


@pytest.mark.parametrize("dtype", ["fp64", "fp32"])
@pytest.mark.parametrize("steps", ["3", "4", "5"])
@pytest.mark.parametrize("fast", ["0", "1", "4", "5"])
@pytest.mark.parametrize("zchunk", ["0", "5", "11"])
def test_tkstrip_interior_fast_path(gpu, monkeypatch, dtype, steps, fast, zchunk):
    """The strip kernel skips the intermediate stages' ghost-cell select
    where the region lies inside the grid in x and y and the stage planes in
    z (STENCIL_TK_FAST bits): per step (1, fp64 one-cell-per-lane shapes) or
    per segment (4, every shape: a tile's z-chunk whose reach stays off the z
    ends).  Interior and edge tiles, z-chunk seams and the z ends, bitwise
    equal to the oracle whichever way."""
    monkeypatch.setenv("STENCIL_TK_STEPS", steps)
    monkeypatch.setenv("STENCIL_TK_ZCHUNK", zchunk)
    monkeypatch.setenv("STENCIL_TK_FAST", fast)
    nx, ny, nz = 300, 250, 40
    p = ob.problem(3, dtype, "star", 1, "naive", nx, ny, nz)
    for it in (int(steps), 2 * int(steps) + 1):
        want = ob.run(p, it, "random", 41 + it)
        _, got = gpu_run(gpu, 3, dtype, "star", 1, "naive", "temporalk", nx, ny, nz, it, "random", 41 + it)
        assert same_bits(got, want), it


@pytest.mark.parametrize("dtype", ["fp32", "fp64"])
def test_tkstrip_packed_schedule_small_shapes(gpu, dtype):
    """The default K-step launch (packed longest-first z-chunks where the
    host's makespan model picks them) at shapes of few tiles, bitwise against
    the oracle; the geometry query shows which launches were packed, and at
    least one of these shapes must be."""
    shapes = [(131, 61, 29), (200, 200, 200), (300, 200, 150), (512, 512, 96), (600, 100, 64), (64, 7, 90)]
    packed = []
    for nx, ny, nz in shapes:
        e = engine(gpu, 3, dtype, "star", 1, "naive", "auto", nx, ny, nz)
        k = e.fuse_steps
        geo = e.sweepk_geometry(k)
        packed.append(geo["packed"])
        it = 2 * k + 1
        p = ob.problem(3, dtype, "star", 1, "naive", nx, ny, nz)
        want = ob.run(p, it, "random", 31)
        e.reset("random", 31)
        fin, _ = e.iterate(it)
        assert same_bits(e.to_numpy(fin), want), ((nx, ny, nz), geo)
    assert any(packed), list(zip(shapes, packed))


@pytest.mark.parametrize("shape", ["star", "box"])
@pytest.mark.parametrize("mode", ["1", "2", "0"])
def test_schedule_choice_modes(gpu, monkeypatch, shape, mode):
    """Packed vs equal z-chunks (kernels_strip.hip pick_schedule): mode 1 (the
    default) times both grids on the first launch of a shape and keeps the
    faster -- six trial launches, all writing the same output; mode 2 launches
    the dispatcher model's choice unmeasured (packed here); mode 0 equal chunks.
    256^3 fp64 is a shape the model packs (and where the measured choice is
    equal chunks on MI355X, profiles/r02gg_pack.log).  Every mode bitwise
    against the oracle, over two launches (the trial, then the verdict)."""
    monkeypatch.setenv("STENCIL_TK_PACK", mode)
    monkeypatch.setenv("STENCIL_BOXK_PACK", mode)
    nx = ny = nz = 256
    e = engine(gpu, 3, "fp64", shape, 1, "naive", "auto", nx, ny, nz)
    k = e.fuse_steps
    if shape == "star":
        assert e.sweepk_geometry(k)["packed"] == (mode != "0")  # before any launch: the model's plan
    it = 2 * k + 1
    p = ob.problem(3, "fp64", shape, 1, "naive", nx, ny, nz)
    want = ob.run(p, it, "random", 19, threads=16)
    e.reset("random", 19)
    fin, _ = e.iterate(it)
    assert same_bits(e.to_numpy(fin), want)
    if shape == "star" and mode == "2":
        assert e.sweepk_geometry(k)["packed"]


@pytest.mark.parametrize("shape", ["star", "box"])
def test_prepare_leaves_grid_a(gpu, shape):
    """stencil_prepare (the one-time schedule trial ahead of a timed run, as
    bench.py and stencil_main do it) writes only grid b: grid a is bitwise
    unchanged, and the job that follows equals the oracle."""
    import torch
    nx, ny, nz = 200, 180, 96
    e = engine(gpu, 3, "fp64", shape, 1, "naive", "auto", nx, ny, nz)
    e.reset("random", 23)
    before = e.a.clone()
    e.prepare()
    torch.cuda.synchronize()
    assert torch.equal(before.view(torch.int64), e.a.view(torch.int64))
    it = 2 * e.fuse_steps + 1
    p = ob.problem(3, "fp64", shape, 1, "naive", nx, ny, nz)
    want = ob.run(p, it, "random", 23, threads=16)
    fin, _ = e.iterate(it)
    assert same_bits(e.to_numpy(fin), want)


@pytest.mark.parametrize("cfg", ["default", "216", "408", "308", "208", "10116", "10216", "20116"])
@pytest.mark.parametrize("zchunk", ["0", "4", "7", "16"])
@pytest.mark.parametrize("dtype", ["fp32", "fp64"])
def test_boxk_chunking(gpu, monkeypatch, cfg, zchunk, dtype):
    """27-point box, two fused sweeps per launch through the separable-sum box
    kernel (kernels_boxk.hip): workgroup shapes (incl. spilling ones), forced
    z-chunks shorter and longer than the 3K-plane pipeline fill, odd iteration
    counts (the remainder single sweep is the same kernel with K = 1)."""
    monkeypatch.setenv("STENCIL_BOXK_ZCHUNK", zchunk)
    if cfg != "default":
        monkeypatch.setenv("STENCIL_BOXK_CFG", cfg)
    nx, ny, nz = 131, 61, 29
    p = ob.problem(3, dtype, "box", 1, "naive", nx, ny, nz)
    for it in (2, 3, 4, 5):
        want = ob.run(p, it, "random", 21 + it)
        _, got = gpu_run(gpu, 3, dtype, "box", 1, "naive", "temporal2", nx, ny, nz, it, "random", 21 + it)
        assert same_bits(got, want), it


@pytest.mark.parametrize("dtype", ["fp32", "fp64"])
@pytest.mark.parametrize("shape3", [(131, 61, 29), (7, 5, 3), (250, 19, 12)])
@pytest.mark.parametrize("cfg", ["default", "10116", "216", "20116", "416", "208"])
@pytest.mark.parametrize("zchunk", ["0", "5"])
def test_boxk_three_steps(gpu, monkeypatch, dtype, shape3, cfg, zchunk):
    """stencil_sweepk(3) on the 27-point box (AUTO's box launch) equals three
    plain sweeps, every workgroup shape, forced short z-chunks; and a whole
    job through AUTO (3-sweep launches + remainder pair / single)."""
    if cfg != "default":
        monkeypatch.setenv("STENCIL_BOXK_CFG", cfg)
    monkeypatch.setenv("STENCIL_BOXK_ZCHUNK", zchunk)
    nx, ny, nz = shape3
    p = ob.problem(3, dtype, "box", 1, "naive", nx, ny, nz)
    want = ob.run(p, 3, "random", 5)
    e = engine(gpu, 3, dtype, "box", 1, "naive", "auto", nx, ny, nz)
    e.reset("random", 5)
    e.sweepk(e.a, e.b, 0, nz, 3)
    assert same_bits(e.to_numpy(e.b), want)
    for it in (7, 8):
        e.reset("random", 5)
        fin, _ = e.iterate(it)
        assert same_bits(e.to_numpy(fin), ob.run(p, it, "random", 5)), it
    assert e.plan(8) == (3, 3)


BOX_STRIP_CFGS = {"fp64": {4: ["910308", "910408", "910508", "910216"],
                            3: ["910408", "910308", "910312", "910212", "910216", "910608"],
                            2: ["910408", "910312", "910216"], 1: ["920408"], 5: ["910408"]},
                   "fp32": {4: ["920308", "920408", "920508"], 3: ["920408", "920312", "920216", "920608"],
                            2: ["920408", "920312", "940208"], 1: ["940408"], 5: ["920408"]}}


@pytest.mark.parametrize("dtype", ["fp32", "fp64"])
@pytest.mark.parametrize("steps", [1, 2, 3, 4, 5])
@pytest.mark.parametrize("shape3", [(131, 61, 29), (7, 5, 3), (250, 119, 12), (64, 300, 40)])
@pytest.mark.parametrize("zchunk", ["0", "5", "13"])
def test_box_strip_shapes(gpu, monkeypatch, dtype, steps, shape3, zchunk):
    """The strip layout of the box kernel (box27_strip: consecutive rows per
    wave, only the strips' first / last row sums through LDS), every shape
    instantiated for the step count: stencil_sweepk(K) bitwise equal to K
    sweeps of the oracle, ragged tiles, forced short z-chunks."""
    monkeypatch.setenv("STENCIL_BOXK_ZCHUNK", zchunk)
    nx, ny, nz = shape3
    p = ob.problem(3, dtype, "box", 1, "naive", nx, ny, nz)
    want = ob.run(p, steps, "random", 17)
    for cfg in BOX_STRIP_CFGS[dtype][steps]:
        monkeypatch.setenv("STENCIL_BOXK_CFG", cfg)
        e = engine(gpu, 3, dtype, "box", 1, "naive", "auto", nx, ny, nz)
        e.reset("random", 17)
        e.sweepk(e.a, e.b, 0, nz, steps)
        assert same_bits(e.to_numpy(e.b), want), cfg


@pytest.mark.parametrize("shape,steps", [("star", 3), ("star", 4), ("box", 2), ("box", 3)])
@pytest.mark.parametrize("dtype", ["fp32", "fp64"])
def test_temporalk_signed_zero_field(gpu, shape, steps, dtype):
    """The K-step kernel folds the reference's leading `0 +` into
    fma(sum, avg, +0); a block of -0.0 cells (where 0 + -0 = +0 matters) and
    mixed-sign data must still match plain sweeps bit for bit."""
    import torch
    nx, ny, nz = 77, 40, 23
    e = engine(gpu, 3, dtype, shape, 1, "naive", "temporalk" if shape == "star" else "temporal2", nx, ny, nz)
    e.reset("random", 11)
    full = e.with_ghosts(e.a)
    inner = e.interior(e.a)
    inner[3:15, 5:30, 10:60] = -0.0
    inner[15:20] *= -1.0
    torch.cuda.synchronize()
    start = full.cpu().numpy().copy()
    p = ob.problem(3, dtype, shape, 1, "naive", nx, ny, nz)
    a, b = start.copy(), start.copy()
    for _ in range(steps):
        ob.sweep(p, a, b, 0, nz)
        a, b = b, a
    e.sweepk(e.a, e.b, 0, nz, steps)
    torch.cuda.synchronize()
    got = e.with_ghosts(e.b).cpu().numpy()
    assert same_bits(np.ascontiguousarray(got), np.ascontiguousarray(a))


@pytest.mark.parametrize("r,order", [(1, "naive"), (1, "dma"), (2, "naive"), (2, "dma")])
@pytest.mark.parametrize("dtype", ["fp32", "fp64"])
@pytest.mark.parametrize("cfg", ["default", "92416", "92808"])
def test_2d_strip_signed_zero_field(gpu, monkeypatch, r, order, dtype, cfg):
    """The 2D strip region folds the reference's leading `0 +` into
    fma(sum, avg, +0) (strip2d.hpp fma0): a block of -0.0 cells with -0.0
    ghosts beside it (where 0 + -0 = +0 matters) and mixed-sign data, through
    AUTO's K-step launches, bit for bit the oracle's plain sweeps."""
    import torch
    if cfg != "default":
        monkeypatch.setenv("STENCIL_TB2D_CFG", cfg)
    nx, ny, it = 301, 170, 23
    e = engine(gpu, 2, dtype, "star", r, order, "auto", nx, ny, 1)
    e.reset("random", 13)
    full = e.with_ghosts(e.a)
    full[:, : nx // 3] = -0.0          # ghost column and ghost rows included
    full[60:90, :] *= -1.0
    full[100:110, 200:] = 0.0
    torch.cuda.synchronize()
    start = full.cpu().numpy().copy()
    e.with_ghosts(e.b).copy_(full)
    p = ob.problem(2, dtype, "star", r, order, nx, ny)
    a, b = start.copy(), start.copy()
    for _ in range(it):
        ob.sweep(p, a, b, 0, ny)
        a, b = b, a
    assert (np.signbit(a) & (a == 0)).any() and (~np.signbit(a) & (a == 0)).any()
    fin, _ = e.iterate(it)
    assert same_bits(e.to_numpy(fin), a)


@pytest.mark.parametrize("dtype", ["fp32", "fp64"])
@pytest.mark.parametrize("zchunk", ["0", "3", "8"])
def test_box_single_sweeps(gpu, monkeypatch, dtype, zchunk):
    """The box's single sweep (the K = 1 instance of kernels_boxk.hip) over the
    whole grid and over sub-ranges of planes."""
    monkeypatch.setenv("STENCIL_BOXK_ZCHUNK", zchunk)
    nx, ny, nz = 150, 47, 21
    p = ob.problem(3, dtype, "box", 1, "naive", nx, ny, nz)
    for it in (1, 3):
        want = ob.run(p, it, "random", 3)
        _, got = gpu_run(gpu, 3, dtype, "box", 1, "naive", "zmarch", nx, ny, nz, it, "random", 3)
        assert same_bits(got, want), it
    e = engine(gpu, 3, dtype, "box", 1, "naive", "zmarch", nx, ny, nz)
    e.reset("random", 9)
    import torch
    ref = e.to_numpy(e.a).copy()
    e.sweep(e.a, e.b, 4, 13)
    torch.cuda.synchronize()
    a = ref.copy()
    b = ref.copy()
    ob.sweep(p, a, b, 4, 13)
    got = e.to_numpy(e.b)
    assert same_bits(got[4 + 1:13 + 1], b[4 + 1:13 + 1])


def test_sweep2_subrange(gpu):
    """stencil_sweep2 on a slab sub-range equals two plain sweeps there."""
    nx, ny, nz = 70, 33, 24
    e = engine(gpu, 3, "fp64", "star", 1, "naive", "auto", nx, ny, nz)
    e.reset("random", 5)
    import torch
    ref = e.a.clone()
    # plain: two sweeps of the whole grid, then take planes [6, 18)
    e.sweep(e.a, e.b, 0, nz)
    e.sweep(e.b, ref, 0, nz)
    e.reset("random", 5)
    out = e.b
    e.sweep2(e.a, out, 6, 18)
    torch.cuda.synchronize()
    gi, ri = e.interior(out), e.interior(ref)
    assert torch.equal(gi[6:18], ri[6:18])


@pytest.mark.parametrize("shape,r", [("box", 1), ("star", 2), ("star", 3), ("box", 2)])
def test_3d_other_shapes(gpu, shape, r):
    p = ob.problem(3, "fp64", shape, r, "naive", 45, 23, 17)
    want = ob.run(p, 3, "random", 5)
    _, got = gpu_run(gpu, 3, "fp64", shape, r, "naive", "auto", 45, 23, 17, 3, "random", 5)
    assert same_bits(got, want)


def test_zero_iterations_and_empty(gpu):
    p = ob.problem(3, "fp64", "star", 1, "naive", 20, 10, 5)
    _, got = gpu_run(gpu, 3, "fp64", "star", 1, "naive", "auto", 20, 10, 5, 0, "random", 9)
    assert same_bits(got, ob.init(p, "random", 9))
    e = engine(gpu, 3, "fp64", "star", 1, "naive", "auto", 0, 4, 4)
    e.reset()
    e.iterate(3)  # empty interior: nothing to do, must not fault


def test_full_size_c2_bitwise_few_iterations(gpu):
    """BASELINE config 2 size (512^3 fp64 7-point) at full size: bitwise
    against the oracle for 3 sweeps (the oracle's multithreaded run takes a
    few seconds), and the two kernel families bitwise against each other."""
    n = 512
    p = ob.problem(3, "fp64", "star", 1, "naive", n, n, n)
    want = ob.run(p, 3, "random", 77, threads=16)
    _, got = gpu_run(gpu, 3, "fp64", "star", 1, "naive", "auto", n, n, n, 3, "random", 77)
    assert same_bits(got, want)


def test_full_size_c2_1000_iterations_properties(gpu):
    """The whole config-2 job (1000 sweeps, reference initial condition):
    ghost cells untouched, bitwise x-mirror symmetry (0+L+R == 0+R+L), all
    values in [0, 1], plane checksums identical across kernel families --
    AUTO (the benched K = 4 strip launches), the single-sweep z-march and the
    direct kernel, whole grids bitwise equal."""
    import torch
    n = 512
    e = engine(gpu, 3, "fp64", "star", 1, "naive", "zmarch", n, n, n)
    e.reset()
    init = e.with_ghosts(e.a).clone()
    fin, _ = e.iterate(1000)
    g = e.with_ghosts(fin)
    inner = e.interior(fin)
    assert torch.equal(inner, torch.flip(inner, dims=[2]))
    assert float(inner.min()) >= 0.0 and float(inner.max()) <= 1.0
    mask = torch.ones_like(g, dtype=torch.bool)
    mask[1:-1, 1:-1, 1:-1] = False
    assert torch.equal(g[mask], init[mask])
    sums_zm = e.plane_sums(fin)
    for kernel in ("direct", "auto"):
        e2 = engine(gpu, 3, "fp64", "star", 1, "naive", kernel, n, n, n)
        e2.reset()
        fin2, _ = e2.iterate(1000)
        assert np.array_equal(sums_zm, e2.plane_sums(fin2)), kernel
        assert torch.equal(e2.interior(fin2), inner), kernel
        del e2, fin2
    torch.cuda.empty_cache()


def test_c2_whole_benched_job_against_oracle(gpu):
    """The headline job exactly as bench.py times it -- BASELINE config 2,
    512^3 fp64 7-point from the reference initial condition, 1000 sweeps
    through AUTO = 250 K = 4 strip launches on the packed schedule the first
    launch measured faster -- bitwise against the oracle's naive loop
    (stencil.cpp:94-131 generalised to 3D, multithreaded, same per-cell
    arithmetic) over the WHOLE job, not a few sweeps."""
    import torch
    from stencil_amd import _lib
    n, it = 512, 1000
    e = engine(gpu, 3, "fp64", "star", 1, "naive", "auto", n, n, n)
    assert e.fuse_steps == 4
    assert e.plan(it) == (250, _lib.KERNEL_TEMPORALK)
    # bench.py first picks the fastest of a few grid placements
    placed = e.place(trials=3)
    assert placed["candidates"] == 3 and 0 <= placed["chosen"] < 3
    assert placed["ms_per_launch"][placed["chosen"]] == min(placed["ms_per_launch"])
    e.reset()
    e.prepare()  # bench.py settles the schedule first; grid a is unchanged
    fin, _ = e.iterate(it)
    assert e.sweepk_geometry(4)["packed"], "the measured choice at the C2 shape is packed (bench.py's launch)"
    got = e.interior(fin).cpu().numpy()
    del e, fin
    torch.cuda.empty_cache()
    p = ob.problem(3, "fp64", "star", 1, "naive", n, n, n)
    want = ob.interior(p, ob.run(p, it, threads=16))
    assert np.array_equal(got.view(np.uint8), np.ascontiguousarray(want).view(np.uint8))
    # the diffusion fronts have reached every cell, so the job is not trivially zero anywhere
    assert float(want.min()) > 0.0


def test_c5_slab_reference_job_against_oracle(gpu):
    """One GPU's slab of BASELINE config 5 (2048^2 x 256 27-point box, fp64)
    from the reference initial condition, 12 sweeps through AUTO = three K = 4
    box strip launches (the benched kernel), bitwise against the oracle."""
    import torch
    from stencil_amd import _lib
    nx, ny, nz, it = 2048, 2048, 256, 12
    e = engine(gpu, 3, "fp64", "box", 1, "naive", "auto", nx, ny, nz)
    assert e.fuse_steps == 4
    assert e.plan(it) == (3, _lib.KERNEL_TEMPORAL2)
    e.reset()
    fin, _ = e.iterate(it)
    got = e.interior(fin).cpu().numpy()
    del e, fin
    torch.cuda.empty_cache()
    p = ob.problem(3, "fp64", "box", 1, "naive", nx, ny, nz)
    want = ob.interior(p, ob.run(p, it, threads=16))
    assert np.array_equal(got.view(np.uint8), np.ascontiguousarray(want).view(np.uint8))


def test_c5_as_benched_whole_2048_cube(gpu):
    """BASELINE config 5 as bench.py --config C5 runs it on ONE GPU: the whole
    2048^3 27-point fp64 box grid through AUTO (prepare(), then K = 4 box
    strip launches with its z-chunking at 2048 planes), from the reference
    initial condition.  The oracle cannot sweep 2048^3, so the check is
    size-independent: the initial condition is z-uniform, so after t sweeps
    every plane more than t from both z ends equals the middle plane of a
    (2t + 1)-plane grid and every other plane the plane as far from the same
    end.  That small grid is checked bitwise against the oracle (whole grid,
    ghosts included); the big grid's per-plane sums against the small grid's
    (same plane-sum kernel: bitwise); whole planes near both ends and in the
    middle, ghost rings included, bitwise against the small grid's; the
    z-ghost planes untouched."""
    import torch
    from stencil_amd import _lib
    n, it = 2048, 12
    t = it
    e = engine(gpu, 3, "fp64", "box", 1, "naive", "auto", n, n, n)
    assert e.fuse_steps == 4
    assert e.plan(it) == (3, _lib.KERNEL_TEMPORAL2)
    e.reset()
    e.prepare()  # as bench.py: the schedule choice settled first, grid a unchanged
    fin, _ = e.iterate(it)
    big_sums = e.plane_sums(fin)
    gh = e.with_ghosts(fin)  # (n + 2, n + 2, n + 2) strided view
    zs = [0, 1, t - 1, t, n // 2, n - t - 1, n - t, n - 2, n - 1]
    planes = {z: gh[z + 1].cpu().numpy() for z in zs}
    ghosts = [gh[0].cpu().numpy(), gh[n + 1].cpu().numpy()]
    del e, fin, gh
    torch.cuda.empty_cache()
    nzs = 2 * t + 1
    small = engine(gpu, 3, "fp64", "box", 1, "naive", "auto", n, n, nzs)
    small.reset()
    sfin, _ = small.iterate(it)
    small_sums = small.plane_sums(sfin)
    small_dense = small.to_numpy(sfin)
    del small, sfin
    torch.cuda.empty_cache()
    p = ob.problem(3, "fp64", "box", 1, "naive", n, n, nzs)
    want_small = ob.run(p, it, threads=16)
    assert np.array_equal(small_dense.view(np.uint8), want_small.view(np.uint8))
    z = np.arange(n)
    idx = np.where(z < t, z, np.where(z >= n - t, nzs - (n - z), t))
    assert np.array_equal(big_sums.view(np.uint64), small_sums[idx].view(np.uint64))
    for zz, plane in planes.items():
        assert np.array_equal(plane.view(np.uint8), want_small[idx[zz] + 1].view(np.uint8)), zz
    ghost_plane = want_small[0]  # x-ghost columns 1, everything else 0, never written
    for g in ghosts:
        assert np.array_equal(g.view(np.uint8), ghost_plane.view(np.uint8))
    assert float(want_small[t + 1].max()) > 0.0 and float(want_small[t + 1, 1:-1, 1:-1].min()) == 0.0


@pytest.mark.parametrize("cfg", ["C5_slab_box_fp64", "C4_slab_fp64", "C3_fp32_4096sq"])
def test_full_size_baseline_configs(gpu, cfg):
    """Per-GPU shapes of BASELINE configs 3-5 at full x/y size, bitwise
    against the multithreaded oracle for a few sweeps (the oracle cannot run
    the full iteration counts in test time):
      C5: one GPU's slab of 2048^3 27-point (2048^2 x 256), 3 sweeps
      C4: one GPU's slab of 2048^2 x 4096 7-point, 2048^2 x 64 planes, 4 sweeps
      C3: 4096^2 x 32 fp32 7-point (4096^3 does not fit), 4 sweeps (fused pairs)"""
    import torch
    shapes = {"C5_slab_box_fp64": ("box", "fp64", (2048, 2048, 256), 3),
              "C4_slab_fp64": ("star", "fp64", (2048, 2048, 64), 4),
              "C3_fp32_4096sq": ("star", "fp32", (4096, 4096, 32), 4)}
    shape, dtype, (nx, ny, nz), it = shapes[cfg]
    p = ob.problem(3, dtype, shape, 1, "naive", nx, ny, nz)
    want = ob.interior(p, ob.run(p, it, "random", 2025, threads=16))
    e = engine(gpu, 3, dtype, shape, 1, "naive", "auto", nx, ny, nz)
    e.reset("random", 2025)
    fin, _ = e.iterate(it)
    got = e.interior(fin).cpu().numpy()
    assert np.array_equal(got.view(np.uint8), np.ascontiguousarray(want).view(np.uint8))
    del e
    torch.cuda.empty_cache()


@pytest.mark.parametrize("pack", ["1", "0"])
def test_box_packed_schedule(gpu, monkeypatch, pack):
    """The box's packed longest-first z-chunk schedule (few-tile fp64 grids,
    kernels_boxk.hip + kernels_strip.hip packed_schedule) at a shape where it
    is used, 7 sweeps (a K = 4 launch, a pair and a single), bitwise against the
    oracle -- and with it switched off."""
    monkeypatch.setenv("STENCIL_BOXK_PACK", pack)
    nx, ny, nz = 400, 400, 400  # 112 tiles: 336 packed workgroups (STENCIL_TK_VERBOSE=1 prints the table size)
    p = ob.problem(3, "fp64", "box", 1, "naive", nx, ny, nz)
    want = ob.run(p, 7, "random", 77, threads=16)
    _, got = gpu_run(gpu, 3, "fp64", "box", 1, "naive", "auto", nx, ny, nz, 7, "random", 77)
    assert same_bits(got, want)


@pytest.mark.parametrize("case", ["C2_512cube_fp64", "C3_4096sq_x32_fp32", "C4_2048sq_x512_fp64",
                                  "C5_2048sq_x256_box_fp64", "box_512cube_fp64", "box_2048sq_x64_fp32"])
def test_benched_kernel_at_benched_shape(gpu, case):
    """The kernels that produce the bench numbers, at the shapes they are
    benched on, through AUTO, bitwise against the multithreaded oracle --
    with the plan asserted, so the tested launch IS the benched one:
      C2: 512^3 fp64, 9 sweeps = two K = 4 strip launches with the packed
          longest-first schedule + a single sweep (bench.py's default line);
      C3: 4096^2 x 32 fp32, 10 sweeps = two K = 5 launches (AUTO's K for fp32
          planes >= 1024^2);
      C4: 2048^2 x 512 fp64 (one GPU's slab of config 4), 8 sweeps = two
          K = 4 launches of equal z-chunks (too many tiles to pack);
      C5: 2048^2 x 256 fp64 box (one GPU's slab of config 5), 9 sweeps = two
          K = 4 strip launches (5 x 8 rows) + a single sweep;
      box 512^3 fp64 and 2048^2 x 64 fp32 (K = 4 strip 5 x 8: box planes >= 384^2)."""
    import torch
    from stencil_amd import _lib
    t2 = _lib.KERNEL_TEMPORAL2  # the box's fused family reports TEMPORAL2
    shapes = {"C2_512cube_fp64": ("star", "fp64", (512, 512, 512), 9, 4, (3, _lib.KERNEL_TEMPORALK), True),
              "C3_4096sq_x32_fp32": ("star", "fp32", (4096, 4096, 32), 10, 5, (2, _lib.KERNEL_TEMPORALK), False),
              "C4_2048sq_x512_fp64": ("star", "fp64", (2048, 2048, 512), 8, 4, (2, _lib.KERNEL_TEMPORALK), False),
              "C5_2048sq_x256_box_fp64": ("box", "fp64", (2048, 2048, 256), 9, 4, (3, t2), None),
              "box_512cube_fp64": ("box", "fp64", (512, 512, 512), 9, 4, (3, t2), None),
              "box_2048sq_x64_fp32": ("box", "fp32", (2048, 2048, 64), 8, 4, (2, t2), None)}
    shape, dtype, (nx, ny, nz), it, k, plan, packed = shapes[case]
    e = engine(gpu, 3, dtype, shape, 1, "naive", "auto", nx, ny, nz)
    assert e.fuse_steps == k
    assert e.plan(it) == plan
    if packed is not None:
        geo = e.sweepk_geometry(k)
        assert geo["packed"] == packed, geo
    e.reset("random", 4242)
    fin, _ = e.iterate(it)
    if packed:  # the first launch timed both grids (pick_schedule): at 512^3 packed wins by ~8 %
        assert e.sweepk_geometry(k)["packed"], "measured choice at the C2 shape: equal chunks"
    got = e.interior(fin).cpu().numpy()
    del e, fin
    torch.cuda.empty_cache()
    p = ob.problem(3, dtype, shape, 1, "naive", nx, ny, nz)
    want = ob.interior(p, ob.run(p, it, "random", 4242, threads=16))
    assert np.array_equal(got.view(np.uint8), np.ascontiguousarray(want).view(np.uint8))


# ------------------------------------------- reference-compatible entry points
@pytest.mark.parametrize("fn,order", [("stencil_iterate_dma", "dma"), ("stencil_iterate_dma_static_unroll", "naive"),
                                      ("stencil_iterate_dma_slave_pack", "dma"), ("stencil_iterate_rma", "dma")])
@pytest.mark.parametrize("n,it,r", [(64, 100, 1), (64, 7, 1), (96, 50, 3), (32, 0, 1)])
def test_reference_abi_entry_points(gpu, fn, order, n, it, r):
    """stencil_iterate_*(Arguments*) with host buffers: the final grid must
    land in `output` when iterations is odd, else in `input`
    (stencil.cpp:88-92,134), equal bit for bit to that variant's order."""
    from stencil_amd import _lib
    lib = _lib.load()
    p = ob.problem(2, "fp32", "star", r, order, n, n)
    a = ob.init(p)
    b = a.copy()
    def view(arr):
        return _lib.MatrixView(n + 2 * r, n + 2 * r, r, r, n + 2 * r, arr.ctypes.data_as(ctypes.POINTER(ctypes.c_float)))
    args = _lib.Arguments(n // 8 or 1, it, view(a), view(b))
    getattr(lib, fn)(ctypes.byref(args))
    assert lib.stencil_last_error() == 0, lib.stencil_last_error_message()
    got = b if it % 2 else a
    assert same_bits(got, ob.run(p, it))


def _reference_block_reach(a, it, r, order, ex, ey, rma):
    """What the reference computes when only blocks (ROW, COL) in 0..7 of b^2
    cells exist (boundary_matrix.hpp:190-218): the [0, 8b)^2 sub-grid, whose
    x = 8b / y = 8b neighbours are the untouched host cells -- or, for RMA,
    synthesised Dirichlet faces 1 / 0 (stencil_rma.cpp:149-166).  Cells past
    8b keep their initial value.  Oracle sweeps on the sub-array."""
    n = a.shape[0] - 2 * r
    sub = a[:ey + 2 * r, :ex + 2 * r].copy()
    if rma:
        if ex < n:
            sub[r:ey + r, ex + r] = 1
        if ey < n:
            sub[ey + r, r:ex + r] = 0
    ps = ob.problem(2, "fp32", "star", r, order, ex, ey)
    A, B = sub.copy(), sub.copy()
    for _ in range(it):
        ob.sweep(ps, A, B, 0, ey)
        A, B = B, A
    full = a.copy()
    full[r:ey + r, r:ex + r] = A[r:ey + r, r:ex + r]
    return full


@pytest.mark.parametrize("fn,order,rma", [("stencil_iterate_dma", "dma", False),
                                          ("stencil_iterate_dma_static_unroll", "naive", False),
                                          ("stencil_iterate_dma_slave_pack", "dma", False),
                                          ("stencil_iterate_rma", "dma", True)])
@pytest.mark.parametrize("n,b,it", [(80, 8, 9), (100, 10, 4), (64, 8, 5), (70, 9, 6), (40, 0, 3)])
def test_reference_abi_block_reach(gpu, fn, order, rma, n, b, it):
    """-s n -b b with n > 8b: the reference never computes rows / columns at
    or past 8b; block_size 0 computes nothing."""
    from stencil_amd import _lib
    lib = _lib.load()
    r = 1
    p = ob.problem(2, "fp32", "star", r, order, n, n)
    a = ob.init(p, "random", 3)
    a0 = a.copy()
    bb = a.copy()
    def view(arr):
        return _lib.MatrixView(n + 2 * r, n + 2 * r, r, r, n + 2 * r, arr.ctypes.data_as(ctypes.POINTER(ctypes.c_float)))
    args = _lib.Arguments(b, it, view(a), view(bb))
    getattr(lib, fn)(ctypes.byref(args))
    assert lib.stencil_last_error() == 0, lib.stencil_last_error_message()
    got = bb if it % 2 else a
    reach = min(n, 8 * b)
    want = a0 if reach == 0 else _reference_block_reach(a0, it, r, order, reach, reach, rma)
    assert same_bits(got, want)
    other = a if it % 2 else bb  # the other buffer: the reference leaves it holding some earlier sweep;
    assert same_bits(other[reach + r:], a0[reach + r:])  # its never-computed rows stay initial


# ----------------------------------------------------------------- CLI
def test_cli_check_result_on_gpu(gpu):
    cli = os.path.join(ROOT, "build", "bin", "stencil_main")
    out = subprocess.run([cli, "-s", "64", "-b", "8", "-i", "100", "-m", "DMA", "DMAStaticUnroll", "DMASlavePack",
                          "RMA", "HIP", "-c", "-R", "2"], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    import re
    for m in ("DMA", "DMAStaticUnroll", "DMASlavePack", "RMA", "HIP"):
        assert f"The results of method {m} is correct." in out.stdout
        assert re.search(rf"The average time taken by {m} method is [0-9.e+-]+ms for 100 iterations\.", out.stdout)
    out = subprocess.run([cli, "-s", "24", "-b", "1", "-i", "5", "-m", "HIP", "HIPDirect", "HIPZMarch", "-c",
                          "--points", "7", "--dtype", "fp64", "--init", "random"], capture_output=True, text=True,
                         timeout=300)
    assert out.returncode == 0, out.stderr + out.stdout
    assert out.stdout.count("is correct.") == 3
    out = subprocess.run([cli, "-s", "300", "-b", "1", "-i", "37", "-m", "HIPPersistent", "HIPTemporal2", "-c"],
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr + out.stdout
    assert out.stdout.count("is correct.") == 2


def test_cli_multi_gpu_slabs(gpu):
    """The drop-in runs a z-slab job from the C++ host: HIPMultiGPU over one
    GPU through RCCL, and 3 / 4 slabs sharing the GPU with device-copy halos
    (RCCL refuses two ranks on one GPU) -- each checked against the CPU naive
    sweep with -c, the reference's stdout lines intact."""
    import re
    cli = os.path.join(ROOT, "build", "bin", "stencil_main")
    base = [cli, "-s", "40", "-b", "1", "-i", "13", "--dims", "3", "--nz", "37", "--init", "random", "-c"]
    runs = [base + ["-m", "HIPMultiGPU", "--dtype", "fp64"],
            base + ["-m", "HIPMultiGPU", "HIP", "--gpus", "3", "--share-device", "--exchange", "copy"],
            base + ["-m", "HIP", "--gpus", "4", "--share-device", "--exchange", "copy", "--points", "27",
                    "--dtype", "fp64"],
            # 700^2 fp64 box planes: K = 4 launches, and over RCCL the face-signalled K = 4 rounds
            [cli, "-s", "700", "-b", "1", "-i", "13", "--dims", "3", "--nz", "12", "--init", "random", "-c",
             "-m", "HIPMultiGPU", "HIP", "--points", "27", "--dtype", "fp64"]]
    for args in runs:
        out = subprocess.run(args, capture_output=True, text=True, timeout=300)
        assert out.returncode == 0, out.stderr + out.stdout
        for m in set(args[args.index("-m") + 1:][:2]) & {"HIPMultiGPU", "HIP"}:
            assert f"The results of method {m} is correct." in out.stdout
            assert re.search(rf"The average time taken by {m} method is [0-9.e+-]+ms for 13 iterations\.",
                             out.stdout)


def test_cli_block_reach(gpu):
    """-s 80 -b 8: the reference methods compute only [0, 64)^2, so their
    check_result fails exactly like the reference's (main.cpp:17-22: the
    "incorrect" line, no timing lines); the GPU-native HIP method computes
    the whole grid."""
    cli = os.path.join(ROOT, "build", "bin", "stencil_main")
    out = subprocess.run([cli, "-s", "80", "-b", "8", "-i", "20", "-m", "DMA", "RMA", "HIP", "-c"],
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 3, out.stderr  # extension: a failed check is a non-zero exit (the reference exits 0)
    for m in ("DMA", "RMA"):
        assert f"The results of method {m} is incorrect." in out.stdout
        assert f"The average time taken by {m} method" not in out.stdout
    assert "The results of method HIP is correct." in out.stdout
    assert out.stdout.count("invalid result at (") == 2


def test_cli_bmp_dump(gpu, tmp_path):
    cli = os.path.join(ROOT, "build", "bin", "stencil_main")
    out = tmp_path / "grid.bmp"
    p = subprocess.run([cli, "-s", "50", "-b", "8", "-i", "200", "-m", "HIP", "--bmp", str(out)],
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr
    data = out.read_bytes()
    assert data[:2] == b"BM" and len(data) == 54 + 50 * (150 + 2)
    # every pixel is the heat-map colour of the oracle's final grid
    p = ob.problem(2, "fp32", "star", 1, "naive", 50, 50)
    grid = ob.interior(p, ob.run(p, 200)).astype(np.float64)

    def heat(v):
        v = min(max(v, 0.0), 1.0)
        if v < 0.25:
            return (255, int(4 * v * 255), 0)
        if v < 0.5:
            return (int((1 + 4 * (0.25 - v)) * 255), 255, 0)
        if v < 0.75:
            return (0, 255, int(4 * (v - 0.5) * 255))
        return (0, int((1 + 4 * (0.75 - v)) * 255), 255)

    for y in range(50):
        row = data[54 + y * 152: 54 + y * 152 + 150]
        want = b"".join(bytes(heat(float(grid[y, x]))) for x in range(50))
        assert row == want, y


@pytest.mark.parametrize("shape", ["star", "box"])
@pytest.mark.parametrize("pw", ["1", "3", "4"])
@pytest.mark.parametrize("zchunk", ["0", "7"])
def test_xcd_patch_tile_orders(gpu, monkeypatch, shape, pw, zchunk):
    """The XCD-patch work orders (debug knobs STENCIL_TK_XCD / STENCIL_BOXK_XCD:
    XCD b % 8 walks its own run of (chunk, tile) units in column strips of pw
    tiles; the grid is rounded up to a multiple of 8 and surplus workgroups
    leave at once) cover every (chunk, tile) unit exactly once: bitwise the
    oracle on ragged grids of many tiles, with forced and automatic z-chunks."""
    monkeypatch.setenv("STENCIL_TK_XCD" if shape == "star" else "STENCIL_BOXK_XCD", pw)
    monkeypatch.setenv("STENCIL_TK_PACK", "0")
    monkeypatch.setenv("STENCIL_TK_ZCHUNK" if shape == "star" else "STENCIL_BOXK_ZCHUNK", zchunk)
    nx, ny, nz = 333, 250, 23
    p = ob.problem(3, "fp64", shape, 1, "naive", nx, ny, nz)
    e = engine(gpu, 3, "fp64", shape, 1, "naive", "auto", nx, ny, nz)
    assert e.lib.stencil_debug_knobs() == 1
    k = e.fuse_steps
    e.reset("random", 61)
    e.sweepk(e.a, e.b, 0, nz, k)
    assert same_bits(e.to_numpy(e.b), ob.run(p, k, "random", 61, threads=16))


@pytest.mark.parametrize("dtype,nx", [("fp64", 4096), ("fp32", 8192), ("fp64", 8192), ("fp64", 8160), ("fp32", 8160),
                                     ("fp64", 4000)])
def test_padded_row_pitch_matches_oracle(gpu, dtype, nx):
    """Rows whose pitch sits within [-512, +256] B of a multiple of 32 KiB get
    padded (stencil_layout_init's pitch rule); the K-step
    launches on such a layout stay bitwise the oracle."""
    e = engine(gpu, 3, dtype, "star", 1, "naive", "auto", nx, 20, 14)
    es = 8 if dtype == "fp64" else 4
    align = 128 // es
    raw = (align + nx + 1 + align - 1) // align * align  # the 128-B-aligned minimum row (r = 1)
    assert e.layout.row > raw, e.layout.row  # the rule applied
    e.reset("random", 21)
    fin, _ = e.iterate(9)
    p = ob.problem(3, dtype, "star", 1, "naive", nx, 20, 14)
    assert same_bits(e.to_numpy(fin), ob.run(p, 9, "random", 21))
