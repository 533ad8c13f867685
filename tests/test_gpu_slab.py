"""Slab decomposition with the HIP kernels, N logical slabs on one GPU.

RCCL cannot put two ranks on one device, so the exchange in the first tests
is a plain device copy between the slabs' grids, written out here.  What
they pin is the GPU side of multi-GPU: deep halos, the HALO_LO/HI flags of
the fused kernels, boundary/interior plane ranges, the face-signalled
launches -- bitwise equal to one undivided grid.  The round logic itself is
the C-ABI slab job's (csrc/slab_core.hpp): its periodic one-slab rings here,
tests/test_gpu_slab_job.py on the GPU, tests/test_slab_core_cpu.py on the
CPU at world 2 / 3."""
import numpy as np
import pytest
import torch

from stencil_amd import _lib
from bench import partition
from stencil_amd.engine import JacobiEngine, SlabJob, StencilSpec

pytestmark = pytest.mark.gpu


def run_slabs(gpu, nx, ny, nz, world, iterations, fused, split, shape="star", split2=False, k=2):
    """`fused`: rounds of k fused sweeps per k-plane exchange (sweepk)."""
    spec = StencilSpec(dims=3, dtype="fp64", halo=max(2, k), shape=shape)
    h = spec.halo
    engines, firsts = [], []
    for r in range(world):
        first, count = partition(nz, world, r)
        flags = (_lib.HALO_LO if r > 0 else 0) | (_lib.HALO_HI if r < world - 1 else 0)
        e = JacobiEngine(spec, nx, ny, count, device=gpu, flags=flags)
        e.reset("random", 17 + first * nx * ny)
        engines.append(e)
        firsts.append((first, count))
    cur = [e.a for e in engines]
    nxt = [e.b for e in engines]

    def exchange(grids):
        for r in range(world - 1):
            lo, hi = engines[r], engines[r + 1]
            n_lo = firsts[r][1]
            hi.plane_view(grids[r + 1], -h, h).copy_(lo.plane_view(grids[r], n_lo - h, h))
            lo.plane_view(grids[r], n_lo, h).copy_(hi.plane_view(grids[r + 1], 0, h))

    exchange(cur)
    done = 0
    if split2:  # two single sweeps per 2-plane exchange, halo planes advanced by the first
        while done + 2 <= iterations:
            for r, e in enumerate(engines):
                n = firsts[r][1]
                lo = -1 if r > 0 else 0
                hi = n + 1 if r < world - 1 else n
                e.sweep(cur[r], nxt[r], lo, hi)
                e.sweep(nxt[r], cur[r], 0, n)
            exchange(cur)
            done += 2
    while done < iterations:
        steps = min(k, iterations - done) if fused else 1
        for r, e in enumerate(engines):
            n = firsts[r][1]
            if split and n > 2 * h:
                e.sweepk(cur[r], nxt[r], 0, h, steps)
                e.sweepk(cur[r], nxt[r], n - h, n, steps)
                e.sweepk(cur[r], nxt[r], h, n - h, steps)
            else:
                e.sweepk(cur[r], nxt[r], 0, n, steps)
        exchange(nxt)
        cur, nxt = nxt, cur
        done += steps
    torch.cuda.synchronize()
    return torch.cat([e.interior(g) for e, g in zip(engines, cur)], dim=0)


@pytest.mark.parametrize("shape", ["star", "box"])
@pytest.mark.parametrize("world", [2, 3, 4])
@pytest.mark.parametrize("fused", [False, True])
@pytest.mark.parametrize("split", [False, True])
def test_slabs_bitwise_equal_single_grid(gpu, world, fused, split, shape):
    nx, ny, nz, it = 70, 45, 29, 7
    ref = JacobiEngine(StencilSpec(dims=3, dtype="fp64", shape=shape, kernel="direct"), nx, ny, nz, device=gpu)
    ref.reset("random", 17)
    fin, _ = ref.iterate(it)
    want = ref.interior(fin)
    got = run_slabs(gpu, nx, ny, nz, world, it, fused, split, shape)
    assert torch.equal(got, want)


@pytest.mark.parametrize("shape,k", [("star", 3), ("star", 4), ("box", 2), ("box", 3)])
@pytest.mark.parametrize("world", [2, 3, 4])
@pytest.mark.parametrize("split", [False, True])
@pytest.mark.parametrize("cfg", ["default", "312", "strip1"])
def test_slabs_k_step_rounds(gpu, monkeypatch, world, shape, k, split, cfg):
    """k fused sweeps per k-plane halo exchange (TEMPORALK -- strip layout by
    default, the interleaved-row layout with cfg 312, the strip default shape
    for the other K -- and the K-step box kernel with HALO_LO/HI): halo planes
    advanced to t+k-1 .. t+1 inside the launch."""
    if cfg == "312":
        monkeypatch.setenv("STENCIL_TK_STRIP", "0")
        monkeypatch.setenv("STENCIL_TK_CFG", cfg)
    elif cfg == "strip1":
        monkeypatch.setenv("STENCIL_TK_STRIP", "404" if k == 4 else "10808")
    monkeypatch.setenv("STENCIL_TK_ZCHUNK", "5")
    monkeypatch.setenv("STENCIL_BOXK_ZCHUNK", "5")
    nx, ny, nz, it = 70, 45, 29, 11
    ref = JacobiEngine(StencilSpec(dims=3, dtype="fp64", kernel="direct", shape=shape), nx, ny, nz, device=gpu)
    ref.reset("random", 17)
    fin, _ = ref.iterate(it)
    got = run_slabs(gpu, nx, ny, nz, world, it, True, split, shape=shape, k=k)
    assert torch.equal(got, ref.interior(fin))


def test_k_step_needs_deep_halo(gpu):
    e = JacobiEngine(StencilSpec(dims=3, dtype="fp64", halo=2), 16, 16, 8, device=gpu, flags=_lib.HALO_HI)
    e.reset()
    with pytest.raises(_lib.StencilError):
        e.sweepk(e.a, e.b, 0, 8, 3)


@pytest.mark.parametrize("shape", ["star", "box"])
@pytest.mark.parametrize("world", [2, 3])
def test_split2_rounds_bitwise(gpu, world, shape):
    nx, ny, nz, it = 70, 45, 29, 7
    ref = JacobiEngine(StencilSpec(dims=3, dtype="fp64", shape=shape, kernel="direct"), nx, ny, nz, device=gpu)
    ref.reset("random", 17)
    fin, _ = ref.iterate(it)
    got = run_slabs(gpu, nx, ny, nz, world, it, False, False, shape, split2=True)
    assert torch.equal(got, ref.interior(fin))


def test_sweep_range_into_halo_needs_flag(gpu):
    e = JacobiEngine(StencilSpec(dims=3, dtype="fp64", halo=2), 16, 16, 8, device=gpu)
    e.reset()
    with pytest.raises(_lib.StencilError):
        e.sweep(e.a, e.b, -1, 8)


def test_fused_needs_deep_halo(gpu):
    e = JacobiEngine(StencilSpec(dims=3, dtype="fp64"), 16, 16, 8, device=gpu, flags=_lib.HALO_LO)
    e.reset()
    with pytest.raises(_lib.StencilError):
        e.sweep2(e.a, e.b, 0, 8)


@pytest.mark.parametrize("dtype", ["fp64", "fp32"])
@pytest.mark.parametrize("steps", [3, 4, 5])
@pytest.mark.parametrize("zchunk", ["0", "5", "9", "40"])
@pytest.mark.parametrize("flags", [0, 3])
def test_sweepk_signal_equals_sweepk(gpu, monkeypatch, dtype, steps, zchunk, flags):
    """stencil_sweepk_signal (last z-chunk marching down, face counters) is
    bitwise stencil_sweepk, and each face counter gets one add per tile."""
    monkeypatch.setenv("STENCIL_TK_ZCHUNK", zchunk)
    nx, ny, nz = 77, 51, 31
    spec = StencilSpec(dims=3, dtype=dtype, halo=5)
    e = JacobiEngine(spec, nx, ny, nz, device=gpu, flags=flags)
    e.reset("random", 9)
    ref = torch.empty_like(e.b)
    ref.copy_(e.b)
    e.sweepk(e.a, ref, 0, nz, steps)
    sig = torch.zeros(4, dtype=torch.int32, device=e.a.device)
    nsig = e.sweepk_signal(e.a, e.b, 0, nz, steps, sig)
    e.wait_counters(sig, nsig, nsig)
    torch.cuda.synchronize()
    # bitwise over the whole buffer (row/plane padding is never written and may hold NaN bits)
    ib = torch.int64 if dtype == "fp64" else torch.int32
    assert torch.equal(e.b.view(ib), ref.view(ib))
    assert sig[0].item() == nsig and sig[1].item() == nsig and sig[2].item() == 0 and nsig > 0


def test_wait_counters_timeout_flag_is_sticky(gpu):
    """A wait whose timeout flag is already set (an earlier wait gave up on a
    lost peer) returns at once instead of spinning another 10 s; a wait whose
    targets are met returns and leaves the flag as it was."""
    import time
    e = JacobiEngine(StencilSpec(dims=3, dtype="fp64"), 16, 16, 8, device=gpu)
    sig = torch.zeros(4, dtype=torch.int32, device=e.a.device)
    sig[2] = 1
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e.wait_counters(sig, 5, 5)  # never met: counters stay 0
    torch.cuda.synchronize()
    assert time.perf_counter() - t0 < 2.0
    assert sig.tolist() == [0, 0, 1, 0]
    sig[2] = 0
    sig[0] = 3
    sig[1] = 4
    e.wait_counters(sig, 3, 4)
    torch.cuda.synchronize()
    assert sig.tolist() == [3, 4, 0, 0]


@pytest.mark.parametrize("flags", [0, 3])
@pytest.mark.parametrize("pack_sig", ["1", "0"])
def test_sweepk_signal_packed_schedule(gpu, monkeypatch, capfd, flags, pack_sig):
    """Face-signalled launches on a grid of few tiles take the packed schedule
    with the faces outward (packed_schedule faces_out: each tile's first full
    chunk at plane 0 marching up, its last one ending at the top marching
    down, the short remainder between): bitwise stencil_sweepk, one counter
    add per tile and face, at the benched 512^3 fp64 shape (110 tiles x 3
    chunks); STENCIL_TK_PACK_SIG=0 (debug) keeps the equal one-round chunks."""
    monkeypatch.setenv("STENCIL_TK_VERBOSE", "1")
    monkeypatch.setenv("STENCIL_TK_PACK_SIG", pack_sig)
    nx = ny = nz = 512
    e = JacobiEngine(StencilSpec(dims=3, dtype="fp64", halo=4), nx, ny, nz, device=gpu, flags=flags)
    e.reset("random", 13)
    ref = torch.empty_like(e.b)
    ref.copy_(e.b)
    e.sweepk(e.a, ref, 0, nz, 4)
    torch.cuda.synchronize()
    capfd.readouterr()
    sig = torch.zeros(4, dtype=torch.int32, device=e.a.device)
    for launch in range(3):  # the counters run on over launches
        nsig = e.sweepk_signal(e.a, e.b, 0, nz, 4, sig)
        e.wait_counters(sig, nsig * (launch + 1), nsig * (launch + 1))
        torch.cuda.synchronize()
        assert torch.equal(e.b.view(torch.int64), ref.view(torch.int64)), launch
    err = capfd.readouterr().err
    assert sig[0].item() == 3 * nsig and sig[1].item() == 3 * nsig and sig[2].item() == 0 and nsig == 110
    # the launch line (STENCIL_TK_VERBOSE) gives the grid: 110 tiles x {230, 230, 52} planes when packed
    assert ("tiles 10x11, zchunk" in err) and (("330 workgroups" in err) == (pack_sig == "1")), err


@pytest.mark.parametrize("dtype", ["fp64", "fp32"])
@pytest.mark.parametrize("steps", [2, 3, 4])
@pytest.mark.parametrize("zchunk", ["0", "5", "9", "40"])
@pytest.mark.parametrize("flags", [0, 3])
@pytest.mark.parametrize("cfg", ["0", "10308", "20308", "10208", "10116", "20116", "910408", "910312", "920408",
                                 "910212", "910216"])
def test_box_sweepk_signal_equals_sweepk(gpu, monkeypatch, dtype, steps, zchunk, flags, cfg):
    """The 27-point box's face-signalled launch (kernels_boxk.hip SIG: the last
    z-chunk marches down, carrying C and two plane sums instead of the
    pre-added A) is bitwise stencil_sweepk, one counter add per tile and face."""
    monkeypatch.setenv("STENCIL_BOXK_ZCHUNK", zchunk)
    monkeypatch.setenv("STENCIL_BOXK_SIG_CFG", cfg)
    nx, ny, nz = 77, 51, 31
    spec = StencilSpec(dims=3, dtype=dtype, shape="box", halo=4)
    e = JacobiEngine(spec, nx, ny, nz, device=gpu, flags=flags)
    e.reset("random", 9)
    ref = torch.empty_like(e.b)
    ref.copy_(e.b)
    e.sweepk(e.a, ref, 0, nz, steps)
    sig = torch.zeros(4, dtype=torch.int32, device=e.a.device)
    nsig = e.sweepk_signal(e.a, e.b, 0, nz, steps, sig)
    e.wait_counters(sig, nsig, nsig)
    torch.cuda.synchronize()
    ib = torch.int64 if dtype == "fp64" else torch.int32
    assert torch.equal(e.b.view(ib), ref.view(ib))
    assert sig[0].item() == nsig and sig[1].item() == nsig and sig[2].item() == 0 and nsig > 0


@pytest.mark.parametrize("dtype,steps", [("fp64", 4), ("fp32", 4), ("fp64", 3), ("fp32", 5)])
def test_face_signal_counts_completed_faces(gpu, dtype, steps):
    """The face signal (HIP signal memory, waited on by the command processor)
    grows by exactly 2 per launch -- one per face, from the workgroup that
    completes that face's count -- and a stream gated on it sees the faces."""
    from stencil_amd.engine import FaceSignal
    nx, ny, nz = 77, 51, 31
    e = JacobiEngine(StencilSpec(dims=3, dtype=dtype, halo=5), nx, ny, nz, device=gpu)
    e.reset("random", 9)
    ref = torch.empty_like(e.b)
    ref.copy_(e.b)
    e.sweepk(e.a, ref, 0, nz, steps)
    fs = FaceSignal()
    fs.reset()
    sig = torch.zeros(4, dtype=torch.int32, device=e.a.device)
    side = torch.cuda.Stream()
    lo = torch.empty(steps * e.unit, dtype=e.b.dtype, device=e.b.device)
    hi = torch.empty_like(lo)
    for launch in range(1, 4):
        side.wait_stream(torch.cuda.current_stream())  # the reset / the previous launch is queued
        nsig = e.sweepk_signal(e.a, e.b, 0, nz, steps, sig, face_signal=fs)
        with torch.cuda.stream(side):
            fs.wait(2 * launch, stream=side)
            lo.copy_(e.plane_view(e.b, 0, steps))
            hi.copy_(e.plane_view(e.b, nz - steps, steps))
        torch.cuda.synchronize()
        assert fs.value() == 2 * launch
        assert sig[0].item() == launch * nsig and sig[1].item() == launch * nsig
    ib = torch.int64 if dtype == "fp64" else torch.int32
    assert torch.equal(e.b.view(ib), ref.view(ib))
    assert torch.equal(lo.view(ib), e.plane_view(ref, 0, steps).view(ib))
    assert torch.equal(hi.view(ib), e.plane_view(ref, nz - steps, steps).view(ib))
    fs.close()


def _periodic_job(gpu, monkeypatch, nx, ny, nz, it, signalled, dtype="fp64", shape="star", exchange="copy"):
    """A one-slab periodic C-ABI job (its halos are its own faces: an
    interior rank's rounds), face-signalled or boundary + interior rounds
    (STENCIL_SLAB_SIGNAL), halos by device copies or RCCL to itself."""
    monkeypatch.setenv("STENCIL_SLAB_SIGNAL", "1" if signalled else "0")
    monkeypatch.setenv("STENCIL_SLAB_STAGED", "0")  # many-round planes: signals, not AUTO's staged rounds
    spec = StencilSpec(dims=3, dtype=dtype, shape=shape)
    job = SlabJob(spec, nx, ny, nz, [gpu], exchange=exchange, periodic=True)
    try:
        job.fill_initial("random", 5)
        job.run(it)
        dense = job.download()
        k = job.info(0)["sweeps_per_round"]
        job.kernel_timing(True)
        job.run(k)
        assert job.kernel_time()["signalled"] == signalled
    finally:
        job.close()
    return dense


@pytest.mark.parametrize("shape3,it", [((70, 45, 33), 13), ((130, 64, 20), 9), ((64, 7, 9), 8)])
def test_signalled_rounds_match_boundary_launches(gpu, monkeypatch, shape3, it):
    """Single-launch face-signalled slab rounds (the exchange gated by the
    wait kernel on the face counters) give bit for bit the two-boundary-launch
    rounds."""
    nx, ny, nz = shape3
    want = _periodic_job(gpu, monkeypatch, nx, ny, nz, it, False)
    got = _periodic_job(gpu, monkeypatch, nx, ny, nz, it, True)
    assert np.array_equal(got.view(np.uint8), want.view(np.uint8))


@pytest.mark.parametrize("dtype", ["fp64", "fp32"])
@pytest.mark.parametrize("steps", ["3", "4", "5"])
@pytest.mark.parametrize("extra,it", [(0, 8), (1, 17), (3, 9), (4, 11), (30, 20)])
def test_signalled_rounds_every_k(gpu, monkeypatch, dtype, steps, extra, it):
    """Face-signalled rounds for K = 3, 4, 5 in fp32 and fp64, on slabs from
    the minimum 2K planes (the launch's chunks shrink to >= K planes each) to
    several chunks, with a remainder of iterations after the K-rounds --
    bitwise the boundary + interior rounds."""
    monkeypatch.setenv("STENCIL_TK_STEPS", steps)
    nz = 2 * int(steps) + extra  # 2K planes: the smallest signalled slab
    nx, ny = 67, 29
    want = _periodic_job(gpu, monkeypatch, nx, ny, nz, it, False, dtype=dtype)
    got = _periodic_job(gpu, monkeypatch, nx, ny, nz, it, True, dtype=dtype)
    assert np.array_equal(got.view(np.uint8), want.view(np.uint8)), (nz, it)


@pytest.mark.parametrize("dtype", ["fp64", "fp32"])
def test_signalled_rounds_then_remainder_large_plane(gpu, monkeypatch, dtype):
    """The round-1 stream race, made deterministic: a minimum slab (nz = 2K)
    with a 2048^2 plane, so the last face-signalled launch runs for
    milliseconds, then a remainder round that must follow the round streams
    -- it reads the grid the last signalled launch writes and the halos the
    exchange receives.  Bitwise the boundary + interior rounds."""
    nx = ny = 2048
    fuse = JacobiEngine(StencilSpec(dims=3, dtype=dtype), nx, ny, 8, device=gpu, allocate=False).fuse_steps
    nz, it = 2 * fuse, 2 * fuse + 2  # two signalled rounds + a remainder pair
    want = _periodic_job(gpu, monkeypatch, nx, ny, nz, it, False, dtype=dtype)
    got = _periodic_job(gpu, monkeypatch, nx, ny, nz, it, True, dtype=dtype)
    assert np.array_equal(got.view(np.uint8), want.view(np.uint8))


@pytest.mark.parametrize("dtype", ["fp64", "fp32"])
@pytest.mark.parametrize("shape3,it", [((70, 45, 33), 13), ((130, 64, 20), 9), ((64, 7, 8), 8), ((64, 7, 9), 10)])
def test_box_signalled_rounds_match_boundary_launches(gpu, monkeypatch, dtype, shape3, it):
    """27-point box slab rounds as one face-signalled launch give bit for bit
    the boundary + interior rounds, with remainders after the K-rounds and the
    minimum slab (nz = 2K)."""
    nx, ny, nz = shape3
    want = _periodic_job(gpu, monkeypatch, nx, ny, nz, it, False, dtype=dtype, shape="box")
    got = _periodic_job(gpu, monkeypatch, nx, ny, nz, it, True, dtype=dtype, shape="box")
    assert np.array_equal(got.view(np.uint8), want.view(np.uint8))


@pytest.mark.parametrize("shape", ["star", "box"])
def test_signalled_rounds_over_rccl(gpu, monkeypatch, shape):
    """The same through RCCL send/recv to self (a one-device communicator)."""
    nx, ny, nz, it = 70, 45, 33, 13
    want = _periodic_job(gpu, monkeypatch, nx, ny, nz, it, False, shape=shape)
    got = _periodic_job(gpu, monkeypatch, nx, ny, nz, it, True, shape=shape, exchange="rccl")
    assert np.array_equal(got.view(np.uint8), want.view(np.uint8))


@pytest.mark.parametrize("rolling", [False, True])
def test_slabs_on_a_padded_row_pitch(gpu, rolling):
    """4096-wide fp64 planes take a padded row pitch (stencil_layout_init):
    whole-plane halo copies between slabs and rolling passes on that layout,
    bitwise one grid."""
    spec = StencilSpec(dims=3, dtype="fp64", shape="star")
    nx, ny, nz, it = 4096, 12, 34, 9
    ref = JacobiEngine(StencilSpec(dims=3, dtype="fp64", shape="star", kernel="direct"), nx, ny, nz, device=gpu)
    ref.reset("random", 5)
    fin, _ = ref.iterate(it)
    want = ref.to_numpy(fin)
    job = SlabJob(spec, nx, ny, nz, [gpu] * 2, exchange="copy", rolling=rolling, margin=12 if rolling else 0)
    try:
        job.fill_initial("random", 5)
        job.run(it)
        got = job.download()
    finally:
        job.close()
    assert np.array_equal(got.view(np.uint8), want.view(np.uint8))


def _rolling_copy_job(gpu, dtype, shape, nslabs, margin_extra=1):
    spec = StencilSpec(dims=3, dtype=dtype, shape=shape)
    nx, ny, nz, it = 70, 45, 23 * nslabs + 1, 11
    ref = JacobiEngine(StencilSpec(dims=3, dtype=dtype, shape=shape, kernel="direct"), nx, ny, nz, device=gpu)
    ref.reset("random", 3)
    fin, _ = ref.iterate(it)
    want = ref.to_numpy(fin)
    k = JacobiEngine(spec, nx, ny, nz, device=gpu, allocate=False).fuse_steps
    job = SlabJob(spec, nx, ny, nz, [gpu] * nslabs, exchange="copy", rolling=True, margin=k + margin_extra)
    try:
        job.fill_initial("random", 3)
        job.run(it)
        got = job.download()
    finally:
        job.close()
    return got, want


@pytest.mark.parametrize("dtype,shape", [("fp64", "star"), ("fp32", "box")])
@pytest.mark.parametrize("nslabs", [2, 3])
def test_rolling_slabs_slow_face_pulls(gpu, monkeypatch, dtype, shape, nslabs):
    """A rolling slab's next pass writes its new grid over the planes its
    neighbours pull faces from, so the copy exchange holds every slab until
    its neighbours' pulls are done (slab_core.hpp exchange).  A 3 ms spin
    before slab 0's pulls (STENCIL_SLAB_COPY_DELAY_US, debug library; its
    neighbour runs on) makes a missing dependency show every time: round 4's
    intermittent mismatch of
    test_rolling_slabs_equal_one_grid[3-fp32-box] was this race."""
    monkeypatch.setenv("STENCIL_SLAB_COPY_DELAY_US", "3000")
    got, want = _rolling_copy_job(gpu, dtype, shape, nslabs)
    assert np.array_equal(got.view(np.uint8), want.view(np.uint8))


def test_rolling_slabs_slow_face_pulls_need_the_wait(gpu, monkeypatch):
    """The test above has teeth: with the wait dropped (debug knob) the slow
    pulls read planes the neighbour's next pass has already overwritten."""
    monkeypatch.setenv("STENCIL_SLAB_COPY_DELAY_US", "3000")
    monkeypatch.setenv("STENCIL_SLAB_NO_PULL_WAIT", "1")
    got, want = _rolling_copy_job(gpu, "fp64", "star", 3)
    assert not np.array_equal(got.view(np.uint8), want.view(np.uint8))


@pytest.mark.parametrize("dtype,shape", [("fp64", "star"), ("fp32", "box")])
@pytest.mark.parametrize("nslabs", [1, 2, 3])
def test_rolling_slabs_equal_one_grid(gpu, dtype, shape, nslabs):
    """ROLLING slab jobs (one grid per slab + a margin, STENCIL_SLAB_ROLLING)
    on slabs sharing the GPU, from one-plane launches to one launch per pass:
    bitwise one grid, and bitwise the two-grid slab job."""
    spec = StencilSpec(dims=3, dtype=dtype, shape=shape)
    nx, ny, nz = 70, 45, 23 * nslabs + 1
    it = 11
    ref = JacobiEngine(StencilSpec(dims=3, dtype=dtype, shape=shape, kernel="direct"), nx, ny, nz, device=gpu)
    ref.reset("random", 3)
    fin, _ = ref.iterate(it)
    want = ref.to_numpy(fin)
    k = JacobiEngine(spec, nx, ny, nz, device=gpu, allocate=False).fuse_steps
    for margin in (k + 1, k + 4, 64):
        job = SlabJob(spec, nx, ny, nz, [gpu] * nslabs, exchange="copy", rolling=True, margin=margin)
        try:
            assert job.rolling_info()["margin"] == margin
            job.fill_initial("random", 3)
            job.run(k)
            job.run(it - k)
            got = job.download()
        finally:
            job.close()
        assert np.array_equal(got.view(np.uint8), want.view(np.uint8)), margin


@pytest.mark.parametrize("shape", ["star", "box"])
def test_cpwait_one_chunk_slab_counts_both_faces(gpu, monkeypatch, shape):
    """in a slab of exactly K planes on one tile, one
    workgroup stores both faces at the same plane step; its face-signal add
    must count 2 (it added 1, and the command-processor wait of
    STENCIL_SLAB_CPWAIT=1 then never returned).  A 20 s job deadline turns a
    regression into a failure instead of a hang."""
    monkeypatch.setenv("STENCIL_SLAB_TIMEOUT_MS", "20000")
    nx, ny = 40, 24  # one x-y tile
    k = JacobiEngine(StencilSpec(dims=3, dtype="fp64", shape=shape), nx, ny, 8, device=gpu, allocate=False).fuse_steps
    it = 3 * k + 1
    want = _periodic_job(gpu, monkeypatch, nx, ny, k, it, False, shape=shape)
    monkeypatch.setenv("STENCIL_SLAB_CPWAIT", "1")
    got = _periodic_job(gpu, monkeypatch, nx, ny, k, it, True, shape=shape)
    assert np.array_equal(got.view(np.uint8), want.view(np.uint8))




@pytest.mark.parametrize("shape", ["star", "box"])
@pytest.mark.parametrize("dtype", ["fp64", "fp32"])
@pytest.mark.parametrize("xcu", ["1", "0"])
def test_many_round_signalled_launch_face_chunks_first(gpu, monkeypatch, shape, dtype, xcu):
    """A face-signalled launch of a plane with more tiles than one round of
    workgroups (2048 x 1024: ~800 tiles) splits every tile into at least 4
    z-chunks and dispatches the two face chunks first (slab rounds then
    confine the exchange to one CU per XCD, STENCIL_SLAB_XCU): bitwise the
    boundary + interior rounds."""
    monkeypatch.setenv("STENCIL_SLAB_XCU", xcu)
    monkeypatch.setenv("STENCIL_SLAB_STAGED", "0")  # face signals, not the staged rounds AUTO runs here
    nx, ny, nz, it = 2048, 1024, 40, 9
    want = _periodic_job(gpu, monkeypatch, nx, ny, nz, it, False, dtype=dtype, shape=shape)
    got = _periodic_job(gpu, monkeypatch, nx, ny, nz, it, True, dtype=dtype, shape=shape, exchange="rccl")
    assert np.array_equal(got.view(np.uint8), want.view(np.uint8))


@pytest.mark.parametrize("shape", ["star", "box"])
@pytest.mark.parametrize("dtype", ["fp64", "fp32"])
@pytest.mark.parametrize("exchange", ["rccl", "copy"])
def test_staged_rounds_match_boundary_launches(gpu, monkeypatch, shape, dtype, exchange):
    """STAGED rounds, AUTO's form for slabs whose launch takes several rounds
    of workgroups (2048 x 1024 planes): the face quarters on every CU, then
    the middle on the CUs the confined exchange leaves; remainders after the
    full rounds -- bitwise the boundary + interior rounds.  21 sweeps: the
    two tuning rounds, then at least two rounds with the TUNED face span
    (11 sweeps never ran one)."""
    nx, ny, nz, it = 2048, 1024, 44, 21
    want = _periodic_job(gpu, monkeypatch, nx, ny, nz, it, False, dtype=dtype, shape=shape)
    monkeypatch.delenv("STENCIL_SLAB_SIGNAL", raising=False)
    monkeypatch.delenv("STENCIL_SLAB_STAGED", raising=False)
    spec = StencilSpec(dims=3, dtype=dtype, shape=shape)
    job = SlabJob(spec, nx, ny, nz, [gpu], exchange=exchange, periodic=True)
    try:
        assert job.round_form() == 4
        job.fill_initial("random", 5)
        job.run(it)
        got = job.download()
    finally:
        job.close()
    assert np.array_equal(got.view(np.uint8), want.view(np.uint8))


def test_face_wait_past_the_deadline_fails_the_job_in_time(gpu, monkeypatch):
    """Bounded-time failure on the HIP path: the first
    face-signalled round waits for more face adds than its launch makes
    (STENCIL_SLAB_SIG_SKEW, debug library), as if a face never came.  With a
    1.5 s job deadline, run() returns STENCIL_ETIMEOUT after about that long --
    the host released the polling wait through its host-coherent flag, well
    before the kernel's own 10 s give-up -- later calls fail at once, and
    destroy returns."""
    import time
    from stencil_amd import _lib
    monkeypatch.setenv("STENCIL_SLAB_SIGNAL", "1")
    monkeypatch.setenv("STENCIL_SLAB_SIG_SKEW", "1000")
    spec = StencilSpec(dims=3, dtype="fp64", shape="star")
    job = SlabJob(spec, 130, 64, 20, [gpu], exchange="rccl", periodic=True)
    try:
        assert job.round_form() == 1
        job.set_timeout(1500)
        job.fill_initial("random", 5)
        t0 = time.monotonic()
        with pytest.raises(_lib.StencilError) as ei:
            job.run(8)
        took = time.monotonic() - t0
        assert ei.value.code == _lib.ETIMEOUT, ei.value
        assert took < 6.0, took
        with pytest.raises(_lib.StencilError, match="failed earlier"):
            job.run(4)
    finally:
        t1 = time.monotonic()
        job.close()
        assert time.monotonic() - t1 < 15.0


def test_missing_rank_fails_communicator_creation_in_time(gpu):
    """Communicator creation (stencil_slab_create_rank) is a collective: rank
    0 of 2 whose peer never arrives gets STENCIL_ETIMEOUT after the job's
    deadline (STENCIL_SLAB_TIMEOUT_MS) instead of blocking in RCCL's bootstrap
    forever.  In a child process: the abandoned helper thread stays blocked
    in the bootstrap until that process exits (slab.hip, HipDev::comm_init_rank)."""
    import json
    import os
    import subprocess
    import sys
    import time
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = (
        "import json, time\n"
        "from stencil_amd import _lib\n"
        "from stencil_amd.engine import SlabJob, StencilSpec\n"
        "spec = StencilSpec(dims=3, dtype='fp64', shape='star')\n"
        "uid = SlabJob.unique_id()\n"
        "t0 = time.monotonic()\n"
        "try:\n"
        f"    SlabJob(spec, 64, 64, 32, [{int(gpu)}], rank=(2, 0, uid)).close()\n"
        "    print(json.dumps({'code': 0, 'took': time.monotonic() - t0}))\n"
        "except _lib.StencilError as e:\n"
        "    print(json.dumps({'code': e.code, 'took': time.monotonic() - t0, 'msg': str(e)}))\n"
    )
    env = dict(os.environ, STENCIL_SLAB_TIMEOUT_MS="2000")
    t0 = time.monotonic()
    p = subprocess.run([sys.executable, "-c", code], cwd=root, env=env, capture_output=True, text=True, timeout=90)
    assert p.returncode == 0, (p.returncode, p.stderr[-2000:])
    res = json.loads(p.stdout.strip().splitlines()[-1])
    assert res["code"] == _lib.ETIMEOUT, res
    assert 1.5 < res["took"] < 10.0, res
    assert "not every rank joined" in res["msg"], res
    assert time.monotonic() - t0 < 60.0


@pytest.mark.parametrize("form", ["signalled", "serial"])
def test_exchange_time_beside_the_launch(gpu, monkeypatch, form):
    """stencil_slab_exchange_time on the HIP path: an interior-rank rehearsal
    (one periodic slab, RCCL to itself) records one exchange per timed round;
    face-signalled rounds run most of the transfer beside their launch,
    serial rounds none of it."""
    monkeypatch.setenv("STENCIL_SLAB_SERIAL", "1" if form == "serial" else "0")
    spec = StencilSpec(dims=3, dtype="fp64", shape="star")
    job = SlabJob(spec, 512, 512, 128, [gpu], exchange="rccl", periodic=True)
    try:
        assert job.round_form() == (1 if form == "signalled" else 3)
        job.fill_initial("reference")
        job.run(8)
        job.kernel_timing(True)
        job.run(24)
        kt, xt = job.kernel_time(), job.exchange_time()
        assert kt["launches"] == 6 and xt["exchanges"] == 6, (kt, xt)
        assert xt["transfer_ms"] > 0 and 0 <= xt["beside_ms"] <= xt["transfer_ms"] + 1e-3, xt
        frac = xt["beside_ms"] / xt["transfer_ms"]
        if form == "signalled":
            assert frac > 0.5, xt
        else:
            assert frac < 0.05, xt
    finally:
        job.close()


def _gated_ring(gpu, monkeypatch, env, nx=130, ny=64, nz=40, it=17):
    """One periodic slab, device-copy halos, face-signalled rounds with the
    given environment: (round_info, final grid)."""
    monkeypatch.setenv("STENCIL_SLAB_SIGNAL", "1")
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    spec = StencilSpec(dims=3, dtype="fp64", shape="star")
    job = SlabJob(spec, nx, ny, nz, [gpu], exchange="copy", periodic=True)
    try:
        info = job.round_info()
        job.fill_initial("random", 5)
        job.run(it)
        return info, job.download()
    finally:
        job.close()


@pytest.mark.parametrize("exchange", ["copy", "rccl"])
def test_gated_rounds_match_boundary_launches(gpu, monkeypatch, exchange):
    """Halo-gated face-signalled rounds (the default for one-round grids such
    as C2's 512^3 slab): the launch follows the previous launch on its queue
    with no event wait for the exchange; only its halo-reading workgroups
    wait for the exchange-completion word.  Bitwise the boundary + interior
    rounds, over copies and RCCL to itself, through remainder rounds."""
    nx, ny, nz, it = 130, 64, 40, 17
    want = _periodic_job(gpu, monkeypatch, nx, ny, nz, it, False)
    monkeypatch.setenv("STENCIL_SLAB_SIGNAL", "1")
    spec = StencilSpec(dims=3, dtype="fp64", shape="star")
    job = SlabJob(spec, nx, ny, nz, [gpu], exchange=exchange, periodic=True)
    try:
        assert job.round_info() == {"form": 1, "gated": True, "confined": False}
        job.fill_initial("random", 5)
        job.run(it - 5)
        job.run(5)  # continued calls: the first round after a sync waits on nothing, gated all the same
        got = job.download()
    finally:
        job.close()
    assert np.array_equal(got.view(np.uint8), want.view(np.uint8))


def test_gated_rounds_slow_exchange(gpu, monkeypatch):
    """A 3 ms spin before every exchange's copies (STENCIL_SLAB_COPY_DELAY_US,
    debug library): each launch's halo-reading chunks must wait for the
    previous exchange's completion word.  Bitwise the boundary + interior
    rounds."""
    want = _periodic_job(gpu, monkeypatch, 130, 64, 40, 17, False)
    info, got = _gated_ring(gpu, monkeypatch, {"STENCIL_SLAB_COPY_DELAY_US": "3000"})
    assert info["gated"] and info["form"] == 1
    assert np.array_equal(got.view(np.uint8), want.view(np.uint8))


def test_gated_rounds_slow_exchange_need_the_gate(gpu, monkeypatch):
    """The test above has teeth: with the gate's need forced to 0
    (STENCIL_SLAB_GATE_SKIP, debug library) nothing orders a launch after the
    slow exchange, and the halos it reads are stale."""
    want = _periodic_job(gpu, monkeypatch, 130, 64, 40, 17, False)
    info, got = _gated_ring(gpu, monkeypatch, {"STENCIL_SLAB_COPY_DELAY_US": "3000", "STENCIL_SLAB_GATE_SKIP": "1"})
    assert info["gated"]
    assert not np.array_equal(got.view(np.uint8), want.view(np.uint8))


def test_gate_off_waits_for_the_exchange_event(gpu, monkeypatch):
    """STENCIL_SLAB_GATE=0: the face-signalled rounds of round 5 (the launch
    waits for the exchange stream's event), bitwise the same."""
    want = _periodic_job(gpu, monkeypatch, 130, 64, 40, 17, False)
    info, got = _gated_ring(gpu, monkeypatch, {"STENCIL_SLAB_GATE": "0", "STENCIL_SLAB_COPY_DELAY_US": "3000"})
    assert not info["gated"] and info["form"] == 1
    assert np.array_equal(got.view(np.uint8), want.view(np.uint8))
