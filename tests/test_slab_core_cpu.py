"""The multi-GPU slab job's round logic on the CPU.

csrc/slab_core.hpp holds the z-slab job -- the z split, the three round forms
(boundary + interior launches, face-signalled launches, rolling one-grid
passes), the halo exchange and its posting order, the remainder rounds, the
ghost-plane restores -- once, over a device backend.  The product binds it to
HIP and RCCL (csrc/slab.hip); tests/cpu_slab/fake_dev.cpp binds it to a CPU
fake device whose sweeps are the oracle's and whose communicator is an
in-process mailbox.  So the code that runs on the 8-GPU node runs here, at
world 2 and 3 (single-process jobs and rank-mode jobs, one thread per rank),
checked bit for bit against ONE grid swept by the oracle.
"""
import threading

import numpy as np
import pytest

from oracle import binding as ob
from stencil_amd import _lib
from stencil_amd.engine import SlabJob, StencilSpec
from tests.cpu_slab import binding as fb

pytestmark = pytest.mark.skipif(not fb.available(), reason="tests/cpu_slab/libslab_fake.so not built (run make)")


@pytest.fixture()
def fake():
    lib = fb.load()
    lib.set_k(0)
    lib.set_signal(True)
    lib.set_free_bytes(1 << 40)
    yield lib
    lib.set_k(0)
    lib.set_signal(True)
    lib.set_free_bytes(1 << 40)


def oracle_grid(spec, nx, ny, nz, sweeps, kind="random", seed=11):
    p = ob.problem(3, spec.dtype, spec.shape, spec.radius, "naive", nx, ny, nz)
    return ob.run(p, sweeps, kind, seed)


def assert_bitwise(got, want):
    assert got.shape == want.shape
    if not np.array_equal(got.view(np.uint8), want.view(np.uint8)):
        diff = np.argwhere(got != want)
        raise AssertionError(f"{len(diff)} cells differ, first at {diff[:4].tolist()}")


SHAPES = [
    ("fp64", "star", 4),
    ("fp32", "star", 5),
    ("fp64", "box", 4),
    ("fp32", "box", 3),
]


@pytest.mark.parametrize("dtype,shape,k", SHAPES)
@pytest.mark.parametrize("nslabs", [1, 2, 3])
@pytest.mark.parametrize("exchange,devices", [("rccl", "distinct"), ("copy", "distinct"), ("copy", "shared")])
def test_single_process_job_equals_one_grid(fake, dtype, shape, k, nslabs, exchange, devices):
    """N slabs from one process (stencil_slab_create), every round form the
    device assignment selects: distinct devices -> face-signalled full rounds,
    shared -> boundary + interior launches; remainder rounds; bitwise."""
    fake.set_k(k)
    spec = StencilSpec(dims=3, dtype=dtype, shape=shape)
    nx, ny, nz = 13, 7, 3 * k * nslabs + 2  # remainder planes to the lowest slabs
    devs = list(range(nslabs)) if devices == "distinct" else [0] * nslabs
    job = SlabJob(spec, nx, ny, nz, devs, exchange=exchange, lib=fake)
    job.fill_initial("random", 11)
    sweeps = 0
    for it in (2 * k + 1, k, 1, k - 1):  # full + remainder rounds, continued calls
        fake.stats(reset=True)
        job.run(it)
        sweeps += it
        st = fake.stats()
        full = it // k
        signalled = len(set(devs)) == len(devs)
        assert st["signal_sweeps"] == (full * nslabs if signalled else 0), st
        assert_bitwise(job.download(), oracle_grid(spec, nx, ny, nz, sweeps))
    job.close()


@pytest.mark.parametrize("dtype,shape,k", SHAPES)
@pytest.mark.parametrize("nslabs", [1, 2, 3])
@pytest.mark.parametrize("exchange", ["rccl", "copy"])
def test_serial_rounds_equal_one_grid(fake, monkeypatch, dtype, shape, k, nslabs, exchange):
    """STENCIL_SLAB_SERIAL=1: every full round as ONE plain launch of the
    whole slab, then the exchange (no face signals, nothing beside the
    launch); distinct devices, remainder rounds; bitwise."""
    monkeypatch.setenv("STENCIL_SLAB_SERIAL", "1")
    fake.set_k(k)
    spec = StencilSpec(dims=3, dtype=dtype, shape=shape)
    nx, ny, nz = 13, 7, 3 * k * nslabs + 2
    job = SlabJob(spec, nx, ny, nz, list(range(nslabs)), exchange=exchange, lib=fake)
    job.fill_initial("random", 11)
    sweeps = 0
    for it in (2 * k + 1, k, 1, k - 1):
        fake.stats(reset=True)
        job.run(it)
        sweeps += it
        assert fake.stats()["signal_sweeps"] == 0
        assert_bitwise(job.download(), oracle_grid(spec, nx, ny, nz, sweeps))
    job.close()


@pytest.mark.parametrize("nslabs", [1, 2, 3])
@pytest.mark.parametrize("exchange", ["rccl", "copy"])
def test_periodic_ring_equals_replicated_grid(fake, nslabs, exchange):
    """PERIODIC joins the z ends (the self-ring rehearsal of an interior
    rank): equal to the middle third of a grid of three copies swept by the
    oracle, for fewer sweeps than one copy's planes."""
    fake.set_k(4)
    spec = StencilSpec(dims=3, dtype="fp64", shape="star")
    nx, ny, nz = 9, 6, 10 * nslabs
    job = SlabJob(spec, nx, ny, nz, list(range(nslabs)), exchange=exchange, periodic=True, lib=fake)
    p1 = ob.problem(3, "fp64", "star", 1, "naive", nx, ny, nz)
    g0 = ob.init(p1, "random", 5)
    job.upload(g0)
    sweeps = 9
    job.run(sweeps)
    got = job.download()
    p3 = ob.problem(3, "fp64", "star", 1, "naive", nx, ny, 3 * nz)
    g3 = ob.init(p3, "reference")
    inner = g0[1:nz + 1]
    g3[1:1 + 3 * nz] = np.concatenate([inner, inner, inner])
    a, b = g3.copy(), g3.copy()
    for _ in range(sweeps):
        ob.sweep(p3, a, b, 0, 3 * nz)
        a, b = b, a
    assert_bitwise(got[1:nz + 1], a[1 + nz:1 + 2 * nz])
    job.close()


@pytest.mark.parametrize("dtype,shape,k", [("fp64", "star", 4), ("fp32", "box", 3)])
@pytest.mark.parametrize("nslabs", [1, 2, 3])
@pytest.mark.parametrize("margin_extra", [1, 3, 40])
@pytest.mark.parametrize("overlap", ["1", "0"])
def test_rolling_slabs_equal_one_grid(fake, monkeypatch, dtype, shape, k, nslabs, margin_extra, overlap):
    """ROLLING: one resident grid per slab plus a margin -- from one-plane
    launches (margin = K r + 1) to one launch per pass; down and up passes,
    remainder passes, the halo exchange (overlapped: faces computed into a
    staging buffer first and exchanged beside the pass; or after the pass)
    and the global ends' ghost restores; bitwise the oracle's one grid."""
    monkeypatch.setenv("STENCIL_SLAB_ROLLING_OVERLAP", overlap)
    fake.set_k(k)
    spec = StencilSpec(dims=3, dtype=dtype, shape=shape)
    nx, ny, nz = 11, 5, 7 * nslabs + 1
    margin = k + margin_extra
    job = SlabJob(spec, nx, ny, nz, list(range(nslabs)), exchange="rccl", rolling=True, margin=margin, lib=fake)
    info = job.rolling_info()
    assert info["margin"] == margin
    assert info["launches_per_pass"] == -(-(nz // nslabs + (1 if nz % nslabs else 0)) // margin_extra)
    job.fill_initial("random", 3)
    sweeps = 0
    for it in (k, 2 * k + 2, 1):  # a down pass, up + down + a 2-sweep remainder pass, a single
        fake.stats(reset=True)
        job.run(it)
        sweeps += it
        st = fake.stats()
        assert st["signal_sweeps"] == 0  # rolling rounds are plain passes
        # launches per pass: the z-range launches, plus one face launch per
        # shared face when overlapped
        rounds = -(-it // k)
        faces = 2 * (nslabs - 1) if overlap == "1" else 0
        per_pass = sum(-(-(nz // nslabs + (1 if r < nz % nslabs else 0)) // margin_extra) for r in range(nslabs))
        assert st["sweeps"] == rounds * (per_pass + faces), st
        assert_bitwise(job.download(), oracle_grid(spec, nx, ny, nz, sweeps, seed=3))
    job.kernel_timing(True)
    job.run(k)
    kt = job.kernel_time()
    assert kt["rolling"] and not kt["signalled"] and kt["launches"] == 1 and kt["cells_per_launch"] > 0
    job.close()


def test_rolling_margin_from_free_memory(fake):
    """margin 0 sizes the margin from the device's free memory (capped at 512
    planes; refused when even 4 (K r + 1) planes do not fit)."""
    fake.set_k(4)
    spec = StencilSpec(dims=3, dtype="fp64", shape="star")
    job = SlabJob(spec, 16, 16, 40, [0, 1], exchange="rccl", rolling=True, margin=0, lib=fake)
    assert job.rolling_info()["margin"] == 512
    job.close()
    fake.set_free_bytes(4 << 30)  # the communicator's reserve and nothing beside it
    with pytest.raises(_lib.StencilError, match="do not fit"):
        SlabJob(spec, 16, 16, 40, [0, 1], exchange="rccl", rolling=True, margin=0, lib=fake)


def _rank_jobs(fake, spec, grid, nranks, fn, rolling=False, margin=0):
    """Run `fn(job, rank)` for a rank-mode job in one thread per rank (ctypes
    releases the GIL: the ranks' blocking receives overlap like processes)."""
    uid = SlabJob.unique_id(lib=fake)
    out, errs = [None] * nranks, [None] * nranks

    def body(r):
        try:
            job = SlabJob(spec, *grid, [r], rank=(nranks, r, uid), rolling=rolling, margin=margin, lib=fake)
            out[r] = fn(job, r)
            job.close()
        except Exception as exc:  # surfaced below
            errs[r] = exc

    th = [threading.Thread(target=body, args=(r,)) for r in range(nranks)]
    for t in th:
        t.start()
    for t in th:
        t.join(120)
    assert not any(t.is_alive() for t in th), "a rank hung"
    return out, errs


@pytest.mark.parametrize("nranks", [2, 3])
@pytest.mark.parametrize("rolling", [False, True, "serial"])
@pytest.mark.parametrize("shape", ["star", "box"])
def test_rank_mode_equals_one_grid(fake, monkeypatch, nranks, rolling, shape):
    """Rank mode (stencil_slab_create_rank: one slab per process, peers by
    global index, as torch.distributed.run launches bench.py on the 8-GPU
    node), one thread per rank: each rank's planes, assembled, bitwise the
    oracle's one grid; face-signalled rounds when not rolling."""
    if rolling == "serial":  # rolling rounds with the exchange after the pass
        monkeypatch.setenv("STENCIL_SLAB_ROLLING_OVERLAP", "0")
        rolling = True
    k = 4 if shape == "star" else 3
    fake.set_k(k)
    spec = StencilSpec(dims=3, dtype="fp64", shape=shape)
    nx, ny, nz = 10, 6, 9 * nranks + 1
    sweeps = 2 * k + 3

    def fn(job, r):
        inf = job.info(0)
        job.fill_initial("random", 21)
        job.run(k + 1)
        job.run(sweeps - k - 1)
        return inf, job.download(), job.plane_sums()

    out, errs = _rank_jobs(fake, spec, (nx, ny, nz), nranks, fn, rolling=rolling, margin=k + 2)
    assert not any(errs), errs
    want = oracle_grid(spec, nx, ny, nz, sweeps, seed=21)
    got = np.zeros_like(want)
    for r in range(nranks):
        inf, dense, _ = out[r]
        z0 = inf["first"] + (0 if r > 0 else -1)
        z1 = inf["first"] + inf["planes"] + (1 if r == nranks - 1 else 0)
        got[z0 + 1:z1 + 1] = dense[z0 + 1:z1 + 1]
    assert_bitwise(got, want)


def test_rank_mode_rejects_tiny_slabs_on_every_rank(fake):
    """A job whose smallest slab is below the halo depth fails on EVERY rank
    before the communicator's collective init (no rank left waiting in it)."""
    fake.set_k(4)
    spec = StencilSpec(dims=3, dtype="fp64", shape="star")
    out, errs = _rank_jobs(fake, spec, (8, 8, 11), 3, lambda job, r: None)  # 11 / 3 = 3 < 4 halo planes
    assert all(isinstance(e, _lib.StencilError) and "use fewer GPUs" in str(e) for e in errs), errs


def test_single_process_rejects_tiny_slabs(fake):
    fake.set_k(4)
    spec = StencilSpec(dims=3, dtype="fp64", shape="star")
    with pytest.raises(_lib.StencilError, match="use fewer GPUs"):
        SlabJob(spec, 8, 8, 7, [0, 1], exchange="copy", lib=fake)


def test_exchange_counts_per_round(fake):
    """Per full round every shared face moves once each way: 2 (N - 1) sends
    and receives for N slabs (a periodic ring: 2 N)."""
    fake.set_k(4)
    spec = StencilSpec(dims=3, dtype="fp64", shape="star")
    for periodic, n in ((False, 3), (True, 3), (True, 1)):
        job = SlabJob(spec, 8, 8, 24, list(range(n)), exchange="rccl", periodic=periodic, lib=fake)
        job.fill_initial("reference")
        fake.stats(reset=True)
        job.run(8)  # two full rounds
        st = fake.stats()
        faces = 2 * n if periodic else 2 * (n - 1)
        assert st["sends"] == st["recvs"] == 2 * faces, (periodic, n, st)
        job.close()


# ---- round 5: bounded-time failure, the rolling upload check, round forms, layout

@pytest.mark.parametrize("nranks", [2, 3])
@pytest.mark.parametrize("rolling", [False, True])
def test_silent_peer_fails_every_rank_in_bounded_time(fake, monkeypatch, nranks, rolling):
    """A rank that stops posting its sends (FAKE_SLAB_MUTE_RANK) after the
    fill's exchange: every rank's run() returns STENCIL_ETIMEOUT within the
    job's deadline -- the ranks waiting on it directly, the muted rank once the
    others stopped (fail fast; stencil_rma.cpp:334-338's
    never-waited reply hangs instead).  Later calls fail at once; destroy works."""
    import time
    k = 4
    fake.set_k(k)
    spec = StencilSpec(dims=3, dtype="fp64", shape="star")
    muted = nranks - 1  # the top rank: one neighbour, one send per exchange
    monkeypatch.setenv("FAKE_SLAB_MUTE_RANK", str(muted))
    monkeypatch.setenv("FAKE_SLAB_MUTE_AFTER", "1" if rolling else "2")  # the fill's exchanges
    timeout_ms = 800

    def fn(job, r):
        job.set_timeout(timeout_ms)
        job.fill_initial("reference")
        t0 = time.monotonic()
        try:
            job.run(6 * k)
            return ("ok", time.monotonic() - t0, None)
        except _lib.StencilError as exc:
            took = time.monotonic() - t0
            try:
                job.run(k)
                again = "ran"
            except _lib.StencilError as exc2:
                again = exc2.code, str(exc2)
            return (exc.code, took, again)

    out, errs = _rank_jobs(fake, spec, (8, 6, 8 * nranks), nranks, fn, rolling=rolling, margin=k + 2)
    assert not any(errs), errs
    for r, (code, took, again) in enumerate(out):
        assert code == _lib.ETIMEOUT, (r, out)
        # a rank waits at most one deadline per receive it is blocked on, and
        # the muted rank only notices once a neighbour has given up
        assert took < 3 * timeout_ms / 1000 + 1.0, (r, took)
        assert again[0] == _lib.ETIMEOUT and "failed earlier" in again[1], again


@pytest.mark.parametrize("nslabs", [1, 2, 3])
@pytest.mark.parametrize("placements", [None, "3", "16"])
def test_grid_placement_search_keeps_results(fake, monkeypatch, nslabs, placements):
    """place_grids with the product's default (STENCIL_SLAB_PLACEMENTS unset:
    one allocation, no search -- round 6: the search gained 0.8 % at C2's 1000
    sweeps) and with 3 / 16 candidate pairs per slab, as bench.py opts in: the
    chosen pair runs the job, the others are freed, and the result is bitwise
    the oracle's one grid."""
    monkeypatch.delenv("FAKE_SLAB_PLACE", raising=False)
    if placements is None:
        monkeypatch.delenv("STENCIL_SLAB_PLACEMENTS", raising=False)
    else:
        monkeypatch.setenv("STENCIL_SLAB_PLACEMENTS", placements)
    fake.set_k(4)
    spec = StencilSpec(dims=3, dtype="fp64", shape="star")
    nx, ny, nz = 11, 6, 9 * nslabs + 1
    job = SlabJob(spec, nx, ny, nz, list(range(nslabs)), exchange="rccl", lib=fake)
    try:
        job.fill_initial("random", 4)
        job.run(10)
        assert_bitwise(job.download(), oracle_grid(spec, nx, ny, nz, 10, seed=4))
    finally:
        job.close()


@pytest.mark.parametrize("present", [1, 2])
def test_missing_rank_fails_creation_in_bounded_time(fake, monkeypatch, present):
    """Communicator creation is a collective: with a rank that never calls
    stencil_slab_create_rank, the ranks that did get STENCIL_ETIMEOUT after
    STENCIL_SLAB_TIMEOUT_MS instead of waiting for it forever."""
    import time
    fake.set_k(4)
    spec = StencilSpec(dims=3, dtype="fp64", shape="star")
    monkeypatch.setenv("STENCIL_SLAB_TIMEOUT_MS", "600")
    nranks = present + 1
    uid = SlabJob.unique_id(lib=fake)
    res = [None] * present

    def body(r):
        t0 = time.monotonic()
        try:
            SlabJob(spec, 8, 6, 8 * nranks, [r], rank=(nranks, r, uid), lib=fake).close()
            res[r] = ("created", time.monotonic() - t0)
        except _lib.StencilError as exc:
            res[r] = (exc.code, time.monotonic() - t0, str(exc))

    th = [threading.Thread(target=body, args=(r,)) for r in range(present)]
    for t in th:
        t.start()
    for t in th:
        t.join(30)
    assert not any(t.is_alive() for t in th), "a rank hung in creation"
    for r in range(present):
        assert res[r][0] == _lib.ETIMEOUT, res
        assert 0.5 < res[r][1] < 5.0, res


@pytest.mark.parametrize("case", ["signalled", "boundary", "staged", "rolling", "serial"])
def test_exchange_time_pairs_every_timed_round(fake, monkeypatch, case):
    """stencil_slab_exchange_time: with kernel timing on, each timed round
    (full or remainder) records one exchange span on slab 0's exchange
    stream, paired with its launch span; fill / upload exchanges are not
    counted; beside <= transfer."""
    k = 4
    fake.set_k(k)
    fake.set_signal(case in ("signalled", "staged"))
    if case == "staged":  # the fake's stand-in for a grid of several rounds of workgroups
        monkeypatch.setenv("FAKE_SLAB_CONFINE", "1")
    if case == "serial":
        monkeypatch.setenv("STENCIL_SLAB_SERIAL", "1")
    spec = StencilSpec(dims=3, dtype="fp64", shape="star")
    job = SlabJob(spec, 10, 6, 40, [0, 1], exchange="rccl", rolling=case == "rolling", margin=k + 2, lib=fake)
    try:
        assert job.round_form() == {"signalled": 1, "boundary": 0, "staged": 4, "rolling": 2, "serial": 3}[case]
        job.fill_initial("reference")
        job.run(k)
        job.kernel_timing(True)
        job.run(3 * k + 1)  # three full rounds and a remainder round
        kt = job.kernel_time()
        xt = job.exchange_time()
        assert kt["launches"] == 4 and xt["exchanges"] == 4, (kt, xt)
        assert 0.0 <= xt["beside_ms"] <= xt["transfer_ms"] + 1e-3, xt
        job.fill_initial("reference")  # fill's exchanges are outside any round
        assert job.exchange_time()["exchanges"] == 4
        job.kernel_timing(False)
        assert job.exchange_time()["exchanges"] == 0
    finally:
        job.close()
        fake.set_signal(True)


def test_upload_checks_the_rolling_ghost_ring(fake):
    """ROLLING slabs need the same x/y ghost ring in every plane:
    upload refuses a host grid whose ring varies with z, and takes it for a
    two-grid job, where it is computed right."""
    fake.set_k(4)
    spec = StencilSpec(dims=3, dtype="fp64", shape="star")
    nx, ny, nz = 9, 6, 12
    p1 = ob.problem(3, "fp64", "star", 1, "naive", nx, ny, nz)
    good = ob.init(p1, "random", 5)
    bad = good.copy()
    bad[7, 0, 3] = 0.5  # a y-ghost cell of plane 6
    job = SlabJob(spec, nx, ny, nz, [0, 1], exchange="rccl", rolling=True, margin=8, lib=fake)
    job.upload(good)
    with pytest.raises(_lib.StencilError, match="same x/y ghost ring"):
        job.upload(bad)
    job.close()
    two = SlabJob(spec, nx, ny, nz, [0, 1], exchange="rccl", lib=fake)
    two.upload(bad)
    two.run(5)
    want = bad.copy()
    a, b = want, want.copy()
    for _ in range(5):
        ob.sweep(p1, a, b, 0, nz)
        a, b = b, a
    assert_bitwise(two.download(), a)
    two.close()


@pytest.mark.parametrize("where", ["interior of ghost plane -2", "ring of ghost plane -1", "ring of plane 5",
                                   "interior of top ghost plane"])
def test_upload_checks_the_rolling_ghost_ring_radius_two(fake, where):
    """with r = 2 the bottom ghost planes -2 and -1 must
    be equal in every cell and every plane's ring must equal plane -2's ring;
    the check used plane r - 1 as its own reference and never compared plane
    -2.  A top ghost plane's interior is not constrained (no pass moves it
    into another plane's slot)."""
    fake.set_k(4)
    spec = StencilSpec(dims=3, dtype="fp64", shape="star", radius=2)
    nx, ny, nz = 9, 6, 12
    p2 = ob.problem(3, "fp64", "star", 2, "naive", nx, ny, nz)
    good = ob.init(p2, "random", 5)
    bad = good.copy()
    # host index = plane + 2, row + 2, column + 2
    z, y, x = {"interior of ghost plane -2": (0, 4, 5), "ring of ghost plane -1": (1, 0, 5),
               "ring of plane 5": (7, 3, 1), "interior of top ghost plane": (nz + 3, 4, 5)}[where]
    bad[z, y, x] = 0.5
    job = SlabJob(spec, nx, ny, nz, [0, 1], exchange="rccl", rolling=True, margin=12, lib=fake)
    try:
        job.upload(good)
        if where == "interior of top ghost plane":
            job.upload(bad)
        else:
            with pytest.raises(_lib.StencilError, match="same x/y ghost ring"):
                job.upload(bad)
    finally:
        job.close()


@pytest.mark.parametrize("case,form", [
    (dict(devs=[0, 1]), 1),                      # distinct devices: face-signalled
    (dict(devs=[0, 0], exchange="copy"), 0),     # shared: boundary + interior
    (dict(devs=[0, 1], rolling=True), 2),
    (dict(devs=[0, 1], serial=True), 3),
])
def test_round_form_and_signalled_flag(fake, monkeypatch, case, form):
    """stencil_slab_round_form gives the form; kernel_time's `signalled`
    stays 0/1 (it had become the form code)."""
    fake.set_k(4)
    if case.get("serial"):
        monkeypatch.setenv("STENCIL_SLAB_SERIAL", "1")
    spec = StencilSpec(dims=3, dtype="fp64", shape="star")
    job = SlabJob(spec, 8, 6, 16, case["devs"], exchange=case.get("exchange", "rccl"),
                  rolling=case.get("rolling", False), margin=6 if case.get("rolling") else 0, lib=fake)
    job.fill_initial("reference")
    job.kernel_timing(True)
    job.run(4)
    kt = job.kernel_time()
    assert job.round_form() == form == kt["form"]
    assert kt["signalled"] == (form == 1)
    job.close()


@pytest.mark.parametrize("dtype", ["fp32", "fp64"])
def test_fake_layout_is_the_product_layout(fake, dtype):
    """The fake device's layout arithmetic is api.hip's, the row-pitch rule
    included, over widths around every padded pitch class."""
    widths = [1, 7, 64, 500, 512, 2048, 3000, 4000, 4080, 4096, 4100, 8176, 8192, 8200, 16384]
    for nx in widths:
        for r, halo in ((1, 0), (1, 4), (2, 0)):
            prob = _lib.make_problem(dims=3, dtype=_lib.F64 if dtype == "fp64" else _lib.F32, radius=r,
                                     nx=nx, ny=5, nz=9, halo=halo)
            want, got = _lib.make_layout(prob), fake.layout(prob)
            for f, _ in _lib.Layout._fields_[1:]:
                assert getattr(got, f) == getattr(want, f), (nx, r, halo, f)


@pytest.mark.parametrize("dtype,shape,k", SHAPES)
@pytest.mark.parametrize("nslabs", [1, 2, 3])
@pytest.mark.parametrize("exchange", ["rccl", "copy"])
def test_staged_rounds_equal_one_grid(fake, monkeypatch, dtype, shape, k, nslabs, exchange):
    """STAGED rounds (the default for slabs whose launch takes several rounds
    of workgroups; FAKE_SLAB_CONFINE=1 makes the fake's slabs such): per full
    round the two face quarters, then the middle, the exchange beside it;
    remainder rounds and continued calls; bitwise one grid."""
    monkeypatch.setenv("FAKE_SLAB_CONFINE", "1")
    fake.set_k(k)
    spec = StencilSpec(dims=3, dtype=dtype, shape=shape)
    nx, ny, nz = 13, 7, 10 * k * nslabs + 3
    job = SlabJob(spec, nx, ny, nz, list(range(nslabs)), exchange=exchange, lib=fake)
    assert job.round_form() == 4
    job.fill_initial("random", 11)
    sweeps = 0
    for it in (2 * k + 1, k, 1, k - 1):
        fake.stats(reset=True)
        job.run(it)
        sweeps += it
        st = fake.stats()
        assert st["signal_sweeps"] == 0
        full, rem = it // k, it % k
        # 3 launches per slab and full round (face quarters + middle); a remainder round: boundary + interior (3)
        assert st["sweeps"] == 3 * nslabs * (full + (1 if rem else 0)), st
        assert_bitwise(job.download(), oracle_grid(spec, nx, ny, nz, sweeps))
    job.close()


@pytest.mark.parametrize("nranks", [2, 3])
def test_staged_rank_mode_equals_one_grid(fake, monkeypatch, nranks):
    monkeypatch.setenv("FAKE_SLAB_CONFINE", "1")
    k = 4
    fake.set_k(k)
    spec = StencilSpec(dims=3, dtype="fp64", shape="star")
    nx, ny, nz = 10, 6, 12 * nranks + 1
    sweeps = 3 * k + 2

    def fn(job, r):
        assert job.round_form() == 4
        job.fill_initial("random", 21)
        job.run(sweeps)
        return job.info(0), job.download()

    out, errs = _rank_jobs(fake, spec, (nx, ny, nz), nranks, fn)
    assert not any(errs), errs
    want = oracle_grid(spec, nx, ny, nz, sweeps, seed=21)
    got = np.zeros_like(want)
    for r in range(nranks):
        inf, dense = out[r]
        z0 = inf["first"] + (0 if r > 0 else -1)
        z1 = inf["first"] + inf["planes"] + (1 if r == nranks - 1 else 0)
        got[z0 + 1:z1 + 1] = dense[z0 + 1:z1 + 1]
    assert_bitwise(got, want)


@pytest.mark.parametrize("nslabs", [1, 2, 3])
@pytest.mark.parametrize("exchange", ["rccl", "copy"])
@pytest.mark.parametrize("gate", [True, False])
def test_gated_rounds_number_their_exchanges(fake, monkeypatch, nslabs, exchange, gate):
    """Halo-gated face-signalled rounds (round 6): every exchange stores its
    number in the slab's completion word, and every gated launch waits for
    the number of the last exchange issued before it -- on the fake's
    synchronous streams that exchange is complete when the launch is issued,
    so any other number is a violation (on a GPU: a launch waiting for an
    exchange that never comes, or reading halos too early).  Full and
    remainder rounds, continued calls, a refill in between; bitwise one grid.
    FAKE_SLAB_GATE=0: the event-waiting rounds, no completion stores."""
    if not gate:
        monkeypatch.setenv("FAKE_SLAB_GATE", "0")
    k = 4
    fake.set_k(k)
    spec = StencilSpec(dims=3, dtype="fp64", shape="star")
    nx, ny, nz = 11, 7, 3 * k * nslabs + 1
    job = SlabJob(spec, nx, ny, nz, list(range(nslabs)), exchange=exchange, lib=fake)
    try:
        assert job.round_info() == {"form": 1, "gated": gate, "confined": False}
        fake.gate_stats(reset=True)
        job.fill_initial("random", 3)
        sweeps = rounds = 0
        for it in (2 * k + 1, k, 3, 2 * k):
            job.run(it)
            sweeps += it
            rounds += it // k + (1 if it % k else 0)
        st = fake.gate_stats()
        full = sum(it // k for it in (2 * k + 1, k, 3, 2 * k))
        assert st["violations"] == 0, st
        assert st["gated"] == (full * nslabs if gate else 0), st
        # fill: two exchanges (both grids), then one per round, on every slab
        assert st["completions"] == ((2 + rounds) * nslabs if gate else 0), st
        assert_bitwise(job.download(), oracle_grid(spec, nx, ny, nz, sweeps, seed=3))
        job.fill_initial("random", 3)  # the numbering restarts with the counters
        job.run(k)
        assert fake.gate_stats()["violations"] == 0
        assert_bitwise(job.download(), oracle_grid(spec, nx, ny, nz, k, seed=3))
    finally:
        job.close()


@pytest.mark.parametrize("mode", ["one process", "rank mode"])
@pytest.mark.parametrize("invert,alt_kept", [("0", True), ("1", False)])
def test_staged_exchange_cu_budget_tuning(fake, monkeypatch, mode, invert, alt_kept):
    """a staged job with a confined exchange times its
    exchange with the default CU budget (1 per XCD) and, when the exchange
    outlasts most of the middle launch, with the alternative (4) in one more
    tuning round, and keeps the faster.  The fake's exchange stream sleeps
    FAKE_SLAB_WIRE_MS / cus ms (x cus when inverted), so the alternative is
    kept, or not; either way the grid stays bitwise one grid, in one process
    and in rank mode (each rank decides for its own slab)."""
    monkeypatch.setenv("FAKE_SLAB_CONFINE", "1")
    # 40 ms (10 ms with the alternative): a margin no scheduling hiccup of a
    # loaded host (pytest -n, the fake's threads) closes
    monkeypatch.setenv("FAKE_SLAB_WIRE_MS", "40")
    monkeypatch.setenv("FAKE_SLAB_WIRE_INVERT", invert)
    k = 4
    fake.set_k(k)
    spec = StencilSpec(dims=3, dtype="fp64", shape="star")
    nx, ny, nz = 10, 6, 12 * 2 + 1
    sweeps = 5 * k + 2

    def fn(job, r):
        info = job.round_info()
        job.fill_initial("random", 4)
        job.run(sweeps)
        return info, job.exchange_budget(), job.download()

    if mode == "one process":
        job = SlabJob(spec, nx, ny, nz, [0, 1], exchange="rccl", lib=fake)
        try:
            outs = [fn(job, 0)]
        finally:
            job.close()
    else:
        outs, errs = _rank_jobs(fake, spec, (nx, ny, nz), 2, fn)
        assert not any(errs), errs
    want = oracle_grid(spec, nx, ny, nz, sweeps, seed=4)
    for info, budget, dense in outs:
        assert info == {"form": 4, "gated": False, "confined": True}, info
        assert budget["alt_cus_per_xcd"] == 4 and budget["round_ms"] > 0 and budget["alt_round_ms"] > 0, budget
        assert budget["cus_per_xcd"] == (4 if alt_kept else 1), budget
        if alt_kept:
            assert budget["alt_round_ms"] < budget["round_ms"], budget
    if mode == "one process":
        assert_bitwise(outs[0][2], want)
    else:
        got = outs[0][2].copy()
        half = nz // 2 + 1  # rank 0 owns the first 13 planes
        got[half + 1:] = outs[1][2][half + 1:]
        assert_bitwise(got, want)


def test_staged_exchange_cu_budget_not_tried_for_a_short_exchange(fake, monkeypatch):
    """An exchange much shorter than the middle launch needs no more CUs: the
    second tuning round sets the face span and the alternative is never run."""
    monkeypatch.setenv("FAKE_SLAB_CONFINE", "1")
    fake.set_k(4)
    spec = StencilSpec(dims=3, dtype="fp64", shape="star")
    job = SlabJob(spec, 64, 48, 40, [0, 1], exchange="rccl", lib=fake)
    try:
        job.fill_initial("random", 4)
        job.run(6 * 4)
        b = job.exchange_budget()
        assert b["cus_per_xcd"] == 1 and b["round_ms"] > 0 and b["alt_round_ms"] == 0, b
    finally:
        job.close()
