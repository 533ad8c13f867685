"""Multi-GPU z-slab jobs driven by the C++ host (stencil_slab_*, csrc/slab.hip).

On a one-GPU box: N logical slabs on device 0 with device-copy halos (RCCL
refuses two ranks on one GPU), bitwise against one undivided grid and the
oracle; and the RCCL path as a periodic ring of one slab that sends its faces
to itself, bitwise against the same ring with device-copy halos."""
import numpy as np
import pytest

from oracle import binding as ob
from stencil_amd.engine import JacobiEngine, SlabJob, StencilSpec

pytestmark = pytest.mark.gpu


def same_bits(a, b):
    return a.shape == b.shape and np.array_equal(a.view(np.uint8), b.view(np.uint8))


def single_grid(gpu, spec, shape, it, seed):
    e = JacobiEngine(spec, *shape, device=gpu)
    e.reset("random", seed)
    fin, _ = e.iterate(it)
    return e.to_numpy(fin)


@pytest.mark.parametrize("dtype", ["fp64", "fp32"])
@pytest.mark.parametrize("shape_name", ["star", "box"])
@pytest.mark.parametrize("nslabs", [1, 2, 3, 4])
def test_slab_job_copy_equals_single_grid(gpu, dtype, shape_name, nslabs):
    """Rounds of K fused sweeps (and a shorter remainder round) over N slabs
    sharing the GPU: the gathered grid equals one grid's, bit for bit, and the
    per-plane sums equal the single grid's."""
    spec = StencilSpec(dims=3, dtype=dtype, shape=shape_name)
    shape = (70, 45, 41)
    job = SlabJob(spec, *shape, devices=[gpu] * nslabs, exchange="copy")
    k = job.info(0)["sweeps_per_round"]
    assert k == (3 if shape_name == "box" else 4)
    assert sum(job.info(i)["planes"] for i in range(nslabs)) == shape[2]
    job.fill_initial("random", 12)
    it = 3 * k + 1
    job.run(it)
    got = job.download()
    want = single_grid(gpu, spec, shape, it, 12)
    assert same_bits(got, want)
    e = JacobiEngine(spec, *shape, device=gpu)
    e.reset("random", 12)
    fin, _ = e.iterate(it)
    assert np.array_equal(job.plane_sums(), e.plane_sums(fin))
    job.close()


def test_slab_job_matches_oracle_and_upload(gpu):
    """Upload an arbitrary dense grid, run, download: the oracle's sweeps."""
    spec = StencilSpec(dims=3, dtype="fp64")
    nx, ny, nz = 33, 20, 26
    p = ob.problem(3, "fp64", "star", 1, "naive", nx, ny, nz)
    start = ob.init(p, "random", 99)
    job = SlabJob(spec, nx, ny, nz, devices=[gpu] * 3, exchange="copy")
    job.upload(start)
    assert same_bits(job.download(), start)
    job.run(11)
    a, b = start.copy(), start.copy()
    for _ in range(11):
        ob.sweep(p, a, b, 0, nz)
        a, b = b, a
    assert same_bits(job.download(), a)
    job.close()


@pytest.mark.parametrize("dtype", ["fp64", "fp32"])
@pytest.mark.parametrize("shape_name", ["star", "box"])
@pytest.mark.parametrize("exchange", ["copy", "rccl"])
def test_slab_job_signalled_rounds_equal_boundary_launches(gpu, monkeypatch, dtype, shape_name, exchange):
    """One slab per GPU: full rounds are ONE face-signalled launch per slab
    (the exchange waits on the face counters, csrc/slab.hip
    slab_round_signal); STENCIL_SLAB_SIGNAL=0 gives boundary + interior
    launches.  A periodic ring of one slab (its faces are its own halos, so
    both faces cross the exchange every round), full rounds and a remainder,
    bitwise equal both ways."""
    spec = StencilSpec(dims=3, dtype=dtype, shape=shape_name)
    shape = (131, 61, 47)
    res = []
    for sig in ("1", "0"):
        monkeypatch.setenv("STENCIL_SLAB_SIGNAL", sig)
        job = SlabJob(spec, *shape, devices=[gpu], exchange=exchange, periodic=True)
        k = job.info(0)["sweeps_per_round"]
        job.fill_initial("random", 23)
        job.run(4 * k + 1)
        job.run(k)
        res.append(job.download())
        job.close()
    assert same_bits(res[0], res[1])


@pytest.mark.parametrize("shape_name", ["star", "box"])
def test_slab_job_rccl_self_ring_equals_copies(gpu, shape_name):
    """The RCCL exchange (ncclCommInitAll over one device, a periodic ring of
    one slab: its faces go out through ncclSend and come back through
    ncclRecv into its own halos) equals the device-copy ring bit for bit."""
    spec = StencilSpec(dims=3, dtype="fp64", shape=shape_name)
    shape = (64, 40, 30)
    res = []
    for exchange in ("copy", "rccl"):
        job = SlabJob(spec, *shape, devices=[gpu], exchange=exchange, periodic=True)
        job.fill_initial("random", 5)
        job.run(9)
        res.append(job.download())
        job.close()
    assert same_bits(res[0], res[1])
    # periodic halos change the answer: not the Dirichlet grid's
    assert not same_bits(res[0], single_grid(gpu, spec, shape, 9, 5))


def test_slab_job_rccl_single_gpu_is_the_grid(gpu):
    """RCCL job of one non-periodic slab (no neighbours): the plain grid."""
    spec = StencilSpec(dims=3, dtype="fp32")
    shape = (50, 31, 22)
    job = SlabJob(spec, *shape, devices=[gpu], exchange="rccl")
    job.fill_initial("random", 8)
    job.run(10)
    assert same_bits(job.download(), single_grid(gpu, spec, shape, 10, 8))
    job.close()


def test_slab_job_rejects_bad_requests(gpu):
    from stencil_amd import _lib
    spec = StencilSpec(dims=3, dtype="fp64")
    with pytest.raises(_lib.StencilError):
        SlabJob(spec, 32, 32, 20, devices=[gpu, gpu], exchange="rccl")  # RCCL: one slab per GPU
    with pytest.raises(_lib.StencilError):
        SlabJob(spec, 32, 32, 6, devices=[gpu] * 3, exchange="copy")  # 2 planes per slab < K = 4
    with pytest.raises(_lib.StencilError):
        SlabJob(StencilSpec(dims=2), 32, 32, 1, devices=[gpu], exchange="copy")
    assert _lib.EXCHANGE_COPY == 1


def _device_count():
    import torch
    return torch.cuda.device_count()


@pytest.mark.skipif(_device_count() < 2, reason="needs at least 2 GPUs (one slab per distinct device)")
@pytest.mark.parametrize("ndev", [2, 4, 8])
@pytest.mark.parametrize("exchange", ["copy", "rccl"])
@pytest.mark.parametrize("signal", ["1", "0"])
@pytest.mark.parametrize("shape_name", ["star", "box"])
def test_slab_job_distinct_gpus(gpu, monkeypatch, ndev, exchange, signal, shape_name):
    """Slabs on DISTINCT GPUs -- cross-device RCCL send/recv, hipMemcpyPeerAsync
    with cross-device event waits, face-signalled rounds with N > 1 -- bitwise
    equal to one undivided grid on GPU 0 (runs only where >= 2 GPUs are
    visible: the driver's 8-GPU node, never the one-GPU test box)."""
    if _device_count() < ndev:
        pytest.skip(f"needs {ndev} GPUs")
    monkeypatch.setenv("STENCIL_SLAB_SIGNAL", signal)
    spec = StencilSpec(dims=3, dtype="fp64", shape=shape_name)
    shape = (131, 61, 12 * ndev + 5)
    job = SlabJob(spec, *shape, devices=list(range(ndev)), exchange=exchange)
    k = job.info(0)["sweeps_per_round"]
    job.fill_initial("random", 31)
    it = 3 * k + 2
    job.run(it)
    got = job.download()
    job.close()
    assert same_bits(got, single_grid(gpu, spec, shape, it, 31))


def test_bench_single_process_slab_job_rehearsal(gpu):
    """bench.py --gpus 2 without a launcher, rehearsed on one GPU (both slabs
    on GPU 0, device-copy halos): the JSON line, its roofline from the slab
    job's kernel events, and the bitwise check against the global grid."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--share-device",
                        "--exchange", "copy", "--n", "128", "--steps", "16", "--warmup", "4"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert p.returncode == 0, p.stderr[-2000:]
    line = json.loads(p.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 2 and line["value"] > 0 and line["config"]["grid"] == [128, 128, 256]
    assert line["multi_gpu_check"]["bitwise_equal"], line["multi_gpu_check"]
    assert line["roofline"]["launches"] > 0 and line["roofline"]["frac"] > 0
    assert "ONE process" in line["config"]["parallelism"]


@pytest.mark.parametrize("shape_name", ["star", "box"])
@pytest.mark.parametrize("periodic", [False, True])
def test_rank_mode_single_rank(gpu, shape_name, periodic):
    """Rank mode (stencil_slab_create_rank: ncclCommInitRank from an id made by
    stencil_slab_unique_id) with one rank: non-periodic it is the plain grid;
    as a periodic ring (the rank sends its faces to itself over RCCL) it equals
    the single-process job's device-copy ring, bit for bit."""
    spec = StencilSpec(dims=3, dtype="fp64", shape=shape_name)
    shape = (64, 40, 30)
    uid = SlabJob.unique_id()
    assert len(uid) == 128
    job = SlabJob(spec, *shape, devices=[gpu], periodic=periodic, rank=(1, 0, uid))
    info = job.info(0)
    assert info["first"] == 0 and info["planes"] == shape[2] and info["device"] == gpu
    job.fill_initial("random", 5)
    k = info["sweeps_per_round"]
    job.run(2 * k + 1)
    got = job.download()
    sums = job.plane_sums()
    job.close()
    if periodic:
        ref = SlabJob(spec, *shape, devices=[gpu], exchange="copy", periodic=True)
        ref.fill_initial("random", 5)
        ref.run(2 * k + 1)
        want = ref.download()
        want_sums = ref.plane_sums()
        ref.close()
    else:
        want = single_grid(gpu, spec, shape, 2 * k + 1, 5)
        e = JacobiEngine(spec, *shape, device=gpu)
        e.reset("random", 5)
        fin, _ = e.iterate(2 * k + 1)
        want_sums = e.plane_sums(fin)
    assert same_bits(got, want)
    assert np.array_equal(sums, want_sums)


def test_rank_mode_rejects_bad_requests(gpu):
    from stencil_amd import _lib
    spec = StencilSpec(dims=3, dtype="fp64")
    uid = SlabJob.unique_id()
    with pytest.raises(_lib.StencilError):
        SlabJob(spec, 32, 32, 20, devices=[gpu], rank=(2, 2, uid))  # rank out of range
    with pytest.raises(_lib.StencilError):
        SlabJob(spec, 32, 32, 20, devices=[gpu], rank=(1, 0, uid[:64]))  # not an RCCL id
    with pytest.raises(ValueError):
        SlabJob(spec, 32, 32, 20, devices=[gpu, gpu], rank=(1, 0, uid))  # one device per rank


@pytest.mark.skipif(_device_count() < 2, reason="needs 2 GPUs (RCCL refuses two ranks on one device)")
def test_bench_rank_mode_two_processes(gpu):
    """bench.py under torch.distributed.run, 2 ranks on 2 GPUs, through the
    C-ABI rank-mode job: the JSON line and its bitwise check against the
    global grid (runs only where >= 2 GPUs are visible)."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", "29587", os.path.join(root, "bench.py"),
                        "--gpus", "2", "--n", "128", "--steps", "16", "--warmup", "4"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert p.returncode == 0, p.stderr[-2000:]
    line = json.loads(p.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 2 and line["multi_gpu_check"]["bitwise_equal"], line
    assert "rank-mode" in line["config"]["parallelism"]


def _bench_line(argv, timeout=300):
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, os.path.join(root, "bench.py")] + argv, capture_output=True, text=True,
                       timeout=timeout, env=env)
    assert p.returncode == 0, p.stderr[-2000:]
    return json.loads(p.stdout.strip().splitlines()[-1])


def test_bench_rolling_slab_job_rehearsal(gpu):
    """bench.py --gpus 2 --rolling on, both slabs on GPU 0 (the NS4096 N = 2
    form at a scaled shape: ONE grid per slab plus a rolling margin, a pass of
    z-range launches then the exchange): bitwise the global grid."""
    line = _bench_line(["--gpus", "2", "--share-device", "--exchange", "copy", "--rolling", "on", "--n", "128",
                        "--steps", "16", "--warmup", "4"])
    assert line["multi_gpu_check"]["bitwise_equal"], line["multi_gpu_check"]
    assert line["config"]["rounds"] == "rolling passes"
    assert "rolling margin" in line["config"]["parallelism"] and line["config"]["slab_plan"]["rolling"]


@pytest.mark.parametrize("exchange", ["loopback", "nccl-self"])
def test_bench_interior_rank_rehearsal(gpu, exchange):
    """--exchange loopback / nccl-self: one periodic slab through the C-ABI
    (halos = its own faces by device copies / RCCL to itself), face-signalled
    rounds."""
    line = _bench_line(["--exchange", exchange, "--n", "128", "--steps", "16", "--warmup", "4"])
    assert line["n_gpus"] == 1 and line["value"] > 0
    assert line["config"]["rounds"] == "face-signalled launches"
    assert "periodic slab" in line["config"]["parallelism"]


@pytest.mark.parametrize("sweeps", [1, 6, 13])
def test_size_independent_plane_check(gpu, sweeps):
    """The multi-GPU check for global grids too large for one GPU (NS4096):
    every plane's sum from a (2t + 1)-plane grid equals the full grid's,
    bit for bit (the reference initial condition is z-uniform)."""
    import bench
    spec = StencilSpec(dims=3, dtype="fp64")
    grid = (96, 80, 70)
    full, how_full = bench.reference_plane_sums(spec, grid, sweeps, gpu)
    red, how_red = bench.reference_plane_sums(spec, grid, sweeps, gpu, force_reduced=True)
    assert how_full.startswith("the global grid") and how_red.startswith("size-independent")
    assert np.array_equal(full.view(np.uint64), red.view(np.uint64))
