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
