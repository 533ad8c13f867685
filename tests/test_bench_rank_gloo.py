"""bench.py's N > 1 path on the CPU: world 2 and 3 over gloo.

Under torch.distributed.run every rank runs bench.main_rank_job: rank 0's
RCCL id broadcast over a gloo group, each rank's own C-ABI slab
(stencil_slab_create_rank), warm-up, the timed rounds, the max-over-ranks
time, the kernel-timing rounds and the per-plane sums gathered on rank 0.
Here each rank is a separate process (torch.multiprocessing, gloo on
127.0.0.1) and its slab runs on the CPU fake device of tests/cpu_slab -- the
same csrc/slab_core.hpp rounds, oracle sweeps, halos through a file mailbox
(FAKE_SLAB_MAILBOX_DIR).  The gathered per-plane sums must equal, bit for
bit, those of the same job run as ONE slab.
"""
import json
import os
import socket
import time
import tempfile

import numpy as np
import pytest
import torch.multiprocessing as mp

import bench
from stencil_amd.engine import SlabJob, StencilSpec
from tests.cpu_slab import binding as fb

pytestmark = pytest.mark.skipif(not fb.available(), reason="tests/cpu_slab/libslab_fake.so not built (run make)")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _rank_main(rank, world, port, mail, argv, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0", FAKE_SLAB_MAILBOX_DIR=mail)
    fake = fb.load()
    fake.set_k(0)
    args = bench.parse(argv)
    line, got, res = bench.main_rank_job(args, world, rank, 0, lib=fake)
    if rank == 0:
        with open(os.path.join(out_dir, "line.json"), "w") as f:
            json.dump(line, f)
        np.save(os.path.join(out_dir, "got.npy"), got)
        np.save(os.path.join(out_dir, "meta.npy"), np.array([res["sweeps"], line["value"] > 0,
                                                             line["n_gpus"], res["k"]], dtype=np.float64))


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("config,extra", [("C2", ["--n", "20"]), ("C2", ["--n", "20", "--no-signal"]),
                                          ("C2", ["--n", "20", "--rolling", "on"])])
def test_bench_rank_job_world_gloo(world, config, extra):
    argv = ["--gpus", str(world), "--config", config, "--steps", "9", "--warmup", "2"] + extra
    with tempfile.TemporaryDirectory() as tmp:
        mail = os.path.join(tmp, "mail")
        os.makedirs(mail)
        ctx = mp.get_context("spawn")
        port = _free_port()
        procs = [ctx.Process(target=_rank_main, args=(r, world, port, mail, argv, tmp)) for r in range(world)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(240)
        codes = [p.exitcode for p in procs]
        for p in procs:
            if p.is_alive():
                p.kill()
        assert codes == [0] * world, codes
        got = np.load(os.path.join(tmp, "got.npy"))
        sweeps, ok, n_gpus, k = np.load(os.path.join(tmp, "meta.npy"))
        assert ok and int(n_gpus) == world
        leftovers = os.listdir(mail)
        assert all(f.startswith("join_") for f in leftovers), leftovers  # every halo message was received
        line = json.load(open(os.path.join(tmp, "line.json")))
        # what ran before the timed region is on the line
        cfg = line["config"]
        assert cfg["settle_launches"] >= 1 and cfg["settle_ms"] >= 0 and "settle" in cfg
        assert "effective_GBps_whole_job" in cfg and "achieved_hbm_GBps_whole_job" not in cfg
        # every rank's exchange of the timed rounds is on the line: one per timed round
        ex = line["exchange"]
        assert len(ex["per_rank"]) == world, ex
        assert all(r["rounds"] == line["roofline"]["launches"] for r in ex["per_rank"]), ex
        assert ex["max_transfer_ms_per_round"] >= 0
    # the same sweeps on ONE slab (no exchange), the fake device's plane sums
    fake = fb.load()
    fake.set_k(0)
    n = 20
    spec = StencilSpec(dims=3, dtype="fp64", shape="star")
    job = SlabJob(spec, n, n, n * world, [0], exchange="rccl", lib=fake)
    job.fill_initial("reference")
    job.run(int(sweeps))
    want = job.plane_sums()
    job.close()
    assert int(k) == 4
    assert np.array_equal(got.view(np.uint64), want.view(np.uint64))


def _silent_rank_main(rank, world, port, mail, argv, muted):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0", FAKE_SLAB_MAILBOX_DIR=mail, FAKE_SLAB_MUTE_RANK=str(muted),
                      FAKE_SLAB_MUTE_AFTER="2")  # after the fill's two exchanges
    fake = fb.load()
    fake.set_k(0)
    bench.main_rank_job(bench.parse(argv), world, rank, 0, lib=fake)


@pytest.mark.parametrize("world", [2, 3])
def test_bench_rank_job_exits_nonzero_when_a_peer_goes_silent(world):
    """VERDICT r04 missing #3: one rank stops posting its halo sends after
    the fill; every rank's job fails with STENCIL_ETIMEOUT within the
    deadline (--slab-timeout-ms), bench.py raises, and every process exits
    non-zero -- no rank is left waiting until the driver kills the job."""
    argv = ["--gpus", str(world), "--config", "C2", "--n", "12", "--steps", "40", "--warmup", "2",
            "--slab-timeout-ms", "1500"]
    with tempfile.TemporaryDirectory() as tmp:
        mail = os.path.join(tmp, "mail")
        os.makedirs(mail)
        ctx = mp.get_context("spawn")
        port = _free_port()
        procs = [ctx.Process(target=_silent_rank_main, args=(r, world, port, mail, argv, world - 1))
                 for r in range(world)]
        t0 = time.monotonic()
        for p in procs:
            p.start()
        for p in procs:
            p.join(120)
        took = time.monotonic() - t0
        codes = [p.exitcode for p in procs]
        for p in procs:
            if p.is_alive():
                p.kill()
    assert all(c is not None and c != 0 for c in codes), codes
    assert took < 90, took  # process start-up (spawn + torch import) dominates; the deadline is 1.5 s
