"""bench.py's launch logic, on the CPU: the single-process multi-GPU path
(--gpus N without a launcher drives N GPUs through the C-ABI slab job) picks
its devices and exchange, or refuses with the reason."""
import argparse
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def args(**kw):
    base = dict(gpus=2, exchange="nccl", share_device=False)
    base.update(kw)
    return argparse.Namespace(**base)


def test_slab_job_one_gpu_per_slab_over_rccl():
    assert bench.slab_job_plan(args(gpus=8), 8) == (list(range(8)), "rccl")
    assert bench.slab_job_plan(args(gpus=4, exchange="copy"), 8) == ([0, 1, 2, 3], "copy")


def test_slab_job_refuses_too_few_gpus():
    with pytest.raises(SystemExit, match="--gpus 2 needs 2 GPUs, 1 visible"):
        bench.slab_job_plan(args(gpus=2), 1)


def test_slab_job_shared_device_rehearsal():
    assert bench.slab_job_plan(args(gpus=3, exchange="copy", share_device=True), 1) == ([0, 0, 0], "copy")
    with pytest.raises(SystemExit, match="needs --exchange copy"):
        bench.slab_job_plan(args(gpus=2, share_device=True), 1)
    with pytest.raises(SystemExit, match="torch.distributed rehearsal"):
        bench.slab_job_plan(args(gpus=2, exchange="host"), 8)


def test_c3_c4_run_on_one_gpu():
    assert bench.PRESETS["C3"]["min_gpus"] == 1  # one resident grid + a rolling margin
    assert bench.PRESETS["C4"]["min_gpus"] == 1


def test_bench_gpus_2_without_launcher_fails_clearly_without_gpus():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["HIP_VISIBLE_DEVICES"] = ""  # no device here (and none on the box for this check)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "4"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert p.returncode != 0
    assert "--gpus 2 needs 2 GPUs, 0 visible" in p.stderr


def rank_args(**kw):
    base = dict(gpus=2, exchange="nccl", share_device=False, driver="auto", no_signal=False, face_signal=False,
                no_overlap=False)
    base.update(kw)
    return argparse.Namespace(**base)


def test_torchrun_uses_the_cabi_rank_job_by_default():
    """Under torch.distributed.run (N > 1) the default driver is the C-ABI
    rank-mode slab job; one rank, --driver python and the rehearsal
    transports keep the Python slab driver."""
    assert bench.rank_job_wanted(rank_args(), 2)
    assert bench.rank_job_wanted(rank_args(driver="cabi"), 8)
    assert not bench.rank_job_wanted(rank_args(), 1)
    assert not bench.rank_job_wanted(rank_args(driver="python"), 2)
    assert not bench.rank_job_wanted(rank_args(exchange="host", share_device=True), 2)
    assert not bench.rank_job_wanted(rank_args(no_signal=True), 2)


def test_cabi_driver_refuses_rehearsal_transports():
    with pytest.raises(SystemExit, match="--driver cabi"):
        bench.rank_job_wanted(rank_args(driver="cabi", exchange="host"), 2)
    with pytest.raises(SystemExit, match="--driver cabi"):
        bench.rank_job_wanted(rank_args(driver="cabi", face_signal=True), 2)
