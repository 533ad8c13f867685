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
    with pytest.raises(SystemExit, match="interior-rank rehearsal"):
        bench.slab_job_plan(args(gpus=2, exchange="loopback"), 8)


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


GB = 10 ** 9
BOX_FREE = int(308.6 * GB)  # what an MI355X box reports free (profiles/r03/r03a_hbm_capacity.txt)


def test_ns4096_refuses_one_gpu_with_the_reason():
    """The north star's own grid: ONE 4096^3 fp64 grid is 550 GB."""
    with pytest.raises(SystemExit, match=r"needs at least 2 GPUs: ONE 4096x4096x4096 fp64 grid is 55\d GB"):
        bench.slab_plan("NS4096", 1, BOX_FREE)


@pytest.mark.parametrize("n_gpus,rolling,planes", [(2, True, 2048), (4, False, 1024), (8, False, 512)])
def test_ns4096_plan_per_gpu_count(n_gpus, rolling, planes):
    """N = 2: one 278 GB slab grid per GPU, so ONE grid + a rolling margin;
    N = 4 / 8: two grids per slab fit beside the reserve."""
    plan = bench.slab_plan("NS4096", n_gpus, BOX_FREE)
    assert plan["grid"] == (4096, 4096, 4096) and plan["scaling"] == "strong"
    assert plan["planes_per_slab"] == planes
    assert plan["rolling"] == rolling
    if rolling:
        assert 150 <= plan["margin_estimate"] <= 512  # ~26 GB of spare 135 MB planes
        assert plan["grid_bytes_per_slab"] + plan["margin_estimate"] * plan["plane_bytes"] < BOX_FREE
    else:
        assert 2 * plan["grid_bytes_per_slab"] + bench.SLAB_RESERVE <= BOX_FREE


@pytest.mark.parametrize("n_gpus", [1, 2, 3, 4, 5, 6, 7, 8])
def test_every_config_plans_for_one_to_eight_gpus(n_gpus):
    for config in ("C2", "C3", "C4", "C5", "NS", "NS4096"):
        if config == "NS4096" and n_gpus == 1:
            continue
        plan = bench.slab_plan(config, n_gpus, BOX_FREE)
        gz = plan["grid"][2]
        assert sum(bench.partition(gz, n_gpus, r)[1] for r in range(n_gpus)) == gz
        per_gpu = plan["grid_bytes_per_slab"] * (1 if plan["rolling"] else 2)
        assert per_gpu < BOX_FREE, (config, n_gpus)
    assert bench.slab_plan("C2", n_gpus, BOX_FREE)["grid"] == (512, 512, 512 * n_gpus)
    assert not bench.slab_plan("C2", n_gpus, BOX_FREE)["rolling"]


def test_c3_at_two_gpus_rolls_only_if_two_grids_do_not_fit():
    plan = bench.slab_plan("C3", 2, BOX_FREE)
    assert plan["rolling"] == (2 * plan["grid_bytes_per_slab"] + bench.SLAB_RESERVE > BOX_FREE)
    assert bench.slab_plan("C3", 2, 200 * GB)["rolling"]
    assert bench.slab_plan("C3", 2, BOX_FREE, rolling="on")["rolling"]
    with pytest.raises(SystemExit, match="--rolling off"):
        bench.slab_plan("C3", 2, 200 * GB, rolling="off")


def test_partition_matches_the_slab_core_split():
    assert [bench.partition(10, 3, r) for r in range(3)] == [(0, 4), (4, 3), (7, 3)]
    assert [bench.partition(4096, 8, r)[1] for r in range(8)] == [512] * 8


def test_old_python_driver_flags_are_gone():
    """One implementation of the slab rounds (csrc/slab_core.hpp): the Python
    slab driver and its flags were retired in round 4."""
    for flag in ("--driver", "--face-signal", "--no-overlap"):
        with pytest.raises(SystemExit):
            bench.parse(["--gpus", "2", flag] + (["python"] if flag == "--driver" else []))
    assert not os.path.exists(os.path.join(ROOT, "stencil_amd", "slab.py"))


@pytest.mark.parametrize("argv,reason", [
    (["--rank-of", "2"], "needs --gpus 1 and --exchange loopback or nccl-self"),
    (["--rank-of", "1", "--exchange", "loopback"], "N >= 2"),
    (["--rank-of", "4", "--gpus", "2", "--exchange", "loopback"], "needs --gpus 1"),
])
def test_rank_of_needs_a_one_gpu_loopback_rehearsal(argv, reason):
    with pytest.raises(SystemExit, match=reason):
        bench.parse(["--config", "NS4096"] + argv)


def test_rank_of_parses_for_the_north_star():
    """`--config NS4096 --rank-of 2 --exchange loopback`: one rank's slab of the
    2-GPU job (4096^2 x 2048 planes, rolling as that plan says) on ONE GPU."""
    a = bench.parse(["--config", "NS4096", "--rank-of", "2", "--exchange", "loopback"])
    assert a.rank_of == 2 and a.gpus == 1
    plan = bench.slab_plan("NS4096", a.rank_of, BOX_FREE)
    assert plan["planes_per_slab"] == 2048 and plan["rolling"]
