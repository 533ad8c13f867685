"""The drop-in CLI (build/bin/stencil_main) keeps the reference's surface
(src/program_options.cpp:13-44, src/main.cpp:53-62).  Parsing only -- no GPU."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, "build", "bin", "stencil_main")


def run(*args):
    return subprocess.run([CLI, *args], capture_output=True, text=True, timeout=60)


def cfg(*args):
    p = run(*args, "--print-config")
    assert p.returncode == 0, p.stderr
    return dict(kv.split("=", 1) for kv in p.stdout.split())


def test_cli_built():
    assert os.access(CLI, os.X_OK)


def test_reference_invocation_parses():
    c = cfg("-s", "1024", "-b", "128", "-i", "100", "-r", "1", "-m", "DMA", "DMAStaticUnroll", "-c")
    assert c["matrix_size"] == "1024" and c["block_size"] == "128" and c["iterations"] == "100"
    assert c["methods"] == "DMA,DMAStaticUnroll" and c["check"] == "1" and c["repeat"] == "1"
    assert c["dims"] == "2" and c["dtype"] == "fp32" and c["nz"] == "1"


def test_long_and_attached_forms():
    c = cfg("--matrix-size=64", "-b8", "--iteration", "3", "--radius=2", "-R", "4", "--methods=RMA", "-m", "HIP")
    assert (c["matrix_size"], c["block_size"], c["iterations"], c["radius"], c["repeat"]) == ("64", "8", "3", "2", "4")
    assert c["methods"] == "RMA,HIP"


def test_extensions():
    c = cfg("-s", "512", "-b", "1", "-i", "1000", "-m", "HIP", "--points", "7", "--dtype", "fp64", "--kernel", "zmarch")
    assert (c["dims"], c["nz"], c["dtype"], c["kernel"], c["shape"]) == ("3", "512", "fp64", "zmarch", "star")
    c = cfg("-s", "16", "-b", "1", "-i", "2", "-m", "HIP", "--points", "27", "--nx", "20", "--nz", "3")
    assert (c["dims"], c["shape"], c["nx"], c["ny"], c["nz"]) == ("3", "box", "20", "16", "3")
    c = cfg("-s", "16", "-b", "1", "-i", "2", "-m", "HIPMultiGPU", "--points", "7", "--gpus", "8")
    assert (c["gpus"], c["exchange"], c["methods"]) == ("8", "rccl", "HIPMultiGPU")
    c = cfg("-s", "16", "-b", "1", "-i", "2", "-m", "HIP", "--gpus=3", "--exchange", "copy", "--share-device")
    assert (c["gpus"], c["exchange"]) == ("3", "copy")


@pytest.mark.parametrize("args", [
    [],                                                     # all required missing
    ["-s", "64", "-i", "3", "-m", "DMA"],                   # -b missing
    ["-s", "64", "-b", "8", "-i", "3"],                     # -m missing
    ["-s", "64", "-b", "8", "-i", "3", "-m", "DMA", "-w", "1"],  # run_expr.py's stale -w
    ["-s", "-5", "-b", "8", "-i", "3", "-m", "DMA"],        # negative unsigned
    ["-s", "abc", "-b", "8", "-i", "3", "-m", "DMA"],
    ["-s", "64", "-b", "8", "-i", "3", "-m"],                # -m needs a value
    ["-s", "64", "-b", "8", "-i", "3", "-m", "DMA", "stray", "--dims", "4"],
    ["--help"],                                             # parse() returns nullopt after help
    ["-s", "64", "-b", "8", "-i", "3", "-m", "HIP", "--gpus", "0"],
    ["-s", "64", "-b", "8", "-i", "3", "-m", "HIP", "--exchange", "mpi"],
])
def test_parse_failures_exit_1(args):
    p = run(*args)
    assert p.returncode == 1


def test_help_lists_reference_flags():
    out = run("--help").stdout
    for flag in ("-s,--matrix-size", "-i,--iteration", "-b,--block-size", "-r,--radius", "-R,--repeat",
                 "-m,--methods", "-c,--check-result"):
        assert flag in out


def test_cli_cpu_method_runs_on_the_host():
    """The CPU method (the reference's check_result loop, timed like a
    method): the reference's stdout lines, -c passes, no GPU."""
    import re
    p = subprocess.run([CLI, "-s", "64", "-b", "8", "-i", "10", "-r", "1", "-m", "CPU", "-c"], capture_output=True,
                       text=True, timeout=120)
    assert p.returncode == 0, p.stderr
    assert "The results of method CPU is correct." in p.stdout
    assert re.search(r"The average time taken by (.*) method is (.*)ms for \d+ iterations\.", p.stdout).group(1) == "CPU"
    assert "[stencil-amd] CPU: host" in p.stdout
