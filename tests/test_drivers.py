"""run_expr.py keeps the reference sweep's regex and CSV surface
(run_expr.py:9,26-43); exercised against a stub binary (no GPU)."""
import csv
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_run_expr_csv(tmp_path):
    stub = tmp_path / "stencil_main"
    stub.write_text("#!/bin/bash\n"
                    "# echo the reference's stdout lines for every -m method\n"
                    "it=0; ms=(); while [ $# -gt 0 ]; do case $1 in -i) it=$2; shift 2;; -m) shift; "
                    "while [ $# -gt 0 ] && [[ $1 != -* ]]; do ms+=($1); shift; done;; *) shift;; esac; done\n"
                    "for m in ${ms[@]}; do echo \"$m Method spent 1.5ms for $it iterations.\"; "
                    "echo \"The average time taken by $m method is 1.23456ms for $it iterations.\"; done\n")
    stub.chmod(0o755)
    out = tmp_path / "out.csv"
    subprocess.run([sys.executable, os.path.join(ROOT, "run_expr.py"), "--binary", str(stub), "--block-sizes", "8",
                    "16", "--iterations", "1", "10", "--methods", "DMA", "HIP", "--out", str(out)], check=True,
                   capture_output=True, text=True)
    rows = list(csv.DictReader(open(out)))
    assert [r["Block Size"] for r in rows] == ["8", "8", "16", "16"]
    assert [r["Iteration"] for r in rows] == ["1", "10", "1", "10"]
    assert all(r["DMA"] == "1.235" and r["HIP"] == "1.235" for r in rows)
    assert list(rows[0].keys()) == ["Block Size", "Iteration", "DMA", "HIP"]


def test_run_sh_uses_current_flags():
    txt = open(os.path.join(ROOT, "run.sh")).read()
    assert "-s 400 -b 50 -i 1000 -r 1" in txt and "bsub" not in txt.split("\n", 5)[-1]


def test_run_expr_cpu_method_bounded(tmp_path):
    """CPU (the reference's naive loop, timed as a method) sits in the sweep's
    default methods, dropped past --cpu-max-iterations."""
    stub = tmp_path / "stencil_main"
    stub.write_text("#!/bin/bash\n"
                    "it=0; ms=(); while [ $# -gt 0 ]; do case $1 in -i) it=$2; shift 2;; -m) shift; "
                    "while [ $# -gt 0 ] && [[ $1 != -* ]]; do ms+=($1); shift; done;; *) shift;; esac; done\n"
                    "for m in ${ms[@]}; do echo \"The average time taken by $m method is 2ms for $it iterations.\"; "
                    "done\n")
    stub.chmod(0o755)
    out = tmp_path / "out.csv"
    subprocess.run([sys.executable, os.path.join(ROOT, "run_expr.py"), "--binary", str(stub), "--block-sizes", "8",
                    "--iterations", "10", "5000", "--out", str(out)], check=True, capture_output=True, text=True)
    rows = list(csv.DictReader(open(out)))
    assert rows[0]["CPU"] == "2.000" and rows[0]["HIP"] == "2.000"
    assert rows[1].get("CPU") in (None, "")  # 5000 > 1000 iterations: not run


def test_run_sh_prints_the_cpu_path():
    txt = open(os.path.join(ROOT, "run.sh")).read()
    assert "HIP CPU" in txt
