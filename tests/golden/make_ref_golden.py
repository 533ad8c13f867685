#!/usr/bin/env python3
"""Golden vectors from the REFERENCE's own code (TEST INFRASTRUCTURE ONLY).

Runs oracle/_ref/ref_naive -- the reference's naive loop
(src/stencil/stencil.cpp:77-131) and initial condition (190-207) compiled from
/root/reference by oracle/ref/build.sh, in this container only -- and stores
what it prints:
  tests/golden/ref_fixtures.npz       full final interiors of the small cases
  tests/golden/ref_known_answers.json sha256 of the interior bytes (and the
                                      sum) of every case, the large ones too
tests/test_oracle_golden.py checks the oracle (oracle/) against both, bit for
bit; tests/test_gpu_parity.py checks the HIP kernels against the fixtures.
fp64 cases run the same loop with float -> double (see oracle/ref/mid2.inc).

usage: bash oracle/ref/build.sh && python tests/golden/make_ref_golden.py"""
import hashlib
import json
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
BIN = os.path.join(ROOT, "oracle", "_ref", "ref_naive")

# (n, iterations, radius): SURVEY §8c's five configurations (C1 = 1024/100),
# plus odd/even counts, zero iterations and radii 2 and 4
CASES = [(32, 3, 1), (64, 100, 1), (400, 1000, 1), (96, 50, 3), (1024, 100, 1),
         (33, 7, 1), (50, 20, 2), (40, 9, 4), (16, 0, 1), (8, 1, 1)]
FULL_MAX_N = 96  # interiors stored whole up to this size


def run(n, it, r, dt):
    out = subprocess.run([BIN, str(n), str(it), str(r), dt], check=True, capture_output=True).stdout
    a = np.frombuffer(out, dtype=np.float32 if dt == "f32" else np.float64)
    assert a.size == n * n, (n, a.size)
    return a.reshape(n, n)


def main():
    fixtures, answers = {}, []
    for n, it, r in CASES:
        for dt in ("f32", "f64"):
            a = run(n, it, r, dt)
            name = f"n{n}_i{it}_r{r}_{dt}"
            answers.append({"name": name, "n": n, "iterations": it, "radius": r, "dtype": dt,
                            "sha256": hashlib.sha256(a.tobytes()).hexdigest(),
                            "sum": float(a.astype(np.float64).sum())})
            if n <= FULL_MAX_N:
                fixtures[name] = a
    np.savez_compressed(os.path.join(HERE, "ref_fixtures.npz"), **fixtures)
    meta = {"_source": "oracle/_ref/ref_naive: the reference's Stencil::check_result loop (stencil.cpp:77-131) and "
                       "generate_initialized_matrix (stencil.cpp:190-207) compiled from /root/reference with its real "
                       "headers by oracle/ref/build.sh; fp64 = the same lines with float -> double. Interior bytes, "
                       "row-major, after `iterations` sweeps.",
            "cases": answers}
    with open(os.path.join(HERE, "ref_known_answers.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print(f"{len(answers)} cases, {len(fixtures)} stored whole")


if __name__ == "__main__":
    main()
