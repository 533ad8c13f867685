"""Regenerate tests/golden/oracle_fixtures.npz from the CPU oracle.

The fixtures freeze the oracle's outputs on small cases (inputs are the
deterministic reference initial condition or splitmix64 random interiors, so
only outputs are stored).  tests/test_oracle_golden.py checks the oracle still
reproduces them and the GPU tests compare the HIP kernels against them.
Run:  python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import binding as ob  # noqa: E402

CASES = [
    # name, dims, dtype, shape, radius, order, nx, ny, nz, iterations, init, seed
    ("2d_r1_f32_naive_17x13", 2, "fp32", "star", 1, "naive", 17, 13, 1, 7, "reference", 0),
    ("2d_r1_f32_dma_17x13", 2, "fp32", "star", 1, "dma", 17, 13, 1, 7, "reference", 0),
    ("2d_r2_f32_dma_rand_20x9", 2, "fp32", "star", 2, "dma", 20, 9, 1, 5, "random", 7),
    ("2d_r3_f64_naive_rand_33x31", 2, "fp64", "star", 3, "naive", 33, 31, 1, 4, "random", 11),
    ("3d_r1_f64_star_rand_9x7x5", 3, "fp64", "star", 1, "naive", 9, 7, 5, 3, "random", 3),
    ("3d_r1_f32_star_70x19x6", 3, "fp32", "star", 1, "naive", 70, 19, 6, 6, "random", 5),
    ("3d_r1_f64_box_rand_10x6x7", 3, "fp64", "box", 1, "naive", 10, 6, 7, 3, "random", 9),
    ("3d_r2_f64_star_rand_12x11x10", 3, "fp64", "star", 2, "naive", 12, 11, 10, 2, "random", 13),
]


def main():
    out = {}
    for name, dims, dtype, shape, r, order, nx, ny, nz, it, init, seed in CASES:
        p = ob.problem(dims, dtype, shape, r, order, nx, ny, nz)
        g = ob.run(p, it, init, seed)
        out[name] = np.ascontiguousarray(ob.interior(p, g))
        out[name + "__meta"] = np.array([dims, 1 if dtype == "fp64" else 0, 1 if shape == "box" else 0, r,
                                         1 if order == "dma" else 0, nx, ny, nz, it, 1 if init == "random" else 0,
                                         seed], dtype=np.int64)
    np.savez_compressed(os.path.join(os.path.dirname(os.path.abspath(__file__)), "oracle_fixtures.npz"), **out)
    print("wrote", len(CASES), "fixtures")


if __name__ == "__main__":
    main()
