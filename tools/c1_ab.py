#!/usr/bin/env python3
"""Interleaved A/B of 2D region variants at C1 (1024^2, 100 sweeps) in ONE
process (debug library; STENCIL_TB2D_CFG is read at every launch).

    python tools/c1_ab.py --dtype fp64 --variant 0 --variant 192416 [--reps 20]

Per rep and variant: one whole 100-sweep stencil_iterate from the same
input, device ms from its HIP events; prints best / median ms and Gcell/s,
and checks each variant's result bit for bit against the first's."""
import argparse
import os
import statistics
import sys

os.environ.setdefault("STENCIL_AB", "1")  # an experiment knob: the debug library loads
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="fp64", choices=["fp32", "fp64"])
    ap.add_argument("--order", default="naive", choices=["naive", "dma"])
    ap.add_argument("--n", type=int, default=1024)
    ap.add_argument("--sweeps", type=int, default=100)
    ap.add_argument("--variant", action="append", default=[])
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    import torch
    from stencil_amd.engine import JacobiEngine, StencilSpec
    e = JacobiEngine(StencilSpec(dims=2, dtype=a.dtype, order=a.order), a.n, a.n, 1, device=0)
    assert e.lib.stencil_debug_knobs() == 1, "experiment knobs need the debug library"
    variants = a.variant or ["0"]
    e.reset("random", 7)
    e.prepare()
    times = {v: [] for v in variants}
    first = None
    for rep in range(a.reps + 2):
        for v in variants:
            os.environ["STENCIL_TB2D_CFG"] = v
            e.reset("random", 7)
            torch.cuda.synchronize()
            fin, ms = e.iterate(a.sweeps, timed=True)
            torch.cuda.synchronize()
            if rep >= 2:
                times[v].append(ms)
            if rep == 0:
                got = e.to_numpy(fin).copy()
                if first is None:
                    first = got
                else:
                    assert (got.view("u1") == first.view("u1")).all(), f"variant {v} differs from {variants[0]}"
    cells = a.n * a.n * a.sweeps
    print(f"C1 A/B {a.dtype} {a.order} {a.n}^2 x {a.sweeps}: results bitwise equal")
    for v in variants:
        b, m = min(times[v]), statistics.median(times[v])
        print(f"  cfg {v:>7}: best {b * 1e3:8.1f} us  median {m * 1e3:8.1f} us  -> {cells / m / 1e6:7.1f} Gcell/s (median)")


if __name__ == "__main__":
    main()
