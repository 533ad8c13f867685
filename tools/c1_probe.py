#!/usr/bin/env python3
"""Where C1's wall time goes (BASELINE config 1: 2D 5-point 1024^2 fp64,
100 sweeps = 10 tb2ds launches of K = 10).

    python tools/c1_probe.py [--reps 30]

Prints, as medians over --reps runs of the whole 100-sweep job:
  eager   -- stencil_iterate on the current stream (what bench.py times):
             host wall, device time between its events;
  graph   -- the same job captured once into a HIP graph and replayed;
  floor   -- an empty sync and a one-launch job, the fixed submit/wait cost.
Under `rocprofv3 --kernel-trace` the trace gives the inter-launch gaps."""
import argparse
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from stencil_amd.engine import JacobiEngine, StencilSpec


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--sweeps", type=int, default=100)
    a = ap.parse_args()
    torch.cuda.set_device(0)
    e = JacobiEngine(StencilSpec(dims=2, dtype="fp64"), 1024, 1024, 1, device=0)
    e.reset("reference", 1)
    e.prepare()
    s = torch.cuda.current_stream()
    print("plan", e.plan(a.sweeps))

    def run_eager():
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        _, ms = e.iterate(a.sweeps, stream=s, timed=True)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e3, ms

    for _ in range(5):
        run_eager()
    eager = [run_eager() for _ in range(a.reps)]
    w = statistics.median(x[0] for x in eager)
    d = statistics.median(x[1] for x in eager)
    print(f"eager: wall {w * 1e3:.1f} us, device {d * 1e3:.1f} us per {a.sweeps} sweeps "
          f"-> {1024 * 1024 * a.sweeps / w / 1e6:.1f} Gcell/s wall, {1024 * 1024 * a.sweeps / d / 1e6:.1f} device")

    # the same job as one graph (an even sweep count ends where it started, so replays chain)
    side = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    side.wait_stream(s)
    with torch.cuda.stream(side):
        e.iterate(a.sweeps, stream=side)  # the schedule choices happen outside the capture
    s.wait_stream(side)
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        e.iterate(a.sweeps, stream=torch.cuda.current_stream())
    torch.cuda.synchronize()

    def run_graph():
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        g.replay()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e3

    for _ in range(5):
        run_graph()
    gw = statistics.median(run_graph() for _ in range(a.reps))
    print(f"graph: wall {gw * 1e3:.1f} us per {a.sweeps} sweeps -> {1024 * 1024 * a.sweeps / gw / 1e6:.1f} Gcell/s")

    def empty():
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e3

    def one_launch():
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e.iterate(10, stream=s)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e3

    ew = statistics.median(empty() for _ in range(a.reps))
    ow = statistics.median(one_launch() for _ in range(a.reps))
    print(f"floor: empty sync {ew * 1e3:.1f} us, one 10-sweep launch {ow * 1e3:.1f} us wall")


if __name__ == "__main__":
    main()
