#!/usr/bin/env python3
"""Host overhead of a short timed region (the driver's 20-step bench): wall
time of stencil_iterate between two torch.cuda.synchronize() calls against
the device time its events see, with and without the events, and with the
timed region's first launch preceded by an idle gap or not.

    python tools/overhead_probe.py [--steps 20] [--reps 7]"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--reps", type=int, default=7)
    args = ap.parse_args()
    import torch
    from stencil_amd.engine import JacobiEngine, StencilSpec
    torch.cuda.set_device(0)
    eng = JacobiEngine(StencilSpec(dims=3, dtype="fp64"), 512, 512, 512, device=0)
    eng.reset("reference")
    eng.prepare()
    s = torch.cuda.current_stream()
    for mode in ("timed", "untimed", "timed", "untimed"):
        walls, devs = [], []
        for _ in range(args.reps):
            eng.iterate(4, stream=s)  # keep the clock up
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            _, ms = eng.iterate(args.steps, stream=s, timed=(mode == "timed"))
            torch.cuda.synchronize()
            walls.append((time.perf_counter() - t0) * 1e3)
            if ms is not None:
                devs.append(ms)
        walls.sort()
        line = f"{mode:8s} steps {args.steps}: wall ms median {walls[len(walls) // 2]:.4f} min {walls[0]:.4f}"
        if devs:
            devs.sort()
            line += f"; events ms median {devs[len(devs) // 2]:.4f}; wall - events {walls[len(walls) // 2] - devs[len(devs) // 2]:.4f}"
        print(line, flush=True)
    # the launch path alone: host time to enqueue the job (no sync)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    eng.iterate(args.steps, stream=s)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    print(f"enqueue only: {(t1 - t0) * 1e3:.4f} ms host for {args.steps} steps", flush=True)


if __name__ == "__main__":
    main()
