#!/usr/bin/env python3
"""Interleaved A/B timing of experiment-knob variants in ONE process (the
debug library reads the knobs at every launch).

    python tools/ab.py --shape box --dtype fp64 --grid 2048 2048 256 --steps 4 \
        --variant STENCIL_BOXK_XCD=0 --variant STENCIL_BOXK_XCD=4 [--reps 5] [--launches 5]

Per rep and variant: `launches` back-to-back stencil_sweepk(steps) launches
(a -> b) timed with HIP events on the current stream; prints the best and
median ms per launch and Gcell/s, and checks every variant's output grid bit
for bit against the first variant's (same input, same sweeps)."""
import argparse
import os
import statistics
import sys

os.environ.setdefault("STENCIL_AB", "1")  # an experiment knob: the debug library loads
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="star", choices=["star", "box"])
    ap.add_argument("--dtype", default="fp64", choices=["fp32", "fp64"])
    ap.add_argument("--grid", type=int, nargs=3, default=[512, 512, 512])
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--variant", action="append", default=[],
                    help="NAME=VALUE[,NAME=VALUE]; STEPS=k overrides --steps for that variant, "
                         "INIT=random|reference its input grid (default random, seed 7), NOCHECK=1 skips its bitwise "
                         "check (a variant with another sum order)")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--launches", type=int, default=5)
    args = ap.parse_args()
    import torch
    from stencil_amd import _lib
    from stencil_amd.engine import JacobiEngine, StencilSpec
    variants = [dict(kv.split("=", 1) for kv in v.split(",")) for v in (args.variant or [""]) if v] or [{}]
    nx, ny, nz = args.grid
    e = JacobiEngine(StencilSpec(dims=3, dtype=args.dtype, shape=args.shape), nx, ny, nz)
    assert e.lib.stencil_debug_knobs() == 1, "experiment knobs need the debug library"
    e.reset("random", 7)
    times = [[] for _ in variants]

    def setenv(v):
        for v2 in variants:
            for k in v2:
                os.environ.pop(k, None)
        os.environ.update({k: x for k, x in v.items() if k not in ("STEPS", "INIT", "NOCHECK")})
        init = v.get("INIT", "random")
        if init != state["init"]:  # the variant's input grid (a; b is overwritten)
            e.reset(init, 7)
            state["init"] = init

    def steps(v):
        return int(v.get("STEPS", args.steps))

    state = {"init": "random"}
    refs = {}
    for vi, v in enumerate(variants):  # warm-up + check against the first variant of the same step count
        setenv(v)
        e.sweepk(e.a, e.b, 0, nz, steps(v))
        torch.cuda.synchronize()
        out = e.interior(e.b).clone()
        k = (steps(v), state["init"])
        if v.get("NOCHECK"):
            print(f"variant {v}: not checked (another sum order)", flush=True)
        elif k not in refs:
            refs[k] = (v, out)
        else:
            it = torch.int64 if args.dtype == "fp64" else torch.int32
            same = torch.equal(out.view(it), refs[k][1].view(it))
            print(f"variant {v}: bitwise equal to {refs[k][0] or 'default'}: {same}", flush=True)
            if not same:
                raise SystemExit(1)
        del out  # only the first output of each step count is kept (wide grids: one interior is 64 GB)
        torch.cuda.empty_cache()
    del refs
    torch.cuda.empty_cache()
    for _ in range(args.reps):
        for vi, v in enumerate(variants):
            setenv(v)
            s = torch.cuda.current_stream()
            t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0.record(s)
            for _ in range(args.launches):
                e.sweepk(e.a, e.b, 0, nz, steps(v))
            t1.record(s)
            t1.synchronize()
            times[vi].append(t0.elapsed_time(t1) / args.launches)
    for v, t in zip(variants, times):
        cells = float(nx) * ny * nz * steps(v)
        print(f"{args.shape} {args.dtype} {nx}x{ny}x{nz} K={steps(v)} {v or 'default'}: "
              f"best {min(t):.4f} ms, median {statistics.median(t):.4f} ms per launch, "
              f"{cells / min(t) / 1e6:.1f} Gcell/s (best)", flush=True)


if __name__ == "__main__":
    main()
