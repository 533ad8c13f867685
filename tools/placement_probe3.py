#!/usr/bin/env python3
"""Is the speed of a placement a function of allocation order?  Allocates
`pairs` grid pairs one after another (all held), times one fused launch on
each in `passes` interleaved passes, then frees the first half and allocates
as many new pairs (which may reuse those pages) and times everything again.

    python tools/placement_probe3.py [--grid 512 512 512] [--dtype fp64] [--pairs 8]"""
import argparse
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grid", type=int, nargs=3, default=[512, 512, 512])
    ap.add_argument("--dtype", default="fp64", choices=["fp32", "fp64"])
    ap.add_argument("--pairs", type=int, default=8)
    ap.add_argument("--passes", type=int, default=3)
    args = ap.parse_args()
    import torch
    from stencil_amd import _lib
    from stencil_amd.engine import JacobiEngine, StencilSpec, _stream_handle
    torch.cuda.set_device(0)
    nx, ny, nz = args.grid
    eng = JacobiEngine(StencilSpec(dims=3, dtype=args.dtype), nx, ny, nz, device=0, allocate=False)
    lib, lay, k = eng.lib, eng.layout, eng.fuse_steps
    n = int(lay.elems) + 64
    dt = torch.float64 if args.dtype == "fp64" else torch.float32
    s = _stream_handle(None)
    fin, ms = ctypes.c_int(0), ctypes.c_float(0.0)

    def run(a, b, timed):
        _lib.check(lib.stencil_iterate(ctypes.byref(lay), ctypes.c_void_p(a.data_ptr()), ctypes.c_void_p(b.data_ptr()),
                                       k, s, ctypes.byref(fin), ctypes.byref(ms) if timed else None), "iterate", lib=lib)
        return ms.value

    def new_pair():
        a, b = torch.empty(n, dtype=dt, device="cuda"), torch.empty(n, dtype=dt, device="cuda")
        for g in (a, b):
            _lib.check(lib.stencil_fill_initial(ctypes.byref(lay), ctypes.c_void_p(g.data_ptr()), _lib.INIT_REFERENCE,
                                                ctypes.c_uint64(0), s), "fill", lib=lib)
        return a, b

    def survey(tag, pairs):
        for _ in range(8):
            run(*pairs[0][1], False)
        best = {i: 1e9 for i, _ in pairs}
        for _ in range(args.passes):
            for i, (a, b) in pairs:
                run(a, b, False)
                best[i] = min(best[i], run(a, b, True), run(a, b, True))
        print(tag + ": " + "  ".join(f"#{i} {best[i]:.4f}" for i, _ in pairs), flush=True)

    pairs = [(i, new_pair()) for i in range(args.pairs)]
    survey("allocated in order", pairs)
    half = args.pairs // 2
    del pairs[:half]
    torch.cuda.synchronize()
    pairs += [(args.pairs + i, new_pair()) for i in range(half)]
    survey("first half freed, re-allocated", pairs)
    torch.cuda.empty_cache()
    pairs += [(2 * args.pairs + i, new_pair()) for i in range(2)]
    survey("two more after empty_cache", pairs)


if __name__ == "__main__":
    main()
