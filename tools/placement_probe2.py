#!/usr/bin/env python3
"""The two grids of a job in ONE allocation, b placed `delta` bytes after
the end of a (rounded up to 2 MiB): is the strip launch's speed a function of
the grids' relative placement?  hipExtMallocWithFlags(contiguous) makes the
physical offset the virtual one; hipMalloc (default) maps 2 MiB fragments
wherever they land.

    python tools/placement_probe2.py [--grid 4096 4096 256] [--dtype fp32]"""
import argparse
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grid", type=int, nargs=3, default=[4096, 4096, 256])
    ap.add_argument("--dtype", default="fp32", choices=["fp32", "fp64"])
    ap.add_argument("--deltas", default="0,256,4096,65536,1048576,2097152,3145728,8388608,33554432")
    ap.add_argument("--modes", default="contiguous,default")
    args = ap.parse_args()
    import torch
    from stencil_amd import _lib
    from stencil_amd.engine import JacobiEngine, StencilSpec, _stream_handle
    torch.cuda.set_device(0)
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
    hip.hipExtMallocWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
    hip.hipFree.argtypes = [ctypes.c_void_p]
    nx, ny, nz = args.grid
    eng = JacobiEngine(StencilSpec(dims=3, dtype=args.dtype), nx, ny, nz, device=0, allocate=False)
    lib, lay = eng.lib, eng.layout
    nbytes = int(lay.elems) * (4 if args.dtype == "fp32" else 8) + 256
    span = (nbytes + (2 << 20) - 1) // (2 << 20) * (2 << 20)
    deltas = [int(d) for d in args.deltas.split(",")]
    k = eng.fuse_steps
    cells = nx * ny * nz
    s = _stream_handle(None)

    def timed(a, b):
        for g in (a, b):
            _lib.check(lib.stencil_fill_initial(ctypes.byref(lay), ctypes.c_void_p(g), _lib.INIT_REFERENCE,
                                                ctypes.c_uint64(0), s), "fill", lib=lib)
        fin, ms = ctypes.c_int(0), ctypes.c_float(0.0)
        lib.stencil_iterate(ctypes.byref(lay), ctypes.c_void_p(a), ctypes.c_void_p(b), 4 * k, s, ctypes.byref(fin), None)
        best = None
        for _ in range(3):
            _lib.check(lib.stencil_iterate(ctypes.byref(lay), ctypes.c_void_p(a), ctypes.c_void_p(b), 5 * k, s,
                                           ctypes.byref(fin), ctypes.byref(ms)), "iterate", lib=lib)
            best = ms.value / 5 if best is None else min(best, ms.value / 5)
        return best

    for mode in args.modes.split(","):
        total = 2 * span + max(deltas) + (2 << 20)
        p = ctypes.c_void_p()
        rc = (hip.hipExtMallocWithFlags(ctypes.byref(p), total, 0x4) if mode == "contiguous"
              else hip.hipMalloc(ctypes.byref(p), total))
        if rc != 0:
            print(f"{mode}: allocation of {total} B failed ({rc})", flush=True)
            continue
        base = p.value
        for d in deltas:
            ms = timed(base, base + span + d)
            print(f"{mode:10s} delta {d:>10d} B: {ms:.4f} ms per K={k} launch, {cells * k / ms / 1e6:.1f} Gcell/s",
                  flush=True)
        # and a -> b the other way round (b first in memory)
        ms = timed(base + span + deltas[0], base)
        print(f"{mode:10s} swapped (b below a): {ms:.4f} ms, {cells * k / ms / 1e6:.1f} Gcell/s", flush=True)
        hip.hipFree(p)
        torch.cuda.synchronize()


if __name__ == "__main__":
    main()
