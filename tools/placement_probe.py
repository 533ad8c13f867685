#!/usr/bin/env python3
"""Does where a grid's pages land change the fp32 strip launch's speed?
(DESIGN.md §9 open end: the same library runs 2508 or 2719 Gcell/s at
4096^2 x 256 fp32 on different boxes.)  In ONE process, allocate the two grids
again and again -- hipMalloc, hipExtMallocWithFlags(contiguous) or torch --
each time behind a spacer allocation of a different size (so the grids land
elsewhere), fill them with the reference initial condition, and time K = 5
launches with the grids' own events.

    python tools/placement_probe.py [--grid 4096 4096 256] [--dtype fp32] [--reps 4]"""
import argparse
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

HIP_CONTIGUOUS = 0x4  # hipDeviceMallocContiguous (hip_runtime_api.h)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grid", type=int, nargs=3, default=[4096, 4096, 256])
    ap.add_argument("--dtype", default="fp32", choices=["fp32", "fp64"])
    ap.add_argument("--reps", type=int, default=4)
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
    k = eng.fuse_steps
    cells = nx * ny * nz

    def hip_alloc(n, flags):
        p = ctypes.c_void_p()
        rc = hip.hipExtMallocWithFlags(ctypes.byref(p), n, flags) if flags else hip.hipMalloc(ctypes.byref(p), n)
        if rc != 0:
            raise RuntimeError(f"allocation of {n} B (flags {flags}) failed: {rc}")
        return p.value

    def timed(a, b):
        s = _stream_handle(None)
        for g in (a, b):
            _lib.check(lib.stencil_fill_initial(ctypes.byref(lay), ctypes.c_void_p(g), _lib.INIT_REFERENCE,
                                                ctypes.c_uint64(0), s), "fill", lib=lib)
        fin, ms = ctypes.c_int(0), ctypes.c_float(0.0)
        lib.stencil_iterate(ctypes.byref(lay), ctypes.c_void_p(a), ctypes.c_void_p(b), 4 * k, s, ctypes.byref(fin), None)
        best = None
        for _ in range(3):
            _lib.check(lib.stencil_iterate(ctypes.byref(lay), ctypes.c_void_p(a), ctypes.c_void_p(b), 5 * k, s,
                                           ctypes.byref(fin), ctypes.byref(ms)), "iterate", lib=lib)
            per = ms.value / 5
            best = per if best is None else min(best, per)
        return best

    gib = 1 << 30
    for rep in range(args.reps):
        for mode in ("hipMalloc", "contiguous", "torch"):
            spacer_gib = 1 + (3 * rep + len(mode)) % 7
            spacer = hip_alloc(spacer_gib * gib, 0)
            if mode == "torch":
                ta = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
                tb = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
                a, b = ta.data_ptr(), tb.data_ptr()
            else:
                flags = HIP_CONTIGUOUS if mode == "contiguous" else 0
                a, b = hip_alloc(nbytes, flags), hip_alloc(nbytes, flags)
            ms = timed(a, b)
            print(f"rep {rep} {mode:10s} spacer {spacer_gib} GiB  a=0x{a:x}: {ms:.4f} ms per K={k} launch, "
                  f"{cells * k / ms / 1e6:.1f} Gcell/s", flush=True)
            if mode == "torch":
                del ta, tb
                torch.cuda.empty_cache()
            else:
                hip.hipFree(ctypes.c_void_p(a))
                hip.hipFree(ctypes.c_void_p(b))
            hip.hipFree(ctypes.c_void_p(spacer))
            torch.cuda.synchronize()


if __name__ == "__main__":
    main()
