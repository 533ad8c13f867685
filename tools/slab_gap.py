#!/usr/bin/env python3
"""Where a slab round's kernel loses against the plain launch on the same
shape (open end 1).  One K = 4 launch of the 7-point strip over
nx x ny x nz fp64, a -> b, timed with HIP events (best of --reps x 3 launches):

  plain      one grid, z ghost depth 1, no halo flags (AUTO's own layout)
  halo4      the slab's layout (z ghost depth 4), no flags
  flags      halo4 + HALO_LO | HALO_HI (the slab's launch geometry)
  signal     flags as a face-signalled launch (stencil_sweepk_signal)
  hipmalloc  flags on grids from stencil_alloc (hipMalloc) instead of torch
  slab       the C-ABI slab job: one periodic slab, face-signalled rounds

    python tools/slab_gap.py [nx ny nz] [--reps 5]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("grid", type=int, nargs="*", default=[4096, 4096, 512])
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    import torch
    from stencil_amd import _lib
    from stencil_amd.engine import JacobiEngine, SlabJob, StencilSpec
    nx, ny, nz = a.grid
    torch.cuda.set_device(0)
    cells = float(nx) * ny * nz * 4

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        best = None
        for _ in range(a.reps):
            t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0.record()
            for _ in range(3):
                fn()
            t1.record()
            t1.synchronize()
            ms = t0.elapsed_time(t1) / 3
            best = ms if best is None else min(best, ms)
        return best

    out = []
    for name, halo, flags in (("plain", 0, 0), ("halo4", 4, 0), ("flags", 4, 3)):
        e = JacobiEngine(StencilSpec(dims=3, dtype="fp64", halo=halo), nx, ny, nz, device=0, flags=flags)
        e.reset("random", 3)
        ms = timed(lambda: e.sweepk(e.a, e.b, 0, nz, 4))
        out.append((name, ms))
        if name == "flags":
            sig = torch.zeros(4, dtype=torch.int32, device=e.a.device)
            ms = timed(lambda: e.sweepk_signal(e.a, e.b, 0, nz, 4, sig))
            out.append(("signal", ms))
        del e
        torch.cuda.empty_cache()
    # the same launch on grids from hipMalloc (stencil_alloc, as the slab job allocates) instead of torch
    import ctypes
    lib = _lib.load()
    lay = _lib.make_layout(StencilSpec(dims=3, dtype="fp64", halo=4).problem(nx, ny, nz, 3))
    pa, pb = ctypes.c_void_p(), ctypes.c_void_p()
    _lib.check(lib.stencil_alloc(ctypes.byref(lay), ctypes.byref(pa)), "stencil_alloc", lib=lib)
    _lib.check(lib.stencil_alloc(ctypes.byref(lay), ctypes.byref(pb)), "stencil_alloc", lib=lib)
    for p_ in (pa, pb):
        _lib.check(lib.stencil_fill_initial(ctypes.byref(lay), p_, _lib.INIT_RANDOM, 3, None), "fill", lib=lib)
    ms = timed(lambda: _lib.check(lib.stencil_sweepk(ctypes.byref(lay), pa, pb, 0, nz, 4,
                                                     ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)),
                                  "stencil_sweepk", lib=lib))
    out.append(("hipmalloc", ms))
    lib.stencil_free(pa)
    lib.stencil_free(pb)
    job = SlabJob(StencilSpec(dims=3, dtype="fp64"), nx, ny, nz, [0], exchange="copy", periodic=True)
    job.fill_initial("random", 3)
    job.run(8)
    job.kernel_timing(True)
    job.run(4 * a.reps)
    kt = job.kernel_time()
    job.close()
    out.append(("slab", kt["total_ms"] / max(1, kt["launches"])))
    for name, ms in out:
        print(f"{name:7s} {nx}x{ny}x{nz} K=4: {ms:8.3f} ms per launch, {cells / ms / 1e6:7.1f} Gcell/s", flush=True)


if __name__ == "__main__":
    main()
