#!/usr/bin/env python3
"""Why do the first ~25 K-step launches of a process run 5-8 % slower?
(VERDICT r03, weak #4.)  Run under `rocprofv3 --kernel-trace` and read the
per-dispatch durations by phase: the phases are separated by a tiny marker
kernel (a 16-byte stencil_copy_bandwidth), so the trace splits cleanly.

  A  prepare() + 60 back-to-back K = 4 launches (the bench's start)
  B  0.3 s host idle, then 30 launches          -> does idle re-trigger a ramp?
  C  re-fill with the reference IC (zeros), 30  -> does the data reset the ramp?
  D  random interior, 30 launches               -> data entropy (DVFS) effect
  E  ~60 ms of copy-kernel streaming, re-fill reference IC, 30 launches
     -> does a settle phase of other streaming work remove the ramp?

512^3 fp64 7-point, the C2 workload."""
import ctypes
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

import torch  # noqa: E402

from stencil_amd import _lib  # noqa: E402
from stencil_amd.engine import JacobiEngine, StencilSpec  # noqa: E402


def marker(lib, buf):
    ms = ctypes.c_float(0.0)
    _lib.check(lib.stencil_copy_bandwidth(ctypes.c_void_p(buf.data_ptr()), ctypes.c_void_p(buf.data_ptr() + 16), 16, 1,
                                          None, ctypes.byref(ms)), "marker", lib=lib)


def main():
    n = int(os.environ.get("RAMP_N", "512"))
    eng = JacobiEngine(StencilSpec(dims=3, dtype="fp64"), n, n, n, device=0)
    lib = eng.lib
    mk = torch.zeros(64, dtype=torch.float32, device="cuda")
    big = torch.empty(1 << 28, dtype=torch.float32, device="cuda")  # 1 GiB
    big2 = torch.empty_like(big)
    eng.reset("reference")
    torch.cuda.synchronize()
    t = {}
    marker(lib, mk)
    t0 = time.perf_counter()
    eng.prepare()
    eng.iterate(240)
    torch.cuda.synchronize()
    t["A"] = time.perf_counter() - t0
    marker(lib, mk)
    torch.cuda.synchronize()
    time.sleep(0.3)
    t0 = time.perf_counter()
    eng.iterate(120)
    torch.cuda.synchronize()
    t["B"] = time.perf_counter() - t0
    marker(lib, mk)
    eng.reset("reference")
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    eng.iterate(120)
    torch.cuda.synchronize()
    t["C"] = time.perf_counter() - t0
    marker(lib, mk)
    eng.reset("random", 7)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    eng.iterate(120)
    torch.cuda.synchronize()
    t["D"] = time.perf_counter() - t0
    marker(lib, mk)
    ms = ctypes.c_float(0.0)
    _lib.check(lib.stencil_copy_bandwidth(ctypes.c_void_p(big2.data_ptr()), ctypes.c_void_p(big.data_ptr()), 1 << 30,
                                          200, None, ctypes.byref(ms)), "copy", lib=lib)
    eng.reset("reference")
    t0 = time.perf_counter()
    eng.iterate(120)
    torch.cuda.synchronize()
    t["E"] = time.perf_counter() - t0
    marker(lib, mk)
    torch.cuda.synchronize()
    print({k: round(v * 1e3, 2) for k, v in t.items()}, "copy ms per rep", ms.value / 200, flush=True)


if __name__ == "__main__":
    main()
