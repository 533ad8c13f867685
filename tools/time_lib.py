"""Time AUTO's whole-job sweeps of one shape through a given build of the product library (the bench's
own path: stencil_prepare, then stencil_iterate from the reference initial condition; device time from
the library's hipEvents), for A/B runs of library variants in separate processes (tools/lib_variants.sh).
usage: python tools/time_lib.py <lib.so> <star|box> <fp32|fp64> nx ny nz sweeps [reps]   (nz = 0: a 2D grid)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from stencil_amd import _lib  # noqa: E402

_lib.LIB_PATH = os.path.abspath(sys.argv[1])
from stencil_amd.engine import JacobiEngine, StencilSpec  # noqa: E402

shape, dtype = sys.argv[2], sys.argv[3]
nx, ny, nz, sweeps = (int(v) for v in sys.argv[4:8])
reps = int(sys.argv[8]) if len(sys.argv) > 8 else 3
dims = 2 if nz == 0 else 3
radius, order = int(os.environ.get("TL_RADIUS", "1")), os.environ.get("TL_ORDER", "naive")  # 2D variants
e = JacobiEngine(StencilSpec(dims=dims, dtype=dtype, shape=shape, radius=radius, order=order), nx, ny, max(1, nz),
                 device=0)
e.reset("reference")
e.prepare()
e.iterate(e.fuse_steps * 2)
best = None
for _ in range(reps):
    ms = e.iterate(sweeps, timed=True)[1]
    best = ms if best is None else min(best, ms)
print(f"{os.path.basename(sys.argv[1])} {shape} r{radius} {order} {dtype} {nx}x{ny}x{nz} {sweeps} sweeps: best {best:.3f} ms, "
      f"{nx * ny * max(1, nz) * sweeps / best / 1e6:.1f} Gcell/s", flush=True)
