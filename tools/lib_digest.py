"""Bitwise check of a library variant (tools/lib_variants.sh) against another build, process by
process: run AUTO's whole job of one shape from a random interior and print the sha256 of the final
grid's interior + ghosts; equal digests across builds = bitwise equal results.
usage: python tools/lib_digest.py <lib.so> <star|box> <fp32|fp64> nx ny nz sweeps [seed]"""
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from stencil_amd import _lib  # noqa: E402

_lib.LIB_PATH = os.path.abspath(sys.argv[1])
from stencil_amd.engine import JacobiEngine, StencilSpec  # noqa: E402

shape, dtype = sys.argv[2], sys.argv[3]
nx, ny, nz, sweeps = (int(v) for v in sys.argv[4:8])
seed = int(sys.argv[8]) if len(sys.argv) > 8 else 5
e = JacobiEngine(StencilSpec(dims=3, dtype=dtype, shape=shape), nx, ny, nz, device=0)
e.reset("random", seed)
grid, _ = e.iterate(sweeps)
dense = e.to_numpy(grid)
print(f"{shape} {dtype} {nx}x{ny}x{nz} {sweeps} sweeps seed {seed}: {hashlib.sha256(dense.tobytes()).hexdigest()[:24]}",
      flush=True)
