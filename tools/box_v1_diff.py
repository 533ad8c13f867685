"""Where a box strip shape differs from the oracle (debug aid): per cfg, the
differing cells by (z, y, x) pattern.  usage: python tools/box_v1_diff.py dtype steps cfg..."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from oracle import binding as ob  # noqa: E402
from stencil_amd.engine import JacobiEngine, StencilSpec  # noqa: E402

dtype, steps = sys.argv[1], int(sys.argv[2])
nx, ny, nz = 64, 48, 20
p = ob.problem(3, dtype, "box", 1, "naive", nx, ny, nz)
want = ob.run(p, steps, "random", 17)
for cfg in sys.argv[3:]:
    os.environ["STENCIL_BOXK_CFG"] = cfg
    e = JacobiEngine(StencilSpec(dims=3, dtype=dtype, shape="box"), nx, ny, nz, device=0)
    e.reset("random", 17)
    e.sweepk(e.a, e.b, 0, nz, steps)
    got = e.to_numpy(e.b)
    d = got != want
    zs, ys, xs = np.nonzero(d)
    print(cfg, "differ", int(d.sum()), "of", d.size, flush=True)
    if len(zs):
        print("  z", np.unique(zs)[:12], "y", np.unique(ys)[:20], "x", np.unique(xs)[:20])
        k = (zs[0], ys[0], xs[0])
        print("  first", k, "got", got[k], "want", want[k], "rel", float(abs(got[k] - want[k]) / abs(want[k])))
        r = np.abs(got - want)[d] / np.maximum(np.abs(want[d]), 1e-30)
        print("  max rel", float(r.max()), "median rel", float(np.median(r)))
