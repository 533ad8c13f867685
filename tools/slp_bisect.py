"""Run the fp32 box probe shapes through one variant of the debug library
(tools/slp_bisect.sh) and count the cells that differ from a reference: the
oracle, or (--ref-cfg, for libraries built from an older box order than the
oracle's) the same library's output for another cfg.
usage: python tools/slp_bisect.py <libdbg_*.so> <steps> [--ref-cfg CFG] <cfg> [cfg ...]
(cfg 95RRNN = the probe's SLP build, 96RRNN = the same source without SLP)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from stencil_amd import _lib  # noqa: E402

_lib.DEBUG_LIB_PATH = os.path.abspath(sys.argv[1])
from stencil_amd.engine import JacobiEngine, StencilSpec  # noqa: E402

steps = int(sys.argv[2])
args = sys.argv[3:]
ref_cfg = None
if args[0] == "--ref-cfg":
    ref_cfg, args = args[1], args[2:]
nx, ny, nz = 64, 48, 20


def run(cfg):
    os.environ["STENCIL_BOXK_CFG"] = cfg
    e = JacobiEngine(StencilSpec(dims=3, dtype="fp32", shape="box"), nx, ny, nz, device=0)
    e.reset("random", 17)
    e.sweepk(e.a, e.b, 0, nz, steps)
    return e.to_numpy(e.b)


if ref_cfg:
    want, ref = run(ref_cfg), f"cfg {ref_cfg}"
else:
    from oracle import binding as ob
    p = ob.problem(3, "fp32", "box", 1, "naive", nx, ny, nz)
    want, ref = ob.run(p, steps, "random", 17), "the oracle"
for cfg in args:
    d = run(cfg) != want
    print(os.path.basename(sys.argv[1]), "steps", steps, "cfg", cfg, "differ from", ref, int(d.sum()), "of", d.size,
          flush=True)
