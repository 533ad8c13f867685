"""The box's packed schedule against equal chunks, bitwise, at shapes where the
schedule is used (STENCIL_BOXK_PACK=1 vs 0; K = the AUTO box depth).
usage: python tools/box_pack_check.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from stencil_amd.engine import JacobiEngine, StencilSpec  # noqa: E402

for dtype in ("fp64", "fp32"):
    for shape in [(512, 512, 512), (400, 400, 400), (640, 640, 320)]:
        res = []
        for pack in ("1", "0"):
            os.environ["STENCIL_BOXK_PACK"] = pack
            e = JacobiEngine(StencilSpec(dims=3, dtype=dtype, shape="box"), *shape, device=0)
            e.reset("random", 5)
            k = e.fuse_steps
            e.sweepk(e.a, e.b, 0, shape[2], k)
            torch.cuda.synchronize()
            res.append(torch.from_numpy(e.to_numpy(e.b)))  # ghosts included, not the row padding
            del e
        ib = torch.int64 if dtype == "fp64" else torch.int32
        same = torch.equal(res[0].view(ib), res[1].view(ib))
        print(dtype, shape, "K", k, "bitwise equal" if same else "DIFFER", flush=True)
