"""STENCIL_TK_PACK parity at full size: the packed longest-first schedule must
give the same bits as the equal-chunk grid (512^3 and 2048^2 x 512 fp64,
random interior, 12 sweeps = 3 K-step launches)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from stencil_amd.engine import JacobiEngine, StencilSpec  # noqa: E402

os.environ["STENCIL_TK_VERBOSE"] = "1"
for shape, dt in (((512, 512, 512), "fp64"), ((2048, 2048, 512), "fp64"), ((512, 512, 512), "fp32")):
    eng = JacobiEngine(StencilSpec(dims=3, dtype=dt, kernel="temporalk"), *shape)
    out = []
    for pack in ("0", "1"):
        os.environ["STENCIL_TK_PACK"] = pack
        eng.reset("random", 99)
        fin, _ = eng.iterate(12)
        torch.cuda.synchronize()
        out.append(fin.clone())
    same = torch.equal(out[0].view(torch.int8), out[1].view(torch.int8))
    print(shape, dt, "bitwise equal" if same else "DIFFERENT", flush=True)
    del out, eng
    torch.cuda.empty_cache()
    if not same:
        sys.exit(1)
