STENCIL_TK_VERBOSE=1 timeout -k 5 60 python - <<'PY' 2>&1 | grep -v amdgpu.ids
import os, sys, torch
sys.path.insert(0, os.environ["GRAFT_REPO_ROOT"])
from stencil_amd import _lib
from stencil_amd.engine import JacobiEngine, StencilSpec
for flags in (0, 3):
    e = JacobiEngine(StencilSpec(dims=3, dtype="fp64", halo=4), 512, 512, 512, device=0, flags=flags)
    e.reset("random", 1)
    print("flags", flags, "sweepk:", flush=True); e.sweepk(e.a, e.b, 0, 512, 4); torch.cuda.synchronize()
    sig = torch.zeros(4, dtype=torch.int32, device="cuda")
    print("signal:", flush=True); e.sweepk_signal(e.a, e.b, 0, 512, 4, sig); torch.cuda.synchronize()
    print("interior [4,508):", flush=True); e.sweepk(e.a, e.b, 4, 508, 4); torch.cuda.synchronize()
PY
