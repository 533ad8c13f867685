import sys, os
sys.path.insert(0, os.getcwd())
import torch
from stencil_amd.engine import JacobiEngine, StencilSpec
torch.cuda.set_device(0)
for dt in ("fp64", "fp32"):
    eng = JacobiEngine(StencilSpec(dims=2, dtype=dt), 1024, 1024, 1, device=0)
    eng.reset()
    eng.prepare()
    for rep in range(2):
        r = eng.place(trials=8, sweeps=100, passes=3)
        print(dt, rep, r["ms_per_launch"], "chose", r["chosen"], flush=True)
