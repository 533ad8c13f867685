import sys, os
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import torch
from stencil_amd.engine import copy_bandwidth
for mb in (8, 16, 32, 64, 96, 128, 256, 1024):
    bw = copy_bandwidth(mb << 20, reps=50)
    print(f"copy {mb:5d} MiB src (+ same dst): {bw:8.0f} GB/s", flush=True)
