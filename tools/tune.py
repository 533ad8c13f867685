"""Interleaved A/B timing of kernel variants selected by environment knobs
(one process, several rounds; see cdna_hip_programming.md §5.4 rule 24).
usage: python tools/tune.py [n] [variants-json]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from stencil_amd.engine import JacobiEngine, StencilSpec, copy_bandwidth  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    variants = json.loads(sys.argv[2]) if len(sys.argv) > 2 else [{}]
    kernel = os.environ.get("TUNE_KERNEL", "auto")
    dtype = os.environ.get("TUNE_DTYPE", "fp64")
    iters = int(os.environ.get("TUNE_ITERS", "50"))
    shape = [int(v) for v in os.environ.get("TUNE_SHAPE", f"{n},{n},{n}").split(",")]
    stencil = os.environ.get("TUNE_STENCIL", "star")
    eng = JacobiEngine(StencilSpec(dims=3, dtype=dtype, kernel=kernel, shape=stencil), *shape)
    cells = shape[0] * shape[1] * shape[2]
    eng.reset()
    es = 8 if dtype == "fp64" else 4
    print(f"copy kernel: {copy_bandwidth(1 << 30, 20):.0f} GB/s", flush=True)
    base_env = {k: v for k, v in os.environ.items() if k.startswith("STENCIL_")}  # set by the caller
    res = {i: [] for i in range(len(variants))}
    for rnd in range(4):
        for i, v in enumerate(variants):
            for k in list(os.environ):
                if k.startswith("STENCIL_") and k not in base_env:
                    del os.environ[k]
            os.environ.update(base_env)
            os.environ.update({k: str(x) for k, x in v.items()})
            eng.iterate(4)
            _, ms = eng.iterate(iters, timed=True)
            launches = eng.plan(iters)[0]
            res[i].append(ms / iters)
    for i, v in enumerate(variants):
        t = sorted(res[i])
        gbs = cells * 2 * es / (t[0] * 1e-3) / 1e9
        print(f"{json.dumps(v):60s} ms/sweep min {t[0]:.4f} med {t[len(t)//2]:.4f}  {gbs:.0f} GB/s alg  "
              f"{cells/(t[0]*1e-3)/1e9:.1f} Gcell/s", flush=True)


if __name__ == "__main__":
    main()
