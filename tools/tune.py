"""Interleaved A/B timing of kernel variants selected by environment knobs
(one process, several rounds; see cdna_hip_programming.md §5.4 rule 24).
usage: python tools/tune.py [n] [variants-json]
TUNE_SWEEPK=k times k-step stencil_sweepk launches over the whole grid instead
of stencil_iterate (the only way to reach e.g. the 3-step box kernel)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from stencil_amd.engine import JacobiEngine, StencilSpec, copy_bandwidth  # noqa: E402


def time_sweepk(eng, k, iters):
    """ms for `iters` sweeps done as iters//k k-step launches (a <-> b)."""
    n = eng.slow_extent
    launches = max(1, iters // k)
    for _ in range(2):
        eng.sweepk(eng.a, eng.b, 0, n, k)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    src, dst = eng.a, eng.b
    for _ in range(launches):
        eng.sweepk(src, dst, 0, n, k)
        src, dst = dst, src
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * iters / (launches * k)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    variants = json.loads(sys.argv[2]) if len(sys.argv) > 2 else [{}]
    kernel = os.environ.get("TUNE_KERNEL", "auto")
    dtype = os.environ.get("TUNE_DTYPE", "fp64")
    iters = int(os.environ.get("TUNE_ITERS", "50"))
    shape = [int(v) for v in os.environ.get("TUNE_SHAPE", f"{n},{n},{n}").split(",")]
    stencil = os.environ.get("TUNE_STENCIL", "star")
    sweepk = int(os.environ.get("TUNE_SWEEPK", "0"))
    dims = int(os.environ.get("TUNE_DIMS", "3"))
    order = os.environ.get("TUNE_ORDER", "naive")
    if dims == 2:
        shape = shape[:2] + [1]
    eng = JacobiEngine(StencilSpec(dims=dims, dtype=dtype, kernel=kernel, shape=stencil, order=order), *shape)
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
            if sweepk:
                ms = time_sweepk(eng, sweepk, iters)
            else:
                eng.iterate(4)
                _, ms = eng.iterate(iters, timed=True)
            res[i].append(ms / iters)
    for i, v in enumerate(variants):
        t = sorted(res[i])
        gbs = cells * 2 * es / (t[0] * 1e-3) / 1e9
        print(f"{json.dumps(v):60s} ms/sweep min {t[0]:.4f} med {t[len(t)//2]:.4f}  {gbs:.0f} GB/s alg  "
              f"{cells/(t[0]*1e-3)/1e9:.1f} Gcell/s", flush=True)


if __name__ == "__main__":
    main()
