"""Measure every BASELINE.json config that fits one MI355X (one GPU, one
process) and write profiles/configs_<tag>.json.  bench.py stays the driver's
contract (config 2 / weak-scaled slabs); this is the per-config table.

  C1  2D 5-point fp64 1024^2, 100 iterations         (full)
  C1r 2D 5-point fp32 1024^2, 100 iterations, DMA order (the reference's own dtype/order)
  C2  3D 7-point fp64 512^3, 1000 iterations          (full)
  C3r 3D 7-point fp32 4096^2 x 1024, 100 iterations   (C3 is 4096^3: 2 x 275 GB does not fit 288 GB)
  C4s 3D 7-point fp64 2048^2 x 512 = one GPU's slab of C4, 100 iterations
  C5s 3D 27-point fp64 2048^2 x 256 = one GPU's slab of C5, 100 iterations

usage: python tools/bench_configs.py <tag> [config ...]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from stencil_amd.engine import JacobiEngine, StencilSpec  # noqa: E402

CONFIGS = {
    "C1": dict(spec=StencilSpec(dims=2, dtype="fp64"), shape=(1024, 1024, 1), iters=100),
    "C1r": dict(spec=StencilSpec(dims=2, dtype="fp32", order="dma"), shape=(1024, 1024, 1), iters=100),
    "C2": dict(spec=StencilSpec(dims=3, dtype="fp64"), shape=(512, 512, 512), iters=1000),
    "C3r": dict(spec=StencilSpec(dims=3, dtype="fp32"), shape=(4096, 4096, 1024), iters=100),
    "C4s": dict(spec=StencilSpec(dims=3, dtype="fp64"), shape=(2048, 2048, 512), iters=100),
    "C5s": dict(spec=StencilSpec(dims=3, dtype="fp64", shape="box"), shape=(2048, 2048, 256), iters=100),
}


# CPU baseline per config: the oracle's naive sweep on the
# host, single-threaded (the reference's CPU path) and with OpenMP over the
# host's CPU share; full size where that fits a ~10 s budget, else the rate
# on a 512^3 sub-problem of the same stencil and dtype.
CPU_SAMPLE = {"C1": (1024, 1024, 1), "C1r": (1024, 1024, 1), "C2": (512, 512, 512), "C3r": (512, 512, 512),
              "C4s": (512, 512, 512), "C5s": (512, 512, 512)}


def cpu_rate(name, c, budget_s=8.0):
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from bench import host_threads
    from oracle import binding as ob
    spec = c["spec"]
    nx, ny, nz = CPU_SAMPLE[name]
    p = ob.problem(spec.dims, spec.dtype, spec.shape, spec.radius, spec.order, nx, ny, nz)
    out = {}
    for threads in (1, host_threads()):
        t1 = ob.timed_run(p, 1, threads=threads)
        it = max(1, min(c["iters"], int(budget_s / max(t1, 1e-6))))
        t = ob.timed_run(p, it, threads=threads)
        out[f"threads_{threads}"] = {"gcell_per_s": round(nx * ny * nz * it / t / 1e9, 4), "iterations": it,
                                     "grid": [nx, ny, nz], "seconds": round(t, 2)}
    return out


def run(name, c):
    spec, (nx, ny, nz), iters = c["spec"], c["shape"], c["iters"]
    e = JacobiEngine(spec, nx, ny, nz)
    e.reset()
    e.iterate(2)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    _, dev_ms = e.iterate(iters, timed=True)
    wall = time.perf_counter() - t0
    launches, kernel = e.plan(iters)
    cells = nx * ny * nz
    out = {"config": name, "grid": [nx, ny, nz], "dims": spec.dims, "dtype": spec.dtype, "shape": spec.shape,
           "order": spec.order, "iterations": iters, "kernel": {1: "direct", 2: "zmarch", 3: "temporal2", 4: "temporalk"}[kernel],
           "launches": launches, "device_ms": round(dev_ms, 4), "wall_ms": round(wall * 1e3, 4),
           "gcell_per_s": round(cells * iters / (dev_ms * 1e-3) / 1e9, 2),
           "alg_GBps": round(cells * iters * 2 * spec.elem_bytes / (dev_ms * 1e-3) / 1e9, 1)}
    del e
    torch.cuda.empty_cache()
    if os.environ.get("CONFIGS_CPU", "1") != "0":
        out["cpu_baseline"] = cpu_rate(name, c)
        best = max(v["gcell_per_s"] for v in out["cpu_baseline"].values())
        out["gpu_over_best_cpu"] = round(out["gcell_per_s"] / best, 1)
    return out


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "run"
    names = sys.argv[2:] or list(CONFIGS)
    rows = []
    for n in names:
        r = run(n, CONFIGS[n])
        print(json.dumps(r), flush=True)
        rows.append(r)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    os.makedirs(os.path.join(root, "gpurun_out"), exist_ok=True)
    json.dump(rows, open(os.path.join(root, "gpurun_out", f"configs_{tag}.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
