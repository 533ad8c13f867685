#!/usr/bin/env python3
"""Benchmark: 3D 7-point fp64 Jacobi (BASELINE.json metric, config 2 size per GPU).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config C1|C2|C3|C4|C5|NS|NS4096]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

One step = one Jacobi sweep of the whole grid.  At N=1 the workload is
BASELINE config 2 (512^3 interior, fp64, 7-point star; the default K=1000 is
exactly its 1000 iterations).  At N>1 every rank owns a 512^3 Z-slab of a
512 x 512 x 512N grid (weak scaling) and exchanges K halo planes with each
neighbour per round of K fused sweeps (K = 4: the strip-layout K-step
kernel) over RCCL, overlapped with the rest of the round's launch
(face-signalled rounds on such few-tile planes; staged rounds on wide ones;
csrc/slab_core.hpp).

Multi-GPU drivers, same job, same JSON line, ONE implementation of the rounds
(the C-ABI slab job, csrc/slab_core.hpp):
  * one process per GPU (launched by torch.distributed.run; WORLD_SIZE set):
    rank mode (stencil_slab_create_rank: each rank its own slab, RCCL between
    the ranks); torch.distributed (gloo, host side only) carries the RCCL id,
    the barriers, the max-over-ranks time and the check's per-plane sums;
  * --gpus N without a launcher (WORLD_SIZE unset): ONE process drives the N
    GPUs (stencil_slab_create; RCCL ncclCommInitAll), the shape of the
    reference's single spawn/join of its whole decomposed job
    (src/stencil/stencil.cpp:34-53);
  * --exchange loopback | nccl-self at N=1: one slab whose z ends form a ring
    (periodic), halos by device copies or RCCL send/recv to itself -- the
    interior-rank rehearsal on one GPU.

--config picks another BASELINE.json config as the workload (C1: the
reference's own 2D 1024^2 case; C3: 4096^3 fp32, C4: 2048x2048x4096 fp64, C5:
2048^3 27-point fp64, their global grids z-slab split over the ranks; NS4096:
the north star's own 4096^3 fp64 7-point grid, 2 GPUs or more).  Slabs whose
two grids do not fit a GPU keep ONE grid plus a rolling margin
(STENCIL_SLAB_ROLLING), as C3 / C4 do on one GPU.

Rank 0 prints one JSON line with the whole-job rate, the live roofline of the
dominant kernel (compulsory bytes per launch / average launch time from HIP
events on the kernel's own stream), and a bounded CPU baseline (the oracle's
restatement of the reference's naive sweep, N=1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

METRIC = "Gcell-updates/s + achieved HBM GB/s vs roofline, 7-pt fp64 Jacobi, 1/2/4/8 GPUs"
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (/opt/skills/guides/MI355X_MICROARCH.md)
GiB = 1 << 30
INIT_SEED = 1  # --init random: splitmix64(seed + cell index)
# HBM kept free beside a slab's grids (RCCL's buffers and the library's scratch)
SLAB_RESERVE = 8 * GiB


# BASELINE.json configs as bench workloads.  C2 (the default, the metric's
# config) is weak-scaled: n^3 per GPU.  C3-C5 and NS4096 are global grids,
# z-slab split over the ranks (strong scaling); at N = 1, C3 and C4 keep ONE
# resident grid (two would need 2 x 279 GB / 2 x 138 GB).
PRESETS = {
    "C1": dict(dims=2, dtype="fp64", shape="star", grid=(1024, 1024, 1), min_gpus=1, max_gpus=1,
               desc="BASELINE config 1: 2D 5-point fp64 Jacobi, 1024x1024 (the reference's own case, run.sh -s 1024)"),
    "C2": dict(dtype="fp64", shape="star", grid=None, min_gpus=1,
               desc="BASELINE config 2: 3D 7-point fp64 Jacobi, {n}^3 interior per GPU"),
    # C3 on one GPU: ONE resident grid + a rolling margin (stencil_rolling_*),
    # since two grids are 2 x 279 GB
    "C3": dict(dtype="fp32", shape="star", grid=(4096, 4096, 4096), min_gpus=1,
               desc="BASELINE config 3: 3D 7-point fp32 Jacobi, 4096^3"),
    # C4 on one GPU likewise (one 138 GB grid + a margin)
    "C4": dict(dtype="fp64", shape="star", grid=(2048, 2048, 4096), min_gpus=1,
               desc="BASELINE config 4: 3D 7-point fp64 Jacobi, 2048x2048x4096"),
    "C5": dict(dtype="fp64", shape="box", grid=(2048, 2048, 2048), min_gpus=1,
               desc="BASELINE config 5: 3D 27-point fp64 stencil, 2048^3, temporal blocking (4 sweeps per launch, "
                    "deeper than the config's 2; bitwise the same result)"),
    # north_star's own grid: 4096^3 fp64 is 550 GB per grid -- not even ONE
    # grid fits a 288 GB MI355X; from 2 GPUs on (N = 2: one rolling 278 GB
    # grid per GPU; N >= 4: two grids per slab)
    "NS4096": dict(dtype="fp64", shape="star", grid=(4096, 4096, 4096), min_gpus=2,
                   desc="north star: 3D 7-point fp64 Jacobi, 4096^3, z-slab split over the GPUs"),
    # its largest single-GPU proxy: 2048^3 fp64, 2 x 70 GB
    "NS": dict(dtype="fp64", shape="star", grid=(2048, 2048, 2048), min_gpus=1,
               desc="north-star proxy: 3D 7-point fp64 Jacobi, 2048^3 (4096^3 does not fit one GPU)"),
}

# Kernel family (bench name) -> the sources that define it, hashed into the
# traffic table so a PMC figure measured on older kernel code is not reported.
KERNEL_SOURCES = {
    "temporalk": ("stencil_amd/csrc/kernels_strip.hip", "stencil_amd/csrc/kernels_strip_ilp.hip",
                  "stencil_amd/csrc/kernels_temporalk.hip"),
    "temporal2": ("stencil_amd/csrc/kernels_temporal.hip",),
    "zmarch": ("stencil_amd/csrc/kernels_zmarch.hip",),
    "direct": ("stencil_amd/csrc/kernels_direct.hip",),
    "boxk": ("stencil_amd/csrc/kernels_boxk.hip",),
    "tb2ds": ("stencil_amd/csrc/kernels_tb2d.hip", "stencil_amd/csrc/strip2d.hpp"),
}


# stencil_iterate / stencil_slab_run calls of at least this many sweeps take
# the long-job work orders (common.hpp kSustainedSweeps)
SUSTAINED_SWEEPS = 256


def kernel_source_sha(kname: str):
    import hashlib
    h = hashlib.sha256()
    for rel in KERNEL_SOURCES.get(kname, ()):
        with open(os.path.join(HERE, rel), "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16] if kname in KERNEL_SOURCES else None


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--config", default="C2", choices=sorted(PRESETS),
                    help="workload (default C2, the metric's config; C3-C5 / NS4096 split a global grid over the ranks)")
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--n", type=int, default=512, help="per-GPU cube edge (config 2: 512)")
    ap.add_argument("--kernel", default="auto", choices=["auto", "direct", "zmarch", "temporal2"])
    ap.add_argument("--placements", type=int, default=16,
                    help="single-GPU two-grid configs: grid placements tried before the run (the fastest kept; "
                         "1 = the first allocation)")
    ap.add_argument("--no-signal", action="store_true",
                    help="multi-GPU rounds as separate boundary/interior launches (no face counters; "
                         "STENCIL_SLAB_SIGNAL=0)")
    ap.add_argument("--exchange", default="nccl", choices=["nccl", "copy", "loopback", "nccl-self"],
                    help="halo transport: RCCL P2P (default) or, without a launcher, device copies between the slabs "
                         "(copy); at N=1, loopback / nccl-self rehearse an interior rank (a periodic slab whose "
                         "halos are its own faces, by device copies / RCCL send-recv to itself)")
    ap.add_argument("--share-device", action="store_true",
                    help="rehearsal without a launcher: every slab on GPU 0 (needs --exchange copy)")
    ap.add_argument("--rank-of", type=int, default=0, metavar="N",
                    help="with --exchange loopback | nccl-self: rehearse ONE interior rank of the N-GPU job (its "
                         "slab of the config's global grid, two grids or rolling as the N-GPU plan says, periodic "
                         "halos) on one GPU -- e.g. --config NS4096 --rank-of 2")
    ap.add_argument("--rolling", choices=["auto", "on", "off"], default="auto",
                    help="slabs: ONE grid + a rolling margin (on), two grids (off), or whatever fits (auto)")
    ap.add_argument("--init", choices=["reference", "random"], default="reference",
                    help="initial grid: the reference's (interior 0, x-ghost faces 1; the default) or a developed "
                         "field (uniform random [0,1) interior, splitmix64(seed 1 + cell index)): the box runs "
                         "12-18 %% faster on the reference's mostly-zero field (DVFS), DESIGN.md §6")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="budget of the CPU baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-check", action="store_true",
                    help="N>1: skip the bitwise check against the global grid run as one grid on rank 0")
    ap.add_argument("--slab-timeout-ms", type=int, default=0,
                    help="N>1 / rehearsals: the slab job's deadline for any device wait (stencil_slab_set_timeout; "
                         "0 = the library's default, 60 s): past it the job aborts its communicators and bench.py "
                         "exits non-zero")
    ap.add_argument("--allow-debug-library", action="store_true",
                    help="bench even when an experiment knob (a STENCIL_* variable the product ignores) is set, "
                         "i.e. on libstencil_hip_debug.so; the JSON line names the library and the knobs either way")
    args = ap.parse_args(argv)
    # slab jobs (the C-ABI) search grid placements only when asked (STENCIL_SLAB_PLACEMENTS, default 1):
    # the bench opts in with its own --placements, as its single-grid engine does (JacobiEngine.place)
    os.environ.setdefault("STENCIL_SLAB_PLACEMENTS", str(max(1, args.placements)))
    from stencil_amd import _lib
    if _lib.debug_knobs_requested() and not args.allow_debug_library:
        knobs = sorted(k for k in os.environ if k.startswith("STENCIL_") and k not in _lib.API_KNOBS)
        raise SystemExit(f"experiment knobs set ({', '.join(knobs)}): this would bench libstencil_hip_debug.so; "
                         "unset them or pass --allow-debug-library")
    if args.no_signal:
        os.environ["STENCIL_SLAB_SIGNAL"] = "0"  # an API knob: read at slab creation
    if args.rank_of and (args.rank_of < 2 or args.gpus != 1 or args.exchange not in ("loopback", "nccl-self")):
        raise SystemExit("--rank-of N (N >= 2) rehearses one rank of an N-GPU job on ONE GPU: it needs --gpus 1 and "
                         "--exchange loopback or nccl-self")
    return args


def _lib_forms():
    from stencil_amd import _lib
    return _lib.SLAB_FORMS


def library_info() -> dict:
    """Which build of the HIP library produced the line, and every STENCIL_*
    variable set in the environment (documented knobs included)."""
    from stencil_amd import _lib
    lib = _lib.load()
    return {"library": os.path.basename(_lib.DEBUG_LIB_PATH if lib.stencil_debug_knobs() else _lib.LIB_PATH),
            "stencil_env": {k: v for k, v in sorted(os.environ.items()) if k.startswith("STENCIL_")}}


def host_threads() -> int:
    """The host cores this process may use (the GPU box's CPU share: its
    OMP_NUM_THREADS, else the affinity mask)."""
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    env = os.environ.get("OMP_NUM_THREADS", "")
    return max(1, min(n, int(env))) if env.isdigit() and int(env) > 0 else n


def cpu_baseline(n: int, budget_s: float, threads: int = 1, dtype: str = "fp64", shape: str = "star", dims: int = 3,
                 iters_cap: int = 200):
    """The oracle (port of check_result's loop, stencil.cpp:94-131, generalised
    to 3D) on the host over a bounded number of sweeps of an n^dims grid of the
    workload's stencil: single-threaded like the reference's own CPU path, or
    with OpenMP over `threads` cores (identical per-cell arithmetic,
    bitwise-equal result)."""
    from oracle import binding as ob
    p = ob.problem(dims, dtype, shape, 1, "naive", n, n, n if dims == 3 else 1)
    t1 = ob.timed_run(p, 1, threads=threads)
    iters = max(1, min(iters_cap, int(budget_s / max(t1, 1e-6))))
    t = ob.timed_run(p, iters, threads=threads)
    cells = float(n) ** dims * iters
    who = "1 host thread" if threads == 1 else f"{threads} host threads (OpenMP)"
    pts = {(3, "star"): "7-point", (3, "box"): "27-point", (2, "star"): "5-point"}[(dims, shape)]
    shape_s = f"{n}^{dims}"
    return {"value": round(cells / t / 1e9, 4), "unit": "Gcell-updates/s", "cores": threads, "kind": "port",
            "sample": f"oracle/ naive sweep, {shape_s} {dtype} {pts}, {iters} sweeps from the reference initial "
                      f"condition, {t:.2f} s on {who}"}


def load_traffic(workload_key: str, kernel_name: str):
    """PMC bytes per launch (FETCH_SIZE x 2 + WRITE_SIZE, tools/summarize_profile.py)
    and the table entry; the bytes are None when the entry was measured on
    other kernel sources than the ones this tree builds (stale)."""
    path = os.path.join(HERE, "profiles", "traffic.json")
    try:
        data = json.load(open(path))
    except (OSError, ValueError):
        return None, None
    ent = data.get(workload_key, {}).get(kernel_name)
    if not ent:
        return None, None
    fresh = ent.get("kernel_source_sha") == kernel_source_sha(kernel_name)
    return (ent.get("hbm_bytes_per_launch") if fresh else None), dict(ent, fresh=fresh)


# ----------------------------------------------------------------- planning
def partition(nz: int, world: int, rank: int):
    """Contiguous z-slab `rank` of `world`: (first plane, planes); the nz %
    world remainder planes go to the lowest ranks (csrc/slab_core.hpp's split)."""
    base, rem = divmod(nz, world)
    return rank * base + min(rank, rem), base + (1 if rank < rem else 0)


def global_grid(config: str, n_gpus: int, n: int = 512):
    pre = PRESETS[config]
    if pre["grid"] is None:  # weak scaling: n^3 per GPU, stacked in z
        return n, n, n * n_gpus
    return pre["grid"]


def layout_bytes(spec, nx, ny, nz, halo=0):
    """Bytes of one padded grid of the library's layout (no GPU call)."""
    from stencil_amd import _lib
    lay = _lib.make_layout(spec.problem(nx, ny, nz) if not halo else
                           _lib.make_problem(dims=3, dtype=_lib.F64 if spec.dtype == "fp64" else _lib.F32,
                                             shape=_lib.BOX if spec.shape == "box" else _lib.STAR, radius=1,
                                             nx=nx, ny=ny, nz=nz, halo=halo))
    return int(lay.bytes), int(lay.plane) * spec.elem_bytes


def fuse_guess(dtype: str, shape: str, nx: int, ny: int) -> int:
    """The sweeps one launch fuses (api.hip's iterate_tk_steps /
    iterate_box_steps defaults): the slabs' halo depth."""
    if shape == "box":
        return 4 if nx * ny >= 384 * 384 else 3
    return 5 if dtype == "fp32" and nx * ny >= (1 << 20) else 4


def slab_plan(config: str, n_gpus: int, free_bytes: int, n: int = 512, rolling: str = "auto"):
    """What the multi-GPU job of `config` on `n_gpus` GPUs with `free_bytes`
    of HBM free per GPU would run: the global grid, each slab's planes and
    bytes, and whether slabs keep two grids or ONE grid plus a rolling margin
    (when two plus SLAB_RESERVE do not fit).  SystemExit with the reason when
    the job cannot run (too few GPUs, not even one grid per slab fits)."""
    from stencil_amd.engine import StencilSpec
    pre = PRESETS[config]
    if pre.get("dims", 3) != 3:
        raise SystemExit(f"--config {config} is 2D: one GPU only")
    if n_gpus < pre["min_gpus"]:
        gx, gy, gz = global_grid(config, n_gpus, n)
        one = layout_bytes(StencilSpec(dims=3, dtype=pre["dtype"], shape=pre["shape"]), gx, gy, gz)[0]
        raise SystemExit(f"--config {config} needs at least {pre['min_gpus']} GPUs: ONE {gx}x{gy}x{gz} "
                         f"{pre['dtype']} grid is {one / 1e9:.0f} GB, more than a GPU holds; run it as "
                         f"`python -m torch.distributed.run --nproc-per-node {pre['min_gpus']} --master-addr 127.0.0.1 "
                         f"bench.py --gpus {pre['min_gpus']} --config {config}`")
    gx, gy, gz = global_grid(config, n_gpus, n)
    spec = StencilSpec(dims=3, dtype=pre["dtype"], shape=pre["shape"])
    k = fuse_guess(pre["dtype"], pre["shape"], gx, gy)
    planes = max(partition(gz, n_gpus, r)[1] for r in range(n_gpus))
    depth = k if n_gpus > 1 else 1
    grid_b, plane_b = layout_bytes(spec, gx, gy, planes, halo=depth if n_gpus > 1 else 0)
    two = 2 * grid_b + SLAB_RESERVE <= free_bytes
    if rolling == "off" and not two:
        raise SystemExit(f"--rolling off: two {grid_b / 1e9:.0f} GB grids per slab do not fit {free_bytes / 1e9:.0f} GB")
    use_rolling = rolling == "on" or (rolling == "auto" and not two)
    if use_rolling:
        margin = min(512, (free_bytes - grid_b - SLAB_RESERVE // 2 - 256) // plane_b)
        if margin < 4 * (k + 1):
            raise SystemExit(f"--config {config} on {n_gpus} GPUs: one {grid_b / 1e9:.0f} GB slab grid does not fit "
                             f"{free_bytes / 1e9:.0f} GB with a rolling margin; use more GPUs")
    else:
        margin = 0
    return {"grid": (gx, gy, gz), "planes_per_slab": planes, "grid_bytes_per_slab": grid_b, "plane_bytes": plane_b,
            "rolling": bool(use_rolling), "margin_estimate": int(margin),
            "scaling": "weak" if pre["grid"] is None else "strong"}


def slab_job_plan(args, visible: int):
    """Devices and exchange of the single-process multi-GPU job (no GPU call:
    `visible` from torch.cuda.device_count()); SystemExit with the reason when
    it cannot run here."""
    n = args.gpus
    if args.exchange not in ("nccl", "copy"):
        raise SystemExit(f"--exchange {args.exchange} is an N=1 interior-rank rehearsal; with --gpus {n} use nccl "
                         "(RCCL) or copy (device copies)")
    if args.share_device:
        if args.exchange != "copy":
            raise SystemExit("--share-device without a launcher needs --exchange copy (RCCL refuses two slabs on "
                             "one GPU)")
        return [0] * n, "copy"
    if visible < n:
        raise SystemExit(f"--gpus {n} needs {n} GPUs, {visible} visible: one process drives them all through the "
                         "C-ABI slab job (stencil_slab_*); rehearse it on one GPU with --share-device --exchange copy, "
                         "or launch one process per GPU with torch.distributed.run")
    return list(range(n)), "rccl" if args.exchange == "nccl" else "copy"


# ------------------------------------------------------------------ checks
def reference_plane_sums(spec, grid, sweeps, device, force_reduced=False, init="reference"):
    """Per-plane sums of the global grid after `sweeps` sweeps from the
    reference initial condition, computed on ONE grid on `device`.  When the
    global grid's two buffers do not fit, the size-independent form: the
    reference initial condition is the same in every interior plane, so after
    t sweeps a plane more than t planes from both z ends equals the middle
    plane of a (2t + 1)-plane grid, and a plane within t of an end equals the
    plane as far from that end of the small grid -- every plane's sum is
    checked, from a grid of 2t + 1 planes.  Returns (sums, how)."""
    import numpy as np
    import torch

    from stencil_amd.engine import JacobiEngine
    gnx, gny, gnz = grid
    free = torch.cuda.mem_get_info(device)[0]
    t = int(sweeps) * spec.radius
    full_b = 2.2 * gnx * gny * gnz * spec.elem_bytes
    if (full_b <= 0.9 * free and not force_reduced) or gnz <= 2 * t + 1:
        nzs = gnz
    elif init != "reference":
        raise RuntimeError("the size-independent check needs the z-uniform reference initial condition")
    else:
        nzs = 2 * t + 1
        if 2.2 * gnx * gny * nzs * spec.elem_bytes > 0.9 * free:
            raise RuntimeError(f"even the {nzs}-plane reference grid does not fit {free / 1e9:.0f} GB")
    ref = JacobiEngine(spec, gnx, gny, nzs, device=device)
    ref.reset(init, INIT_SEED)
    fin, _ = ref.iterate(sweeps)
    small = ref.plane_sums(fin)
    del ref, fin
    torch.cuda.empty_cache()
    if nzs == gnz:
        return small, "the global grid as one grid, same sweeps"
    z = np.arange(gnz)
    idx = np.where(z < t, z, np.where(z >= gnz - t, nzs - (gnz - z), t))
    return small[idx], (f"size-independent: every plane against a {nzs}-plane grid after the same {sweeps} sweeps "
                        f"(the reference initial condition is z-uniform: planes > {t} from both ends equal its "
                        "middle plane, the others its plane as far from the same end)")


def periodic_slab_check(spec, grid, sweeps, got, device, init="reference"):
    """A rehearsal's periodic slab (its halos its own faces) from the
    reference initial condition, which is z-uniform: every plane stays equal
    to every other (bitwise) and to the middle plane of a (2t + 1)-plane grid
    run as one grid for the same sweeps, which no z end reaches.  The second
    half is skipped (and said so) when that grid does not fit."""
    import numpy as np
    import torch
    if init != "reference":
        return {"skipped": "the periodic check needs the z-uniform reference initial condition"}
    gnx, gny, gnz = grid
    bits = got.view(np.uint64)
    out = {"planes": int(gnz), "sweeps": int(sweeps),
           "planes_differing_from_plane_0": int(np.count_nonzero(bits != bits[0]))}
    t = int(sweeps) * spec.radius
    need = 2.2 * gnx * gny * (2 * t + 1) * spec.elem_bytes
    if need > 0.8 * torch.cuda.mem_get_info(device)[0]:
        out["reference"] = f"z-uniformity only: the {2 * t + 1}-plane one-grid reference does not fit"
        out["bitwise_equal"] = out["planes_differing_from_plane_0"] == 0
        return out
    try:
        want, _ = reference_plane_sums(spec, (gnx, gny, 2 * t + 1), sweeps, device)
        mid = want[t:t + 1].view(np.uint64)[0]
        out["planes_differing"] = int(np.count_nonzero(bits != mid))
        out["bitwise_equal"] = out["planes_differing"] == 0
        out["reference"] = (f"every plane against the middle plane of a {2 * t + 1}-plane grid run as one grid on "
                            f"GPU {device} (no z end reaches it in {sweeps} sweeps)")
    except Exception as exc:  # a check, never the measurement
        out["error"] = f"{type(exc).__name__}: {exc}"[:300]
    return out


def global_grid_check(spec, grid, sweeps, got, device, init="reference"):
    """The multi-GPU job's per-plane sums `got` against the same sweeps of one
    grid on `device` (reference_plane_sums), bit for bit."""
    import numpy as np
    try:
        want, how = reference_plane_sums(spec, grid, sweeps, device, init=init)
        bad = int(np.count_nonzero(want.view(np.uint64) != got.view(np.uint64)))
        return {"planes": int(grid[2]), "sweeps": int(sweeps), "planes_differing": bad, "bitwise_equal": bad == 0,
                "reference": f"{how}, per-plane sums on GPU {device}"}
    except Exception as exc:  # a check, never the measurement
        return {"error": f"{type(exc).__name__}: {exc}"[:300]}


# ------------------------------------------------------------------- drivers
def main(argv=None):
    args = parse(argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if "WORLD_SIZE" in os.environ and world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    if world > 1:
        return main_rank_job(args, world, int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0")))
    if args.gpus > 1 or args.exchange in ("loopback", "nccl-self"):
        return main_slab_job(args)
    if args.config == "C1":
        return main_2d(args)
    return main_single(args)


def main_single(args):
    """N = 1: the whole grid on one GPU -- two grids, or (C3 / C4) ONE grid plus
    a rolling margin of spare planes (stencil_rolling_*)."""
    import torch

    from stencil_amd.engine import JacobiEngine, RollingGrid, StencilSpec
    pre = PRESETS[args.config]
    if pre["min_gpus"] > 1:
        slab_plan(args.config, 1, 0, args.n)  # raises the reason
    gnx, gny, gnz = global_grid(args.config, 1, args.n)
    spec = StencilSpec(dims=3, dtype=pre["dtype"], shape=pre["shape"], radius=1, order="naive", kernel=args.kernel)
    torch.cuda.set_device(0)
    rolling = args.config in ("C3", "C4")
    if rolling:
        free = torch.cuda.mem_get_info(0)[0]
        plane_b = RollingGrid.bytes_needed(spec, gnx, gny, 1, 64) - RollingGrid.bytes_needed(spec, gnx, gny, 1, 63)
        need = RollingGrid.bytes_needed(spec, gnx, gny, gnz, 8)
        shift = int(min(512, (free - need - (2 << 30)) // plane_b + 8))
        if shift < 16:
            raise SystemExit(f"--config {args.config} on one GPU needs {need / GiB:.0f} GiB + a margin; "
                             f"{free / GiB:.0f} GiB free")
        grid = RollingGrid(spec, gnx, gny, gnz, shift, device=0)
        grid.reset(args.init, INIT_SEED)
        kname = "temporalk"
        sweeps_per_launch = grid.sweeps_per_pass
        grid.iterate(args.warmup)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        dev_ms, kernel_launches = grid.iterate(args.steps, stream=torch.cuda.current_stream(), timed=True)[1:]
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
        kernel_ms_total = dev_ms
        cells_per_launch = float(gnx) * gny * gnz  # charged per pass of K sweeps over the whole grid
        extra = dict(settle_config(0, 0.0, "none beyond the warm-up sweeps"),
                     rolling={"shift_planes": shift, "launch_planes": shift - sweeps_per_launch,
                              "launches": kernel_launches, "grid_bytes": grid.bytes})
        kernels_per_launch = kernel_launches / max(1.0, args.steps / sweeps_per_launch)
        del grid
        torch.cuda.empty_cache()  # the copy-kernel calibration needs 2 GiB
        parallelism = ("1 GPU, ONE resident grid + a rolling margin of %d planes (stencil_rolling_iterate: "
                       "%d-plane launches, bitwise the two-grid job)" % (shift, shift - sweeps_per_launch))
        timing = "hipEvents of stencil_rolling_iterate over the timed region"
        key = "C3_rolling_4096" if args.config == "C3" else f"{args.config}_rolling"
    else:
        eng = JacobiEngine(spec, gnx, gny, gnz, device=0)
        # where the grids' pages land moves the launch by up to 8 %: the
        # engine picks the fastest of a few placements (untimed; §9.1j)
        # (candidates within a quarter of the free memory: C2 gets 16; the 70 GB grids of NS / C5 none --
        # measured with one extra pair each, their two placements ran within 0.6 %, r05ap)
        placement = eng.place(trials=args.placements) if args.placements > 1 else None
        eng.reset(args.init, INIT_SEED)
        kernel_id = eng.plan(12)[1]
        kname = {1: "direct", 2: "zmarch", 3: "temporal2", 4: "temporalk"}[kernel_id]
        if spec.shape == "box" and kname in ("temporal2", "temporalk"):
            kname = "boxk"  # the box's fused family (kernels_boxk.hip)
        sweeps_per_launch = eng.fuse_steps
        # settle the one-time per-shape choice (packed vs equal z-chunks, timed
        # on the first launch of a shape) outside the timed region whatever W
        # is: one fused launch a -> b, grid a unchanged
        settle = eng.prepare()
        eng.iterate(args.warmup)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        _, kernel_ms_total = eng.iterate(args.steps, stream=torch.cuda.current_stream(), timed=True)
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
        kernel_launches = eng.plan(args.steps)[0]
        cells_per_launch = float(gnx) * gny * gnz
        extra, kernels_per_launch = settle_config(settle["launches"], settle["device_ms"],
                                                  "stencil_prepare2: the schedule trial + ~25 ms of the job's own "
                                                  "launch (a -> b, grid a unchanged)"), 1.0
        if placement is not None:
            extra["placement"] = dict(placement, basis="JacobiEngine.place: candidate grid pairs allocated while "
                                                       "the earlier ones are held, one fused launch timed on each "
                                                       "(untimed region), the fastest kept")
        parallelism = "1 GPU, one process, the whole grid (no decomposition)"
        timing = "hipEvents of stencil_iterate over the timed region"
        key = f"3d7pt_fp64_{args.n}cube_per_gpu" if args.config == "C2" else f"{args.config}_slab_{gnz}"
        # calls of >= 256 sweeps run at the package power limit and take the XCD-patch packed tables
        # (DESIGN.md §5.2, §6): a separate PMC traffic entry
        long_job = args.steps >= SUSTAINED_SWEEPS
        extra["work_order"] = ("XCD-patch packed z-chunk tables (one stencil_iterate call of >= %d sweeps)" if long_job
                               else "tile-major packed z-chunk tables (a call of < %d sweeps)") % SUSTAINED_SWEEPS
        if long_job:
            key += "_long"
        del eng
    # device time per `sweeps_per_launch` sweeps, charged pro rata (with K = 4
    # a 1000-step job is 250 fused launches; a K that does not divide the step
    # count adds a remainder pair / single sweep)
    launch_ms = kernel_ms_total * sweeps_per_launch / max(1, args.steps)
    report(args, pre, spec, kname, (gnx, gny, gnz), 1, elapsed, launch_ms, cells_per_launch, sweeps_per_launch,
           kernel_launches, parallelism, rounds=None, launch_timing=timing, workload_key=key, local=0, check=None,
           cpu=True, extra_config=extra, kernels_per_launch=kernels_per_launch)


def main_2d(args):
    """BASELINE config 1, the reference's own case (run.sh: -s 1024 -i 100):
    2D 5-point 1024^2 fp64 through AUTO (tb2ds, K sweeps per launch).  The
    grid is 16.8 MB: launch- and barrier-latency bound, not HBM bound -- the
    line reports us per sweep beside the Gcell/s, and the CPU baseline runs
    the whole config on the host (1 thread and all cores)."""
    import torch

    from stencil_amd.engine import JacobiEngine, StencilSpec
    pre = PRESETS["C1"]
    nx, ny, _ = pre["grid"]
    spec = StencilSpec(dims=2, dtype=pre["dtype"], shape="star", radius=1, order="naive", kernel=args.kernel)
    torch.cuda.set_device(0)
    eng = JacobiEngine(spec, nx, ny, 1, device=0)
    eng.reset(args.init, INIT_SEED)
    launches, _ = eng.plan(args.steps)
    settle = eng.prepare()  # untimed settle (a -> b, grid a unchanged): ~25 ms of launches, as every other driver
    eng.iterate(args.warmup)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    _, dev_ms = eng.iterate(args.steps, stream=torch.cuda.current_stream(), timed=True)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    sweeps_per_launch = args.steps / max(1, launches)
    launch_ms = dev_ms / max(1, launches)
    report(args, pre, spec, "tb2ds", (nx, ny, 1), 1, elapsed, launch_ms, float(nx) * ny, sweeps_per_launch,
           launches, "1 GPU, one process, the whole grid", rounds=None,
           launch_timing="hipEvents of stencil_iterate over the timed region", workload_key="C1_2d_1024",
           local=0, check=None, cpu=True,
           extra_config=dict(settle_config(settle["launches"], settle["device_ms"],
                                           "stencil_prepare2: ~25 ms of the job's own K-sweep launch"),
                             us_per_sweep_device=round(dev_ms * 1e3 / max(1, args.steps), 3),
                             bound="launch + per-sweep barrier latency (a 16.8 MB grid; DESIGN.md §5, §9.3)"),
           cpu_full=True)


def _slab_spec(args, pre):
    from stencil_amd.engine import StencilSpec
    return StencilSpec(dims=3, dtype=pre["dtype"], shape=pre["shape"], radius=1, order="naive", kernel=args.kernel)


SETTLE_MS = 25.0  # as stencil_prepare: the GPU's clock settles over ~15 ms of heavy launches after idling


def settle_config(launches, ms, what):
    """What ran before the timed region besides the W warm-up steps (the
    line's `warmup` counts only those): the settle's launches (or rounds) and
    their time, DESIGN.md §6."""
    return {"settle_launches": int(launches), "settle_ms": round(float(ms), 3), "settle": what}


def settle_rounds(job, k, rounds=None):
    """Untimed rounds for about SETTLE_MS (at most 64 rounds): `rounds` of
    them, or -- one process -- as many as one timed round says fit.  Returns
    (sweeps run -- the check counts them --, rounds, host ms).  Ranks of one
    job must run the same rounds (every round exchanges halos): they pass
    `rounds` from settle_rounds_for(), which depends only on the global
    problem."""
    if rounds is None:
        ms = job.run(k)
        n = int(min(64, SETTLE_MS / ms)) if ms > 0 else 0
        if n:
            ms += job.run(n * k)
        return k * (n + 1), n + 1, ms
    ms = job.run(rounds * k) if rounds else 0.0
    return rounds * k, rounds, ms


def settle_rounds_for(grid, world, k, rate_gcell=1000.0):
    """The same settle round count on every rank: SETTLE_MS at an assumed
    rate_gcell per GPU, 1 to 64 rounds."""
    gnx, gny, gnz = grid
    round_ms = float(gnx) * gny * gnz / world * k / (rate_gcell * 1e9) * 1e3
    return int(max(1, min(64, round(SETTLE_MS / max(round_ms, 1e-6)))))


def rank_job_run(args, world, rank, device, spec, grid, rolling, uid, lib=None, barrier=None):
    """The per-rank body of the rank-mode job: build this rank's slab, warm
    up, time exactly args.steps sweeps, time the compute launches of extra
    rounds, collect this rank's per-plane sums.  Returns a dict (no
    torch.distributed call: `barrier` is the caller's)."""
    from stencil_amd.engine import SlabJob
    gnx, gny, gnz = grid
    job = SlabJob(spec, gnx, gny, gnz, [device], rank=(world, rank, uid), rolling=rolling, margin=0, lib=lib)
    try:
        if args.slab_timeout_ms:
            job.set_timeout(args.slab_timeout_ms)
        info = job.info(0)
        roll = job.rolling_info()
        k = info["sweeps_per_round"]
        job.fill_initial(args.init, INIT_SEED)
        sweeps = k + 1 + args.warmup
        job.run(k + 1)  # a full and a remainder round: both launch paths' one-time costs
        if barrier:
            barrier()
        settled = settle_rounds(job, k, settle_rounds_for(grid, world, k))  # the same rounds on every rank
        sweeps += settled[0]
        job.run(args.warmup)
        if barrier:
            barrier()
        elapsed = job.run(args.steps) * 1e-3  # this rank's rounds, its device synchronised at both ends
        sweeps += args.steps
        extra = k * max(4, min(args.steps // max(1, k), 8))
        job.kernel_timing(True)
        job.run(extra)
        kt = job.kernel_time()
        xt = dict(job.exchange_time(), round_info=job.round_info(), budget=job.exchange_budget())
        job.kernel_timing(False)
        sweeps += extra
        sums = None if args.no_check else job.plane_sums()[info["first"]:info["first"] + info["planes"]].copy()
        return {"info": info, "rolling": roll, "k": k, "elapsed": elapsed, "kt": kt, "xt": xt, "sweeps": sweeps,
                "sums": sums, "settle": settled}
    finally:
        job.close()


def main_rank_job(args, world, rank, local, lib=None, check_device=None):
    """One process per GPU (torch.distributed.run) through the C-ABI rank-mode
    slab job (stencil_slab_unique_id / stencil_slab_create_rank,
    csrc/slab_core.hpp): each rank builds and runs only its own z-slab, the
    halos over RCCL between the ranks' slabs, face-signalled rounds (rolling
    passes for slabs whose two grids do not fit) -- the shape of an
    MPI-per-rank launch.  torch.distributed (gloo, host side only) hands rank
    0's RCCL id to the others and carries the barriers, the max-over-ranks
    time and the per-plane sums of the check; it moves no halo data.  `lib`:
    the library running the slabs (the CPU tests pass the fake device; then
    nothing here touches a GPU and the check is the caller's)."""
    import numpy as np
    import torch
    import torch.distributed as dist

    from stencil_amd.engine import SlabJob
    pre = PRESETS[args.config]
    on_gpu = lib is None
    if args.exchange != "nccl" or args.share_device:
        raise SystemExit("under torch.distributed.run the halos go over RCCL between distinct GPUs "
                         "(--exchange nccl, no --share-device); rehearse on one GPU without a launcher")
    spec = _slab_spec(args, pre)
    dist.init_process_group("gloo")
    try:
        # one plan for every rank: the least free HBM of any rank decides
        # whether slabs keep two grids or roll one
        free = torch.tensor([torch.cuda.mem_get_info(local)[0] if on_gpu else (1 << 40)], dtype=torch.float64)
        dist.all_reduce(free, op=dist.ReduceOp.MIN)
        plan = slab_plan(args.config, world, int(free.item()), args.n, args.rolling)
        uid = [SlabJob.unique_id(lib=lib) if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        if on_gpu:
            torch.cuda.set_device(local)
        res = rank_job_run(args, world, rank, local, spec, plan["grid"], plan["rolling"], uid[0], lib=lib,
                           barrier=dist.barrier)
        t = torch.tensor([res["elapsed"]], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        # every rank's exchange times (its transfers over RCCL, and how much of
        # them ran beside its own launches) for the line
        x, ri, b = res["xt"], res["xt"]["round_info"], res["xt"]["budget"]
        xrow = torch.tensor([x["transfer_ms"], x["beside_ms"], float(x["exchanges"]), float(ri["gated"]),
                             float(ri["confined"]), float(b["cus_per_xcd"]), float(b["alt_cus_per_xcd"]),
                             b["round_ms"], b["alt_round_ms"]], dtype=torch.float64)
        xrows = [torch.zeros_like(xrow) for _ in range(world)]
        dist.all_gather(xrows, xrow)
        xts = [{"transfer_ms": float(r[0]), "beside_ms": float(r[1]), "exchanges": int(r[2]),
                "round_info": {"form": ri["form"], "gated": bool(r[3]), "confined": bool(r[4])},
                "budget": {"cus_per_xcd": int(r[5]), "alt_cus_per_xcd": int(r[6]), "round_ms": round(float(r[7]), 4),
                           "alt_round_ms": round(float(r[8]), 4)}} for r in xrows]
        got = None
        if not args.no_check:
            width = plan["grid"][2] // world + 1
            buf = torch.zeros(width, dtype=torch.float64)
            buf[:len(res["sums"])] = torch.from_numpy(res["sums"])
            parts = [torch.zeros_like(buf) for _ in range(world)]
            dist.all_gather(parts, buf)
            counts = [partition(plan["grid"][2], world, r)[1] for r in range(world)]
            got = np.concatenate([parts[r].numpy()[:counts[r]] for r in range(world)])
        check = None
        if rank == 0 and got is not None and on_gpu:
            check = global_grid_check(spec, plan["grid"], res["sweeps"], got, local, init=args.init)
        dist.barrier()
    finally:
        dist.destroy_process_group()
    if rank == 0:
        kt = res["kt"]
        roll = res["rolling"]
        kname = "boxk" if spec.shape == "box" else "temporalk"
        parallelism = (f"z-slab x{world}, one process per GPU (torch.distributed.run) through the C-ABI rank-mode "
                       "slab job (stencil_slab_create_rank), RCCL send/recv between the ranks' slabs" +
                       (f"; ONE grid per slab + a rolling margin of {roll['margin']} planes" if roll["margin"] else ""))
        form = _lib_forms()[kt["form"]]
        line = report(args, pre, spec, kname, plan["grid"], world, elapsed, kt["total_ms"] / max(1, kt["launches"]),
                      float(kt["cells_per_launch"]), res["k"], kt["launches"], parallelism,
                      rounds=form, launch_timing=f"hipEvents around rank 0's {form} of extra rounds after the timed "
                                                 "region",
                      workload_key=(f"3d7pt_fp64_{args.n}cube_per_gpu_slab_x{world}" if args.config == "C2" else
                                    f"{args.config}_slab_{res['info']['planes']}_x{world}"),
                      local=local, check=check if on_gpu else {"skipped": "no GPU (CPU rehearsal)"}, cpu=False,
                      kernels_per_launch=float(max(1, roll["launches_per_pass"])) if roll["margin"] else 1.0,
                      extra_config=dict(settle_config(res["settle"][1], res["settle"][2],
                                                      "untimed full rounds (the same count on every rank), after one "
                                                      "full and one remainder round"),
                                        slab_plan={k: v for k, v in plan.items() if k != "grid"}),
                      calibrate=on_gpu, emit=on_gpu, exchange=exchange_summary(xts, "rank"))
        return line, got, res
    return None, got, res


def main_slab_job(args):
    """Without a launcher: ONE process drives N GPUs through the C-ABI slab job
    (stencil_slab_create/run/plane_sums, csrc/slab_core.hpp): z-slabs, one per
    GPU, RCCL send/recv from one host thread, face-signalled rounds -- the
    shape of the reference's one spawn/join of its whole decomposed job
    (src/stencil/stencil.cpp:34-53).  At N = 1 with --exchange loopback /
    nccl-self: one periodic slab (its halos are its own faces) -- an interior
    rank's rounds on one GPU.  Same JSON line as the per-process driver; the
    roofline from hipEvents on slab 0's compute stream over extra rounds after
    the timed region; multi_gpu_check against one grid on GPU 0."""
    import torch

    from stencil_amd.engine import SlabJob
    pre = PRESETS[args.config]
    loop = args.gpus == 1 and args.exchange in ("loopback", "nccl-self")
    if loop:
        devices, exchange = [0], ("copy" if args.exchange == "loopback" else "rccl")
    else:
        devices, exchange = slab_job_plan(args, torch.cuda.device_count())
    n_gpus = args.gpus
    free = torch.cuda.mem_get_info(0)[0]
    shared = len(set(devices)) < len(devices)
    # slabs sharing GPU 0 share its memory too
    plan = rank_plan = None
    if args.rank_of:
        # one interior rank of the N-GPU job: the N-way plan (per-GPU memory =
        # this GPU's), then that rank's slab alone, its halos its own faces
        rank_plan = slab_plan(args.config, args.rank_of, free, args.n, args.rolling)
        gnx, gny, gz = rank_plan["grid"]
        plan = dict(rank_plan, grid=(gnx, gny, rank_plan["planes_per_slab"]))
    else:
        plan = slab_plan(args.config, n_gpus, free // (n_gpus if shared else 1), args.n, args.rolling)
    spec = _slab_spec(args, pre)
    gnx, gny, gnz = plan["grid"]
    job = SlabJob(spec, gnx, gny, gnz, devices, exchange=exchange, periodic=loop, rolling=plan["rolling"], margin=0)
    if args.slab_timeout_ms:
        job.set_timeout(args.slab_timeout_ms)
    job.fill_initial(args.init, INIT_SEED)
    k = job.info(0)["sweeps_per_round"]
    roll = job.rolling_info()
    # one full round and one shorter remainder round before the timed region:
    # the one-time costs of both launch paths (schedule trials, first launches)
    sweeps = k + 1 + args.warmup
    job.run(k + 1)
    settled = settle_rounds(job, k)
    sweeps += settled[0]
    job.run(args.warmup)
    elapsed = job.run(args.steps) * 1e-3  # host wall time, every device synchronised at both ends
    sweeps += args.steps
    extra = k * max(4, min(args.steps // max(1, k), 8))
    job.kernel_timing(True)
    job.run(extra)
    kt = job.kernel_time()
    xt = dict(job.exchange_time(), round_info=job.round_info(), budget=job.exchange_budget())
    job.kernel_timing(False)
    sweeps += extra
    sums = job.plane_sums() if not args.no_check else None
    job.close()
    if sums is None:
        check = None
    elif loop:
        check = periodic_slab_check(spec, plan["grid"], sweeps, sums, 0, init=args.init)
    else:
        check = global_grid_check(spec, plan["grid"], sweeps, sums, 0, init=args.init)
    kname = "boxk" if spec.shape == "box" else "temporalk"
    form = _lib_forms()[kt["form"]]
    if loop:
        parallelism = ("1 GPU rehearsing an interior rank" +
                       (f" of the {args.rank_of}-GPU job (its {gnz}-plane slab of the "
                        f"{'x'.join(str(v) for v in rank_plan['grid'])} grid)" if args.rank_of else "") +
                       ": one periodic slab whose halos are its own faces, " +
                       ("device copies" if exchange == "copy" else "RCCL send/recv to itself") +
                       " (C-ABI slab job)" +
                       (f"; ONE grid + a rolling margin of {roll['margin']} planes" if roll["margin"] else ""))
    else:
        where = "GPU 0 shared by every slab (rehearsal)" if args.share_device else f"{n_gpus} GPUs"
        parallelism = (f"z-slab x{n_gpus}, ONE process driving {where} through the C-ABI slab job (stencil_slab_*), " +
                       ("RCCL send/recv (ncclCommInitAll)" if exchange == "rccl" else "device-copy halos") +
                       (f"; ONE grid per slab + a rolling margin of {roll['margin']} planes" if roll["margin"] else ""))
    report(args, pre, spec, kname, plan["grid"], n_gpus, elapsed, kt["total_ms"] / max(1, kt["launches"]),
           float(kt["cells_per_launch"]), k, kt["launches"], parallelism, rounds=form,
           launch_timing=f"hipEvents around slab 0's {form} of extra rounds after the timed region",
           workload_key=(f"3d7pt_fp64_{args.n}cube_per_gpu_slab_x{n_gpus}" if args.config == "C2" else
                         f"{args.config}_slab_{gnz // n_gpus}_x{args.rank_of or n_gpus}") + ("_loop" if loop else ""),
           local=0, check=check if n_gpus > 1 else None, cpu=False,
           kernels_per_launch=float(max(1, roll["launches_per_pass"])) if roll["margin"] else 1.0,
           extra_config=dict({"slab_plan": {k2: v for k2, v in plan.items() if k2 != "grid"}},
                             **settle_config(settled[1], settled[2], "untimed full rounds after one full and one "
                                                                    "remainder round"),
                             **({"rehearsal_check": check} if loop else {}),
                             **({"rank_of": args.rank_of, "global_grid": list(rank_plan["grid"])} if args.rank_of
                                else {})),
           exchange=exchange_summary([xt], "slab 0"))


def exchange_summary(xts, who):
    """The `exchange` object of a slab line: per rank (or slab 0), the mean
    transfer time per timed round on its exchange stream and the fraction of
    it that ran beside the same round's timed launches
    (stencil_slab_exchange_time)."""
    rows = []
    for x in xts:
        n = max(1, x["exchanges"])
        row = {"transfer_ms_per_round": round(x["transfer_ms"] / n, 4),
               "beside_launch_frac": round(x["beside_ms"] / x["transfer_ms"], 3) if x["transfer_ms"] > 0 else None,
               "rounds": x["exchanges"]}
        ri, b = x.get("round_info"), x.get("budget")
        if ri is not None:
            # halo-gated: the launches never wait for the exchange stream (stencil_slab_round_info)
            row["halo_gated"], row["confined"] = ri["gated"], ri["confined"]
        if b is not None and ri is not None and ri["confined"]:
            # the exchange's CU budget chosen from the tuning rounds (stencil_slab_exchange_budget)
            row["cu_budget"] = dict(b, chosen=b["cus_per_xcd"])
        rows.append(row)
    fracs = [r["beside_launch_frac"] for r in rows if r["beside_launch_frac"] is not None]
    return {"basis": f"hipEvents on {who}'s exchange stream over the timed extra rounds: from the end of the face "
                     "wait (or face launches) to the end of the RCCL send/recv; beside = the part that ran while the "
                     "same round's timed launches ran",
            "max_transfer_ms_per_round": max(r["transfer_ms_per_round"] for r in rows) if rows else None,
            "min_beside_launch_frac": min(fracs) if fracs else None,
            "per_rank" if len(rows) > 1 else "slab0": rows if len(rows) > 1 else rows[0]}


def report(args, pre, spec, kname, grid, n_gpus, elapsed, launch_ms, cells_per_launch, sweeps_per_launch,
           kernel_launches, parallelism, rounds, launch_timing, workload_key, local, check, cpu, extra_config=None,
           kernels_per_launch=1.0, calibrate=True, emit=True, cpu_full=False, exchange=None):
    """Print the one JSON line.  Roofline of the dominant kernel: one launch
    advances its cells by `sweeps_per_launch` fused sweeps; its compulsory HBM
    traffic is one read plus one write of those cells (2 * sizeof(T) per cell,
    whatever K is): `achieved` = compulsory bytes / mean launch time, a true
    fraction of the HBM peak.  The per-sweep algorithmic figure of SURVEY
    8(d) (2 * sizeof(T) per cell-UPDATE, K per cell per launch) is
    `effective_GBps`.  kernels_per_launch: kernel launches per charged
    "launch" (a rolling pass runs several z-range launches; the PMC table
    holds bytes per kernel launch)."""
    gnx, gny, gnz = grid
    total_updates = float(gnx) * gny * gnz * args.steps
    gcell = total_updates / elapsed / 1e9
    bytes_per_update = 2 * spec.elem_bytes
    compulsory_bytes_launch = cells_per_launch * bytes_per_update
    alg_bytes_launch = compulsory_bytes_launch * sweeps_per_launch
    achieved = compulsory_bytes_launch / (launch_ms * 1e-3) / 1e9 if launch_ms > 0 else 0.0
    effective = alg_bytes_launch / (launch_ms * 1e-3) / 1e9 if launch_ms > 0 else 0.0
    traffic, traffic_entry = load_traffic(workload_key, kname)
    if traffic:
        traffic = traffic * kernels_per_launch
    desc = pre["desc"].format(n=args.n)
    gdesc = f"{gnx}x{gny}" + (f"x{gnz}" if pre.get("dims", 3) == 3 else "")
    out = {
        "metric": METRIC,
        "value": round(gcell, 3),
        "unit": "Gcell-updates/s",
        "n_gpus": n_gpus,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed * 1e3 / args.steps, 5),
        "higher_is_better": True,
        "scaling": "weak" if pre["grid"] is None else "strong",
        "vs_baseline": None,
        "dtype": "f64" if spec.dtype == "fp64" else "f32",
        "data": ("synthetic: the reference initial condition (x-ghost faces 1, everything else 0)"
                 if getattr(args, "init", "reference") == "reference" else
                 "synthetic: a developed field -- uniform random [0,1) interior (splitmix64), x-ghost faces 1"),
        "config": {
            "workload": f"{desc} (global {gdesc}), one step = one sweep",
            "grid": [gnx, gny, gnz] if pre.get("dims", 3) == 3 else [gnx, gny],
            "kernel": kname,
            "parallelism": parallelism,
            # SURVEY 8(d)'s algorithmic bytes (2 x sizeof(T) per cell-update) at the
            # whole job's rate: K fused sweeps per launch put it above the HBM
            # peak; the roofline's `achieved` is the HBM-side (compulsory) figure
            "effective_GBps_whole_job": round(gcell * bytes_per_update, 1),
            "rounds": rounds,
            **library_info(),
        },
        "roofline": {
            "bound": "hbm",
            "kernel": kname,
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBPS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBPS, 4),
            "traffic": traffic,
            "bytes_basis": "compulsory: one read + one write of the launch's cells (2 x %d B per cell), "
                           "%g fused sweeps per launch" % (spec.elem_bytes, sweeps_per_launch),
            "compulsory_bytes_per_launch": compulsory_bytes_launch,
            "effective_GBps": round(effective, 1),
            "effective_basis": "SURVEY 8(d) algorithmic: 2 x %d B per cell-update x %g sweeps per launch"
                               % (spec.elem_bytes, sweeps_per_launch),
            "alg_bytes_per_launch": alg_bytes_launch,
            "mean_launch_ms": round(launch_ms, 5),
            "launches": kernel_launches,
            "launch_timing": launch_timing,
        },
    }
    if extra_config:
        out["config"].update(extra_config)
    if exchange is not None:
        out["exchange"] = exchange
    if n_gpus > 1:
        out["multi_gpu_check"] = check if check is not None else {"skipped": "--no-check"}
        out["multi_gpu_status"] = ("the rounds' code (csrc/slab_core.hpp) is bitwise-tested at world 2/3 on the CPU "
                                   "(tests/test_slab_core_cpu.py) and as slabs sharing one GPU; this line's "
                                   "multi_gpu_check is its check on distinct GPUs")
    if traffic_entry is not None:
        out["roofline"]["traffic_source"] = {k: traffic_entry.get(k) for k in
                                             ("source", "kernel", "kernel_source_sha", "fresh")}
    if traffic and launch_ms > 0:
        # the PMC-measured bytes of one launch (L2->fabric: HBM plus
        # Infinity-Cache hits) over its live mean duration; traffic well
        # above the compulsory bytes = re-reads (tile rings, halos)
        out["roofline"]["traffic_GBps"] = round(traffic / (launch_ms * 1e-3) / 1e9, 1)
        out["roofline"]["traffic_frac"] = round(out["roofline"]["traffic_GBps"] / HBM_PEAK_GBPS, 4)
    if calibrate:
        try:
            from stencil_amd.engine import copy_bandwidth
            out["roofline"]["copy_kernel_GBps"] = round(copy_bandwidth(1 << 30, reps=10, device=local), 1)
        except Exception as exc:  # calibration only
            out["roofline"]["copy_kernel_GBps"] = f"unavailable: {exc}"
    if cpu and not args.no_cpu_baseline:
        cb = dict(dtype=spec.dtype, shape=spec.shape)
        if cpu_full:  # the whole 2D config on the host (C1: 1024^2 x steps)
            n = gnx
            out["cpu_baseline"] = cpu_baseline(n, args.cpu_seconds, dims=2, iters_cap=args.steps, **cb)
            out["cpu_baseline_all_cores"] = cpu_baseline(n, args.cpu_seconds / 2, threads=host_threads(), dims=2,
                                                         iters_cap=args.steps, **cb)
        else:
            n = min(args.n, 512)
            out["cpu_baseline"] = cpu_baseline(n, args.cpu_seconds, **cb)
            # the same loop with OpenMP over the host's cores too
            out["cpu_baseline_all_cores"] = cpu_baseline(n, args.cpu_seconds / 2, threads=host_threads(), **cb)
    else:
        out["cpu_baseline"] = None
    if emit:
        _JSON_OUT.write(json.dumps(out) + "\n")
        _JSON_OUT.flush()
    return out


# The one JSON line goes to the process's original stdout; everything else
# written to fd 1 while the bench runs -- RCCL prints a version banner there
# when a communicator is created -- is sent to stderr (see __main__ below).
_JSON_OUT = sys.stdout


def _route_stdout_to_stderr():
    global _JSON_OUT
    sys.stdout.flush()
    _JSON_OUT = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)


if __name__ == "__main__":
    _route_stdout_to_stderr()
    main()
