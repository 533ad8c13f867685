#!/usr/bin/env python3
"""Benchmark: 3D 7-point fp64 Jacobi (BASELINE.json metric, config 2 size per GPU).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config C2|C3|C4|C5|NS]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

Multi-GPU drivers, same job, same JSON line:
  * one process per GPU (launched by torch.distributed.run; WORLD_SIZE set):
    the C-ABI rank-mode slab job (stencil_slab_create_rank: each rank its own
    slab, RCCL between the ranks); --driver python (or a rehearsal transport)
    runs stencil_amd/slab.py over torch.distributed instead;
  * --gpus N without a launcher (WORLD_SIZE unset): ONE process drives the N
    GPUs through the C-ABI slab job (stencil_slab_*, csrc/slab.hip; RCCL
    ncclCommInitAll), the shape of the reference's single spawn/join of its
    whole decomposed job (src/stencil/stencil.cpp:34-53).

--config picks another BASELINE.json config as the workload (C3: 4096^3 fp32,
C4: 2048x2048x4096 fp64, C5: 2048^3 27-point fp64), its global grid z-slab
split over the N ranks; the default C2 is the metric's own config.

One step = one Jacobi sweep of the whole grid.  At N=1 the workload is
BASELINE config 2 (512^3 interior, fp64, 7-point star; the default K=1000 is
exactly its 1000 iterations).  At N>1 every rank owns a 512^3 Z-slab of a
512 x 512 x 512N grid (weak scaling) and exchanges K halo planes with each
neighbour per round of K fused sweeps (K = 4: the strip-layout K-step
kernel) over RCCL, the boundary planes' launch and the send/recv overlapped
with the interior launch on a second stream.

Rank 0 prints one JSON line with the whole-job rate, the live roofline of the
dominant kernel (algorithmic bytes per launch / average launch time from HIP
events on the kernel's own stream), and a bounded CPU baseline (the oracle's
single-thread restatement of the reference's naive sweep, N=1 only).
"""
from __future__ import annotations

import argparse
import dataclasses
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

METRIC = "Gcell-updates/s + achieved HBM GB/s vs roofline, 7-pt fp64 Jacobi, 1/2/4/8 GPUs"
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (/opt/skills/guides/MI355X_MICROARCH.md)


# BASELINE.json configs as bench workloads.  C2 (the default, the metric's
# config) is weak-scaled: n^3 per GPU.  C3-C5 are the configs' global grids,
# z-slab split over the ranks (strong scaling); at N = 1, C3 and C4 keep ONE
# resident grid (two would need 2 x 275 GB / 2 x 137 GB).
PRESETS = {
    "C2": dict(dtype="fp64", shape="star", grid=None, min_gpus=1,
               desc="BASELINE config 2: 3D 7-point fp64 Jacobi, {n}^3 interior per GPU"),
    # C3 on one GPU: ONE resident grid + a rolling margin (stencil_rolling_*),
    # since two grids are 2 x 279 GB
    "C3": dict(dtype="fp32", shape="star", grid=(4096, 4096, 4096), min_gpus=1,
               desc="BASELINE config 3: 3D 7-point fp32 Jacobi, 4096^3"),
    # C4 on one GPU likewise (one 137 GB grid + a margin)
    "C4": dict(dtype="fp64", shape="star", grid=(2048, 2048, 4096), min_gpus=1,
               desc="BASELINE config 4: 3D 7-point fp64 Jacobi, 2048x2048x4096"),
    "C5": dict(dtype="fp64", shape="box", grid=(2048, 2048, 2048), min_gpus=1,
               desc="BASELINE config 5: 3D 27-point fp64 stencil, 2048^3, temporal blocking (4 sweeps per launch, "
                    "deeper than the config's 2; bitwise the same result)"),
    # north_star's 4096^3 fp64 needs 2 x 550 GB; its largest single-GPU
    # proxy is 2048^3 fp64: 2 x 70 GB with ghosts and padding
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
}


def kernel_source_sha(kname: str):
    import hashlib
    h = hashlib.sha256()
    for rel in KERNEL_SOURCES.get(kname, ()):
        with open(os.path.join(HERE, rel), "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16] if kname in KERNEL_SOURCES else None


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--config", default="C2", choices=sorted(PRESETS),
                    help="workload (default C2, the metric's config; C3-C5 split a global grid over the ranks)")
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--n", type=int, default=512, help="per-GPU cube edge (config 2: 512)")
    ap.add_argument("--kernel", default="auto", choices=["auto", "direct", "zmarch", "temporal2"])
    ap.add_argument("--no-overlap", action="store_true")
    ap.add_argument("--no-signal", action="store_true",
                    help="multi-GPU rounds as separate boundary/interior launches (no face counters)")
    ap.add_argument("--face-signal", action="store_true",
                    help="face-signalled rounds gated by hipStreamWaitValue64 on a signal word, not the wait kernel")
    ap.add_argument("--exchange", default="nccl", choices=["nccl", "host", "loopback", "nccl-self", "copy"],
                    help="halo transport: RCCL P2P (default) or host-staged gloo (single-GPU rehearsal only); "
                         "without a launcher, copy = device copies between the slabs (hipMemcpyPeerAsync)")
    ap.add_argument("--share-device", action="store_true",
                    help="rehearsal: every rank / slab uses GPU 0 (needs --exchange host, or copy without a launcher)")
    ap.add_argument("--driver", default="auto", choices=["auto", "cabi", "python"],
                    help="under torch.distributed.run: the C-ABI rank-mode slab job (auto/cabi) or the Python slab "
                         "driver over torch.distributed (python; auto picks it for the rehearsal transports)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="budget of the CPU baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-check", action="store_true",
                    help="N>1: skip the bitwise check against the global grid run as one grid on rank 0")
    ap.add_argument("--allow-debug-library", action="store_true",
                    help="bench even when an experiment knob (a STENCIL_* variable the product ignores) is set, "
                         "i.e. on libstencil_hip_debug.so; the JSON line names the library and the knobs either way")
    args = ap.parse_args()
    from stencil_amd import _lib
    if _lib.debug_knobs_requested() and not args.allow_debug_library:
        knobs = sorted(k for k in os.environ if k.startswith("STENCIL_") and k not in _lib.API_KNOBS)
        raise SystemExit(f"experiment knobs set ({', '.join(knobs)}): this would bench libstencil_hip_debug.so; "
                         "unset them or pass --allow-debug-library")
    return args


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


def cpu_baseline(n: int, budget_s: float, threads: int = 1, dtype: str = "fp64", shape: str = "star"):
    """The oracle (port of check_result's loop, stencil.cpp:94-131, generalised
    to 3D) on the host over a bounded number of sweeps of an n^3 grid of the
    workload's stencil: single-threaded like the reference's own CPU path, or
    with OpenMP over `threads` cores (identical per-cell arithmetic,
    bitwise-equal result)."""
    from oracle import binding as ob
    p = ob.problem(3, dtype, shape, 1, "naive", n, n, n)
    t1 = ob.timed_run(p, 1, threads=threads)
    iters = max(1, min(200, int(budget_s / max(t1, 1e-6))))
    t = ob.timed_run(p, iters, threads=threads)
    cells = float(n) ** 3 * iters
    who = "1 host thread" if threads == 1 else f"{threads} host threads (OpenMP)"
    pts = "7-point" if shape == "star" else "27-point"
    return {"value": round(cells / t / 1e9, 4), "unit": "Gcell-updates/s", "cores": threads, "kind": "port",
            "sample": f"oracle/ naive sweep, {n}^3 {dtype} {pts}, {iters} sweeps from the reference initial "
                      f"condition, {t:.1f} s on {who}"}


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


def verify_slabs(eng, slab, spec, grid, world, rank, sweeps, on_gpu, local):
    """End-to-end check of a multi-GPU run, after the timed region: every
    rank's per-plane sums (fp64, one deterministic sum per plane) gathered on
    rank 0 and compared BIT FOR BIT with the same number of sweeps of the
    whole global grid run as ONE grid on rank 0's GPU -- the slabs' exchange,
    fused rounds and face signalling must not change a single bit (SURVEY
    8(e)).  Skipped when the global grid does not fit beside rank 0's slab."""
    import numpy as np
    import torch
    import torch.distributed as dist

    from stencil_amd.engine import JacobiEngine
    from stencil_amd.slab import partition

    gnx, gny, gnz = grid
    counts = [partition(gnz, world, r)[1] for r in range(world)]
    dev = torch.device("cuda", local) if on_gpu else torch.device("cpu")
    buf = torch.zeros(max(counts), dtype=torch.float64)
    buf[:counts[rank]] = torch.from_numpy(eng.plane_sums(slab.cur))
    buf = buf.to(dev)
    parts = [torch.zeros_like(buf) for _ in range(world)]
    dist.all_gather(parts, buf)
    result = None
    if rank == 0:
        try:
            got = np.concatenate([parts[r].cpu().numpy()[:counts[r]] for r in range(world)])
            need = 2.2 * gnx * gny * gnz * spec.elem_bytes  # two padded grids
            free = torch.cuda.mem_get_info(local)[0]
            if need > 0.9 * free:
                result = {"skipped": f"global grid needs {need / 1e9:.0f} GB, {free / 1e9:.0f} GB free"}
            else:
                ref = JacobiEngine(dataclasses.replace(spec, halo=0), gnx, gny, gnz, device=local)
                ref.reset("reference")
                fin, _ = ref.iterate(sweeps)
                want = ref.plane_sums(fin)
                bad = int(np.count_nonzero(want.view(np.uint64) != got.view(np.uint64)))
                result = {"planes": int(gnz), "sweeps": int(sweeps), "planes_differing": bad,
                          "bitwise_equal": bad == 0,
                          "reference": "the global grid as one grid on rank 0's GPU, same sweeps, per-plane sums"}
                del ref, fin
                torch.cuda.empty_cache()
        except Exception as exc:  # a check, never the measurement
            result = {"error": f"{type(exc).__name__}: {exc}"[:300]}
    dist.barrier()
    return result


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    from stencil_amd import _lib
    from stencil_amd.engine import JacobiEngine, StencilSpec, copy_bandwidth
    from stencil_amd.slab import (HostStagedExchanger, LoopbackExchanger, SelfP2PExchanger, SlabInfo, SlabJacobi,
                                  TorchDistExchanger, partition)

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return main_slab_job(args)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    if rank_job_wanted(args, world):
        return main_rank_job(args, world, rank, local)
    # 1 process, 1 GPU, the structure of an interior rank: halos = own
    # boundary planes (periodic), by device copies or by RCCL send/recv to self
    loop = args.exchange in ("loopback", "nccl-self")
    if loop and world != 1:
        raise SystemExit("--exchange loopback / nccl-self are single-process rehearsals")
    if args.share_device:
        if args.exchange != "host":
            raise SystemExit("--share-device needs --exchange host (RCCL refuses two ranks on one GPU)")
        local = 0
    torch.cuda.set_device(local)
    if world > 1:
        if args.exchange == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")
    elif args.exchange == "nccl-self":
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29561")
        dist.init_process_group("nccl", device_id=torch.device("cuda", local), rank=0, world_size=1)

    pre = PRESETS[args.config]
    if world < pre["min_gpus"]:
        raise SystemExit(f"--config {args.config} needs at least {pre['min_gpus']} GPUs (grid memory)")
    n = args.n
    if pre["grid"] is None:  # weak scaling: n^3 per rank
        gnx, gny, gnz = n, n, n * world
        first, count = rank * n, n
    else:                    # strong scaling: the global grid split in z-slabs
        gnx, gny, gnz = pre["grid"]
        first, count = partition(gnz, world, rank)
    # C3 / C4 on one GPU: two grids do not fit (C3 2 x 279 GB) or leave no room
    # (C4 2 x 138 GB); ONE resident grid plus a rolling margin of spare planes
    # (stencil_rolling_*, bitwise the two-grid job), the margin as deep as the
    # free HBM allows (at most 512 planes)
    rolling = args.config in ("C3", "C4") and world == 1 and not loop
    spec = StencilSpec(dims=3, dtype=pre["dtype"], shape=pre["shape"], radius=1, order="naive", kernel=args.kernel)
    multi = world > 1 or loop  # the slab round structure (exchange + two streams)
    extra = 0

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    if rolling:
        from stencil_amd.engine import RollingGrid
        free = torch.cuda.mem_get_info(local)[0]
        plane_b = RollingGrid.bytes_needed(spec, gnx, gny, 1, 64) - RollingGrid.bytes_needed(spec, gnx, gny, 1, 63)
        need = RollingGrid.bytes_needed(spec, gnx, gny, gnz, 8)
        shift = int(min(512, (free - need - (2 << 30)) // plane_b + 8))
        if shift < 16:
            raise SystemExit(f"--config {args.config} on one GPU needs {need / 2**30:.0f} GiB + a margin; "
                             f"{free / 2**30:.0f} GiB free")
        grid = RollingGrid(spec, gnx, gny, gnz, shift, device=local)
        grid.reset("reference")
        kname = "temporalk"
        sweeps_per_launch = grid.sweeps_per_pass
        grid.iterate(args.warmup)
        barrier()
        t0 = time.perf_counter()
        dev_ms, kernel_launches = grid.iterate(args.steps, stream=torch.cuda.current_stream(), timed=True)[1:]
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
        kernel_ms_total = dev_ms
        cells_per_launch = float(gnx) * gny * gnz  # charged per pass of K sweeps over the whole grid
        rolling_info = {"shift_planes": shift, "launch_planes": shift - sweeps_per_launch,
                        "launches": kernel_launches, "grid_bytes": grid.bytes}
    else:
        # Multi-GPU slabs keep K-deep z halos (K = sweeps one fused launch does:
        # 4 for the 7-point star, 3 or 4 for the box) so K sweeps fuse across the
        # exchange too (one K-plane exchange per K-sweep round).
        fuse = JacobiEngine(spec, gnx, gny, count, device=local, allocate=False).fuse_steps
        if world > 1 or loop:
            spec = dataclasses.replace(spec, halo=max(2, fuse))
        flags = (_lib.HALO_LO if rank > 0 or loop else 0) | (_lib.HALO_HI if rank < world - 1 or loop else 0)
        eng = JacobiEngine(spec, gnx, gny, count, device=local, flags=flags)
        if loop:
            exchanger = LoopbackExchanger() if args.exchange == "loopback" else SelfP2PExchanger(0, 1)
            info = SlabInfo(0, 3, first, count)  # drives the multi-rank round structure
        else:
            exchanger = (TorchDistExchanger if args.exchange == "nccl" else HostStagedExchanger)(rank, world)
            info = SlabInfo(rank, world, first, count)
        SlabJacobi.use_signal = not args.no_signal
        SlabJacobi.use_face_signal = args.face_signal
        slab = SlabJacobi(eng, info, exchanger, overlap=not args.no_overlap)
        slab.init("reference")
        kernel_id = eng.plan(12)[1]
        kname = {1: "direct", 2: "zmarch", 3: "temporal2", 4: "temporalk"}[kernel_id]
        if spec.shape == "box" and kname in ("temporal2", "temporalk"):
            kname = "boxk"  # the box's fused family (kernels_boxk.hip)
        sweeps_per_launch = eng.fuse_steps if not multi else slab.launches_per_round()

        # ---------------- warmup
        if not multi:
            # settle the one-time per-shape choice (packed vs equal z-chunks, timed
            # on the first launch of a shape) outside the timed region whatever W
            # is: one fused launch a -> b, grid a unchanged
            eng.prepare()
            eng.iterate(args.warmup)
        else:
            slab.run(args.warmup)
        barrier()

        # ---------------- timed region: exactly K sweeps
        stream = torch.cuda.current_stream()
        t0 = time.perf_counter()
        if not multi:
            _, dev_ms = eng.iterate(args.steps, stream=stream, timed=True)
            kernel_ms_total = dev_ms
            kernel_launches = eng.plan(args.steps)[0]
        else:
            slab.run(args.steps)
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([elapsed], dtype=torch.float64, device="cuda" if args.exchange == "nccl" else "cpu")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed = float(t.item())
            dist.barrier()
        if multi and slab.signal_timeouts():
            raise SystemExit("a face-counter wait timed out: the slab rounds did not complete")
        if multi:
            # Interior launch time for the roofline, from HIP events on the
            # interior stream over a few more rounds AFTER the timed region: the
            # events are extra queue packets (~5 us each per round on MI355X) that
            # the timed rounds do not carry.
            slab.start_kernel_timing()
            extra = max(4, min(args.steps, 8)) * slab.launches_per_round()
            slab.run(extra)
            kernel_ms_total, kernel_launches = slab.stop_kernel_timing()
            if world > 1:
                dist.barrier()
        check = None
        if world > 1 and not args.no_check:
            check = verify_slabs(eng, slab, spec, (gnx, gny, gnz), world, rank, args.warmup + args.steps + extra,
                                 args.exchange == "nccl", local)
        # the timed launch: the whole slab (single-GPU job, or face-signalled
        # slab rounds) or the interior between the two boundary launches
        cells_here = float(gnx) * gny * count
        edge = slab.depth if slab.fused else max(1, slab.depth)
        whole = not multi or slab.signalled
        cells_per_launch = cells_here if whole else cells_here * (count - 2 * edge) / count
        rolling_info = None

    if not multi:
        # device time per `sweeps_per_launch` sweeps, charged pro rata (with
        # K = 4 a 1000-step job is 250 fused launches; a K that does not divide
        # the step count adds a remainder pair / single sweep)
        launch_ms = kernel_ms_total * sweeps_per_launch / max(1, args.steps)
    else:
        launch_ms = kernel_ms_total / max(1, kernel_launches)
    if rolling:
        del grid
        torch.cuda.empty_cache()  # the copy-kernel calibration needs 2 GiB
    if rank == 0:
        if rolling:
            parallelism = ("1 GPU, ONE resident grid + a rolling margin of %d planes (stencil_rolling_iterate: "
                           "%d-plane launches, bitwise the two-grid job)" % (shift, shift - sweeps_per_launch))
        elif loop:
            parallelism = ("1 GPU rehearsing an interior rank (periodic halo, two streams, " +
                           ("device copies)" if args.exchange == "loopback" else "RCCL send/recv to self)"))
        elif world == 1:
            parallelism = "1 GPU, one process, the whole grid (no decomposition)"
        else:
            parallelism = f"z-slab x{world}, one process per GPU (torch.distributed.run)" + (
                ", RCCL halo P2P overlapped" if args.exchange == "nccl" else ", host-staged gloo halo (rehearsal)")
        report(args, pre, spec, kname, (gnx, gny, gnz), world, elapsed, launch_ms, cells_per_launch, sweeps_per_launch,
               kernel_launches, parallelism,
               rounds=(None if not multi else "one face-signalled launch per round" if slab.signalled else
                       "boundary + interior launches per round"),
               launch_timing=("hipEvents of stencil_rolling_iterate over the timed region" if rolling else
                              "hipEvents of stencil_iterate over the timed region" if not multi else
                              "events around the face-signalled whole-slab launches of extra rounds after the timed "
                              "region" if slab.signalled else
                              "events around the interior launches of extra rounds after the timed region"),
               workload_key=(f"3d7pt_fp64_{args.n}cube_per_gpu" + (f"_slab_x{world}" if multi else ""))
               if args.config == "C2" else
               ("C3_rolling_4096" if rolling and args.config == "C3" else f"{args.config}_rolling" if rolling else
                f"{args.config}_slab_{count}" + (f"_x{world}" if multi else "")),
               local=local, check=(check if world > 1 else None), cpu=(world == 1 and not loop),
               extra_config={"rolling": rolling_info} if rolling else None,
               kernels_per_launch=(kernel_launches / max(1.0, args.steps / sweeps_per_launch)) if rolling else 1.0)
    if world > 1 or args.exchange == "nccl-self":
        dist.destroy_process_group()


def rank_job_wanted(args, world: int) -> bool:
    """Under torch.distributed.run with N > 1: the C-ABI rank-mode job unless
    --driver python or a rehearsal transport asks for the Python slab driver."""
    if world <= 1 or args.driver == "python":
        return False
    if args.exchange != "nccl" or args.share_device or args.no_signal or args.face_signal or args.no_overlap:
        if args.driver == "cabi":
            raise SystemExit("--driver cabi: RCCL between distinct GPUs, default rounds (drop --exchange / "
                             "--share-device / --no-signal / --face-signal / --no-overlap, or use --driver python)")
        return False
    return True


def slab_job_plan(args, visible: int):
    """Devices and exchange of the single-process multi-GPU job (no GPU call:
    `visible` from torch.cuda.device_count()); SystemExit with the reason when
    it cannot run here."""
    n = args.gpus
    if args.exchange not in ("nccl", "copy"):
        raise SystemExit(f"--exchange {args.exchange} is a torch.distributed rehearsal: without a launcher use "
                         "nccl (RCCL) or copy (device copies)")
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


def global_grid_check(spec, grid, sweeps, got, device):
    """The multi-GPU job's per-plane sums `got` against the same sweeps of the
    global grid run as ONE grid on `device`, bit for bit (skipped when the
    global grid does not fit beside the job)."""
    import numpy as np
    import torch

    from stencil_amd.engine import JacobiEngine
    gnx, gny, gnz = grid
    try:
        need = 2.2 * gnx * gny * gnz * spec.elem_bytes
        free = torch.cuda.mem_get_info(device)[0]
        if need > 0.9 * free:
            return {"skipped": f"global grid needs {need / 1e9:.0f} GB, {free / 1e9:.0f} GB free on GPU {device}"}
        ref = JacobiEngine(spec, gnx, gny, gnz, device=device)
        ref.reset("reference")
        fin, _ = ref.iterate(sweeps)
        want = ref.plane_sums(fin)
        bad = int(np.count_nonzero(want.view(np.uint64) != got.view(np.uint64)))
        del ref, fin
        torch.cuda.empty_cache()
        return {"planes": int(gnz), "sweeps": int(sweeps), "planes_differing": bad, "bitwise_equal": bad == 0,
                "reference": f"the global grid as one grid on GPU {device}, same sweeps, per-plane sums"}
    except Exception as exc:  # a check, never the measurement
        return {"error": f"{type(exc).__name__}: {exc}"[:300]}


def main_rank_job(args, world, rank, local):
    """One process per GPU (torch.distributed.run) through the C-ABI rank-mode
    slab job (stencil_slab_unique_id / stencil_slab_create_rank, csrc/slab.hip):
    each rank builds and runs only its own z-slab, the halos over RCCL between
    the ranks' slabs, face-signalled rounds -- the shape of an MPI-per-rank
    launch.  torch.distributed (gloo, host side only) hands rank 0's RCCL id to
    the others and carries the barriers, the max-over-ranks time and the
    per-plane sums of the check; it moves no halo data."""
    import numpy as np
    import torch
    import torch.distributed as dist

    from stencil_amd.engine import SlabJob, StencilSpec

    pre = PRESETS[args.config]
    if world < pre["min_gpus"]:
        raise SystemExit(f"--config {args.config} needs at least {pre['min_gpus']} GPUs (grid memory)")
    dist.init_process_group("gloo")
    n = args.n
    gnx, gny, gnz = (n, n, n * world) if pre["grid"] is None else pre["grid"]
    spec = StencilSpec(dims=3, dtype=pre["dtype"], shape=pre["shape"], radius=1, order="naive", kernel=args.kernel)
    uid = [SlabJob.unique_id() if rank == 0 else None]
    dist.broadcast_object_list(uid, src=0)
    job = SlabJob(spec, gnx, gny, gnz, [local], rank=(world, rank, uid[0]))
    info = job.info(0)
    k = info["sweeps_per_round"]
    job.fill_initial("reference")
    sweeps = k + 1 + args.warmup
    job.run(k + 1)  # a full and a remainder round: both launch paths' one-time costs
    job.run(args.warmup)
    dist.barrier()
    elapsed = job.run(args.steps) * 1e-3  # this rank's rounds, its device synchronised at both ends
    t = torch.tensor([elapsed], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    sweeps += args.steps
    extra = k * max(4, min(args.steps // max(1, k), 8))
    job.kernel_timing(True)
    job.run(extra)
    kt = job.kernel_time()
    job.kernel_timing(False)
    sweeps += extra
    check = None
    if not args.no_check:
        sums = job.plane_sums()  # this rank's planes filled in, the rest zero
        mine = torch.from_numpy(sums[info["first"]:info["first"] + info["planes"]].copy())
        width = gnz // world + 1
        buf = torch.zeros(width, dtype=torch.float64)
        buf[:mine.numel()] = mine
        parts = [torch.zeros_like(buf) for _ in range(world)]
        dist.all_gather(parts, buf)
        counts = [None] * world
        dist.all_gather_object(counts, info["planes"])
        job.close()
        if rank == 0:
            got = np.concatenate([parts[r].numpy()[:counts[r]] for r in range(world)])
            check = global_grid_check(spec, (gnx, gny, gnz), sweeps, got, local)
        dist.barrier()
    else:
        job.close()
    if rank == 0:
        kname = "boxk" if spec.shape == "box" else "temporalk"
        parallelism = (f"z-slab x{world}, one process per GPU (torch.distributed.run) through the C-ABI rank-mode "
                       "slab job (stencil_slab_create_rank), RCCL send/recv between the ranks' slabs")
        report(args, pre, spec, kname, (gnx, gny, gnz), world, elapsed, kt["total_ms"] / max(1, kt["launches"]),
               float(kt["cells_per_launch"]), k, kt["launches"], parallelism,
               rounds="one face-signalled launch per round" if kt["signalled"] else
               "boundary + interior launches per round",
               launch_timing="hipEvents around rank 0's " + ("whole-slab face-signalled" if kt["signalled"] else
                                                             "interior") + " launches of extra rounds after the timed region",
               workload_key=f"3d7pt_fp64_{n}cube_per_gpu_slab_x{world}" if args.config == "C2" else
               f"{args.config}_slab_{info['planes']}_x{world}",
               local=local, check=check, cpu=False)
    dist.destroy_process_group()


def main_slab_job(args):
    """--gpus N without a launcher: ONE process drives N GPUs through the C-ABI
    slab job (stencil_slab_create/run/plane_sums, csrc/slab.hip): z-slabs, one
    per GPU, RCCL send/recv from one host thread, face-signalled rounds -- the
    shape of the reference's one spawn/join of its whole decomposed job
    (src/stencil/stencil.cpp:34-53).  Same JSON line as the per-process
    driver; the roofline from hipEvents on slab 0's compute stream over extra
    rounds after the timed region; multi_gpu_check against the global grid run
    as one grid on GPU 0."""
    import torch

    from stencil_amd.engine import SlabJob, StencilSpec

    devices, exchange = slab_job_plan(args, torch.cuda.device_count())
    n_gpus = args.gpus
    pre = PRESETS[args.config]
    n = args.n
    gnx, gny, gnz = (n, n, n * n_gpus) if pre["grid"] is None else pre["grid"]
    spec = StencilSpec(dims=3, dtype=pre["dtype"], shape=pre["shape"], radius=1, order="naive", kernel=args.kernel)
    job = SlabJob(spec, gnx, gny, gnz, devices, exchange=exchange)
    job.fill_initial("reference")
    k = job.info(0)["sweeps_per_round"]
    # one full round and one shorter remainder round before the timed region:
    # the one-time costs of both launch paths (schedule trials, first launches)
    sweeps = k + 1 + args.warmup
    job.run(k + 1)
    job.run(args.warmup)
    elapsed = job.run(args.steps) * 1e-3  # host wall time, every device synchronised at both ends
    sweeps += args.steps
    extra = k * max(4, min(args.steps // max(1, k), 8))
    job.kernel_timing(True)
    job.run(extra)
    kt = job.kernel_time()
    job.kernel_timing(False)
    sweeps += extra
    check = None
    if not args.no_check:
        check = global_grid_check(spec, (gnx, gny, gnz), sweeps, job.plane_sums(), 0)
    job.close()
    kname = "boxk" if spec.shape == "box" else "temporalk"
    where = "GPU 0 shared by every slab (rehearsal)" if args.share_device else f"{n_gpus} GPUs"
    parallelism = (f"z-slab x{n_gpus}, ONE process driving {where} through the C-ABI slab job (stencil_slab_*), " +
                   ("RCCL send/recv (ncclCommInitAll)" if exchange == "rccl" else "device-copy halos"))
    report(args, pre, spec, kname, (gnx, gny, gnz), n_gpus, elapsed, kt["total_ms"] / max(1, kt["launches"]),
           float(kt["cells_per_launch"]), k, kt["launches"], parallelism,
           rounds="one face-signalled launch per round" if kt["signalled"] else "boundary + interior launches per round",
           launch_timing="hipEvents around slab 0's " + ("whole-slab face-signalled" if kt["signalled"] else "interior")
                         + " launches of extra rounds after the timed region",
           workload_key=(f"3d7pt_fp64_{n}cube_per_gpu_slab_x{n_gpus}" if args.config == "C2" else
                         f"{args.config}_slab_{gnz // n_gpus}_x{n_gpus}"),
           local=0, check=check, cpu=False)


def report(args, pre, spec, kname, grid, n_gpus, elapsed, launch_ms, cells_per_launch, sweeps_per_launch,
           kernel_launches, parallelism, rounds, launch_timing, workload_key, local, check, cpu, extra_config=None,
           kernels_per_launch=1.0):
    """Print the one JSON line.  Roofline of the dominant kernel: one launch
    advances its cells by `sweeps_per_launch` fused sweeps; its compulsory HBM
    traffic is one read plus one write of those cells (2 * sizeof(T) per cell,
    whatever K is): `achieved` = compulsory bytes / mean launch time, a true
    fraction of the HBM peak.  The per-sweep algorithmic figure of SURVEY
    8(d) (2 * sizeof(T) per cell-UPDATE, K per cell per launch) is
    `effective_GBps`.  kernels_per_launch: kernel launches per charged
    "launch" (a rolling pass runs several z-range launches; the PMC table
    holds bytes per kernel launch)."""
    from stencil_amd.engine import copy_bandwidth
    gnx, gny, gnz = grid
    total_updates = float(gnx) * gny * gnz * args.steps
    gcell = total_updates / elapsed / 1e9
    bytes_per_update = 2 * spec.elem_bytes
    compulsory_bytes_launch = cells_per_launch * bytes_per_update
    alg_bytes_launch = compulsory_bytes_launch * sweeps_per_launch
    achieved = compulsory_bytes_launch / (launch_ms * 1e-3) / 1e9
    effective = alg_bytes_launch / (launch_ms * 1e-3) / 1e9
    traffic, traffic_entry = load_traffic(workload_key, kname)
    if traffic:
        traffic = traffic * kernels_per_launch
    desc = pre["desc"].format(n=args.n)
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
        "data": "synthetic: the reference initial condition (x-ghost faces 1, everything else 0)",
        "config": {
            "workload": f"{desc} (global {gnx}x{gny}x{gnz}), one step = one sweep",
            "grid": [gnx, gny, gnz],
            "kernel": kname,
            "parallelism": parallelism,
            "achieved_hbm_GBps_whole_job": round(gcell * bytes_per_update, 1),
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
                           "%d fused sweeps per launch" % (spec.elem_bytes, sweeps_per_launch),
            "compulsory_bytes_per_launch": compulsory_bytes_launch,
            "effective_GBps": round(effective, 1),
            "effective_basis": "SURVEY 8(d) algorithmic: 2 x %d B per cell-update x %d sweeps per launch"
                               % (spec.elem_bytes, sweeps_per_launch),
            "alg_bytes_per_launch": alg_bytes_launch,
            "mean_launch_ms": round(launch_ms, 5),
            "launches": kernel_launches,
            "launch_timing": launch_timing,
        },
    }
    if extra_config:
        out["config"].update(extra_config)
    if n_gpus > 1:
        out["multi_gpu_check"] = check if check is not None else {"skipped": "--no-check"}
    if traffic_entry is not None:
        out["roofline"]["traffic_source"] = {k: traffic_entry.get(k) for k in
                                             ("source", "kernel", "kernel_source_sha", "fresh")}
    if traffic and launch_ms > 0:
        # the PMC-measured bytes of one launch (L2->fabric: HBM plus
        # Infinity-Cache hits) over its live mean duration; traffic well
        # above the compulsory bytes = re-reads (tile rings, halos)
        out["roofline"]["traffic_GBps"] = round(traffic / (launch_ms * 1e-3) / 1e9, 1)
        out["roofline"]["traffic_frac"] = round(out["roofline"]["traffic_GBps"] / HBM_PEAK_GBPS, 4)
    try:
        out["roofline"]["copy_kernel_GBps"] = round(copy_bandwidth(1 << 30, reps=10, device=local), 1)
    except Exception as exc:  # calibration only
        out["roofline"]["copy_kernel_GBps"] = f"unavailable: {exc}"
    if cpu and not args.no_cpu_baseline:
        cb = dict(dtype=spec.dtype, shape=spec.shape)
        n = min(args.n, 512)
        out["cpu_baseline"] = cpu_baseline(n, args.cpu_seconds, **cb)
        # the same loop with OpenMP over the host's cores too
        out["cpu_baseline_all_cores"] = cpu_baseline(n, args.cpu_seconds / 2, threads=host_threads(), **cb)
    else:
        out["cpu_baseline"] = None
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
