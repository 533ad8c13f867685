"""The sustained-load slowdown of C2: BASELINE's 1000-sweep
512^3 fp64 job runs its launches ~9 % slower than the same launches in the
placement search.  This runs bench.py's single-GPU path (placement search,
prepare, warm-up) and then the timed jobs, while a thread samples the GPU's
own telemetry through amdsmi (in-process: no wrapper, no re-exec) -- socket
power, gfx / memory clocks, temperatures and the throttle flags -- every
~1 ms, on the host's monotonic clock.  Run it under a rocprofv3 kernel trace
(per-launch durations) and, in a separate run, with --pmc GRBM_GUI_ACTIVE
(cycles per launch -> effective clock); tools/sustained_analyze.py joins them
by launch index and by time.

usage: python tools/sustained_probe.py --out gpurun_out/x/sustained.json [--steps 1000] [--jobs 3] [--gap-ms 300]
"""
import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


class Telemetry(threading.Thread):
    """amdsmi gpu-metrics samples of GPU 0 every `period` seconds."""

    KEYS = ("power", "clk", "temp", "throttle", "activity", "energy", "voltage", "residency", "timestamp",
            "accumulation", "lock")

    def __init__(self, period=0.001):
        super().__init__(daemon=True)
        self.period = period
        self.samples = []
        self.error = None
        self.stop_ev = threading.Event()
        try:
            import amdsmi
            amdsmi.amdsmi_init()
            self.smi = amdsmi
            self.handle = amdsmi.amdsmi_get_processor_handles()[0]
            self.smi.amdsmi_get_gpu_metrics_info(self.handle)  # fails here if unreadable
        except Exception as e:  # noqa: BLE001 -- telemetry is optional, the trace is not
            self.smi = None
            self.error = f"{type(e).__name__}: {e}"

    @staticmethod
    def _scalar(v):
        if isinstance(v, (int, float)):
            return v
        if isinstance(v, (list, tuple)):
            vals = [x for x in v if isinstance(x, (int, float)) and x not in (0xFFFF, 0xFFFFFFFF, 0xFFFFFFFFFFFFFFFF)]
            return vals or None
        return None

    def run(self):
        if self.smi is None:
            return
        while not self.stop_ev.is_set():
            t = time.monotonic_ns()
            try:
                m = self.smi.amdsmi_get_gpu_metrics_info(self.handle)
            except Exception as e:  # noqa: BLE001
                self.error = f"{type(e).__name__}: {e}"
                return
            rec = {"t_ns": t}
            # the data-fabric and memory clocks (not in gpu_metrics): the
            # memory-bound kernel's time tracks the memory side, not gfxclk
            for name in ("DF", "MEM", "SOC"):
                try:
                    ci = self.smi.amdsmi_get_clock_info(self.handle, getattr(self.smi.AmdSmiClkType, name))
                    if isinstance(ci.get("clk"), (int, float)):
                        rec[f"clk_{name.lower()}"] = ci["clk"]
                except Exception:  # noqa: BLE001 -- not every clock is readable everywhere
                    pass
            for k, v in m.items():
                if any(s in k for s in self.KEYS):
                    sv = self._scalar(v)
                    if sv is not None:
                        rec[k] = sv
            self.samples.append(rec)
            time.sleep(self.period)

    def stop(self):
        self.stop_ev.set()
        if self.is_alive():
            self.join(2.0)
        if self.smi is not None:
            try:
                self.smi.amdsmi_shut_down()
            except Exception:  # noqa: BLE001
                pass


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--jobs", type=int, default=3, help="timed jobs, back to back after the first")
    ap.add_argument("--gap-ms", type=float, default=300.0, help="idle time before each later job")
    ap.add_argument("--long", type=int, default=4000, help="one more job of this many sweeps at the end (0: none)")
    ap.add_argument("--placements", type=int, default=16)
    args = ap.parse_args()

    import torch

    from stencil_amd.engine import JacobiEngine, StencilSpec

    tel = Telemetry()
    tel.start()
    marks = []

    def mark(name):
        torch.cuda.synchronize()
        marks.append({"name": name, "t_ns": time.monotonic_ns(),
                      "boottime_ns": time.clock_gettime_ns(time.CLOCK_BOOTTIME)})

    torch.cuda.set_device(0)
    eng = JacobiEngine(StencilSpec(dims=3, dtype="fp64", shape="star"), 512, 512, 512, device=0)
    mark("placement_begin")
    placement = eng.place(trials=args.placements) if args.placements > 1 else None
    mark("placement_end")
    eng.reset("reference", 0)
    settle = eng.prepare()
    eng.iterate(20)
    mark("warm")
    jobs = []
    sizes = [args.steps] * args.jobs + ([args.long] if args.long > 0 else [])
    for i, steps in enumerate(sizes):
        if i > 0 and args.gap_ms > 0:
            time.sleep(args.gap_ms / 1e3)
        mark(f"job{i}_begin")
        t0 = time.perf_counter()
        _, dev_ms = eng.iterate(steps, stream=torch.cuda.current_stream(), timed=True)
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        mark(f"job{i}_end")
        launches = eng.plan(steps)[0]
        jobs.append({"steps": steps, "launches": launches, "wall_ms": wall * 1e3, "device_ms": dev_ms,
                     "ms_per_launch": dev_ms / launches,
                     "gcells": 512 ** 3 * steps / wall / 1e9})
    time.sleep(0.05)
    tel.stop()
    out = {"placement": placement, "settle": settle, "jobs": jobs, "marks": marks,
           "telemetry_error": tel.error, "telemetry": tel.samples}
    os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
    with open(args.out, "w") as f:
        json.dump(out, f)
    for j in jobs:
        print(json.dumps(j))
    print(f"telemetry: {len(tel.samples)} samples, error {tel.error}")


if __name__ == "__main__":
    main()
