"""Join tools/sustained_probe.py's telemetry with the kernel trace of the same
run (and the GRBM_GUI_ACTIVE pass of a second run): per timed job, the K-step
launches in bins of `--bin` launches -- mean duration, and the GPU's own
gfx clock / socket power / temperature / throttle and power-limit residency
sampled during the bin -- plus, from the counter pass, cycles per launch and
the effective clock (GRBM_GUI_ACTIVE / XCDs / duration).

usage: python tools/sustained_analyze.py <dir with sustained_trace.json, sust_trace/> [--bin 25] [--pmc-dir sust_pmc]
"""
import argparse
import csv
import glob
import json
import os
import statistics


def kernel_rows(d):
    paths = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    rows = []
    for p in paths:
        rows += list(csv.DictReader(open(p)))
    return [r for r in rows if "tkstrip" in r["Kernel_Name"]]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--bin", type=int, default=25)
    ap.add_argument("--probe", default="sustained_trace.json")
    ap.add_argument("--trace-dir", default="sust_trace")
    ap.add_argument("--pmc-dir", default="sust_pmc")
    ap.add_argument("--pmc-probe", default="sustained_pmc.json")
    args = ap.parse_args()
    probe = json.load(open(os.path.join(args.dir, args.probe)))
    tel = probe["telemetry"]
    marks = {m["name"]: m for m in probe["marks"]}
    ks = kernel_rows(os.path.join(args.dir, args.trace_dir))
    ks.sort(key=lambda r: int(r["Start_Timestamp"]))
    # which host clock the trace's timestamps are on: the one that puts the
    # most launches inside the jobs' [begin, end] marks
    best = None
    for clk in ("t_ns", "boottime_ns"):
        inside = 0
        for i in range(len(probe["jobs"])):
            b, e = marks[f"job{i}_begin"][clk], marks[f"job{i}_end"][clk]
            inside += sum(1 for r in ks if b <= int(r["Start_Timestamp"]) <= e)
        if best is None or inside > best[1]:
            best = (clk, inside)
    clk = best[0]
    # telemetry samples are on monotonic time; map the trace clock onto it
    off = 0 if clk == "t_ns" else marks["job0_begin"]["t_ns"] - marks["job0_begin"]["boottime_ns"]

    def tel_mean(t0, t1, key):
        v = []
        for s in tel:
            if t0 <= s["t_ns"] <= t1 and key in s:
                x = s[key]
                v.append(statistics.mean(x) if isinstance(x, list) else x)
        return statistics.mean(v) if v else None

    out = {"clock": clk, "launches_in_jobs": best[1], "jobs": []}
    for i, job in enumerate(probe["jobs"]):
        b, e = marks[f"job{i}_begin"][clk], marks[f"job{i}_end"][clk]
        jl = [r for r in ks if b <= int(r["Start_Timestamp"]) <= e]
        bins = []
        for j in range(0, len(jl), args.bin):
            chunk = jl[j:j + args.bin]
            t0 = int(chunk[0]["Start_Timestamp"]) + off
            t1 = int(chunk[-1]["End_Timestamp"]) + off
            dur = statistics.mean((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in chunk)
            row = {"launches": f"{j}-{j + len(chunk) - 1}", "mean_us": round(dur, 1)}
            for key in ("current_gfxclk", "current_gfxclks", "average_gfxclk_frequency", "current_socket_power",
                        "average_socket_power", "temperature_hotspot", "temperature_mem", "current_uclk", "clk_df",
                        "clk_mem", "clk_soc", "current_socclk"):
                v = tel_mean(t0 - 2_000_000, t1 + 2_000_000, key)
                if v is not None:
                    row[key] = round(v, 1)
            # power from the energy accumulator (15.259 uJ units on MI300-class parts) over the bin
            ev = [(s["t_ns"], s["energy_accumulator"]) for s in tel
                  if t0 - 2_000_000 <= s["t_ns"] <= t1 + 2_000_000 and "energy_accumulator" in s]
            if len(ev) >= 2 and ev[-1][0] > ev[0][0]:
                row["power_W_from_energy"] = round((ev[-1][1] - ev[0][1]) * 15.259e-6 / ((ev[-1][0] - ev[0][0]) * 1e-9), 1)
            # residency counters: the increase over the bin (accumulators)
            for key in ("ppt_residency_acc", "socket_thm_residency_acc", "prochot_residency_acc", "throttle_status",
                        "indep_throttle_status", "accumulation_counter"):
                vs = [s[key] for s in tel if t0 - 2_000_000 <= s["t_ns"] <= t1 + 2_000_000 and key in s]
                if vs and all(isinstance(x, (int, float)) for x in vs):
                    row[key] = vs[-1] - vs[0] if key.endswith("_acc") else max(vs)
            bins.append(row)
        out["jobs"].append({"steps": job["steps"], "ms_per_launch_events": round(job["ms_per_launch"], 4),
                            "gcells_wall": round(job["gcells"], 1), "bins": bins})
    pmc = glob.glob(os.path.join(args.dir, args.pmc_dir, "**", "*counter_collection.csv"), recursive=True)
    if pmc:
        cyc = {}
        for p in pmc:
            for r in csv.DictReader(open(p)):
                if "tkstrip" in r["Kernel_Name"] and r["Counter_Name"] == "GRBM_GUI_ACTIVE":
                    cyc[r["Dispatch_Id"]] = cyc.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
        kp = kernel_rows(os.path.join(args.dir, args.pmc_dir))
        kp.sort(key=lambda r: int(r["Start_Timestamp"]))
        series = []
        for r in kp:
            if r["Dispatch_Id"] in cyc:
                dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
                series.append((dur, cyc[r["Dispatch_Id"]]))
        rows = []
        for j in range(0, len(series), args.bin):
            ch = series[j:j + args.bin]
            d = statistics.mean(x[0] for x in ch)
            c = statistics.mean(x[1] for x in ch)
            rows.append({"dispatches": f"{j}-{j + len(ch) - 1}", "mean_us": round(d * 1e6, 1), "grbm_cycles": round(c),
                         "clock_MHz_if_8_xcds": round(c / 8 / d / 1e6, 1)})
        out["pmc"] = rows
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
