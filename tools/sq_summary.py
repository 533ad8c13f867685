"""Summarise a profiles/collect_sq.sh run (gpurun_out/sq_<tag>/p1..p3): per
kernel, the per-dispatch mean of every SQ / TCC / GRBM counter and the
decomposition of wave time (MI355X_MICROARCH.md §rocprofv3 PMC slots: the
SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* counters are quad-cycles, and
SQ_WAIT_ANY + SQ_WAIT_INST_ANY + SQ_ACTIVE_INST_ANY ~= SQ_WAVE_CYCLES):
  parked   SQ_WAIT_ANY / SQ_WAVE_CYCLES       (s_waitcnt and barrier waits)
  stalled  SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES  (issue stalls: dependencies, pipes)
  issuing  SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES
  VALU / LDS issue shares, LDS bank-conflict cycles per LDS-array cycle,
  effective clock = GRBM_GUI_ACTIVE / 8 XCDs / kernel time.
usage: python tools/sq_summary.py <gpurun_out/sq_tag dir> [kernel-substring] [--json out.json]
"""
import collections
import csv
import glob
import json
import os
import sys


def main():
    d = sys.argv[1]
    pat = sys.argv[2] if len(sys.argv) > 2 and not sys.argv[2].startswith("--") else "tkstrip"
    out_json = sys.argv[sys.argv.index("--json") + 1] if "--json" in sys.argv else None
    vals = collections.defaultdict(list)
    durs = []
    for p in sorted(glob.glob(os.path.join(d, "p*"))):
        per = collections.defaultdict(dict)
        for f in glob.glob(os.path.join(p, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                if pat not in r["Kernel_Name"]:
                    continue
                key = r["Dispatch_Id"]
                per[key][r["Counter_Name"]] = per[key].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        for f in glob.glob(os.path.join(p, "**", "*kernel_trace.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                if pat in r["Kernel_Name"]:
                    durs.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
        for disp, cs in per.items():
            for k, v in cs.items():
                vals[k].append(v)
    mean = {k: sum(v) / len(v) for k, v in vals.items()}
    n = {k: len(v) for k, v in vals.items()}
    wc = mean.get("SQ_WAVE_CYCLES")
    derived = {}
    if wc:
        for k, name in (("SQ_WAIT_ANY", "parked"), ("SQ_WAIT_INST_ANY", "issue_stalled"),
                        ("SQ_ACTIVE_INST_ANY", "issuing"), ("SQ_ACTIVE_INST_VALU", "valu_active"),
                        ("SQ_ACTIVE_INST_LDS", "lds_active"), ("SQ_WAIT_INST_LDS", "lds_issue_stalled")):
            if k in mean:
                derived[name + "_frac_of_wave_cycles"] = round(mean[k] / wc, 4)
    if "SQ_LDS_BANK_CONFLICT" in mean and mean.get("SQ_LDS_IDX_ACTIVE"):
        derived["lds_bank_conflict_frac"] = round(mean["SQ_LDS_BANK_CONFLICT"] / mean["SQ_LDS_IDX_ACTIVE"], 4)
    if "SQ_BUSY_CYCLES" in mean and "GRBM_GUI_ACTIVE" in mean:
        derived["sq_busy_frac_of_gui_active"] = round(mean["SQ_BUSY_CYCLES"] / mean["GRBM_GUI_ACTIVE"], 4)
    if durs and "GRBM_GUI_ACTIVE" in mean:
        t = sum(durs) / len(durs)
        derived["mean_dispatch_ms_profiled"] = round(t * 1e3, 4)
        derived["effective_clock_MHz"] = round(mean["GRBM_GUI_ACTIVE"] / 8 / t / 1e6, 1)
    if "TCC_HIT_sum" in mean and "TCC_MISS_sum" in mean:
        derived["l2_hit_frac"] = round(mean["TCC_HIT_sum"] / (mean["TCC_HIT_sum"] + mean["TCC_MISS_sum"]), 4)
    if "SQ_WAVES" in mean and wc:
        derived["wave_cycles_per_wave"] = round(wc / mean["SQ_WAVES"], 1)
    res = {"dir": d, "kernel": pat, "dispatches_per_counter": n, "mean": {k: round(v, 1) for k, v in mean.items()},
           "derived": derived}
    print(json.dumps(res, indent=1))
    if out_json:
        json.dump(res, open(out_json, "w"), indent=1)


if __name__ == "__main__":
    main()
