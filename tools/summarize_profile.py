"""Summarise a profiles/collect.sh run (gpurun_out/prof_<tag>) into
profiles/<tag>_kernel_stats.csv, profiles/<tag>_summary.json and the
bench's traffic table profiles/traffic.json.

HBM traffic per launch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 bytes: rocprofv3
reports both in KiB, and on gfx950 FETCH_SIZE counts exactly half the bytes of
wide coalesced streaming reads (MI355X_MICROARCH.md §HBM: FETCH_SIZE = RDREQ x 64 B
while the requests are 128 B) -- the strip kernels' reads are all 128-B requests
(RDREQ_128B = RDREQ), whatever their lane width (8 B fp64 V = 1,
16 B otherwise), so the factor 2 applies; calibrated in the same run by the copy
kernel (1 GiB read, FETCH_SIZE = 512 MiB), and without it the fp64 strip kernel's
reads would fall below the compulsory 1.07 GB per 512^3 launch.
usage: python tools/summarize_profile.py <tag> [workload-key]"""
import collections
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name):
    """Kernel family name as bench.py reports it."""
    table = (("tkstrip_7pt", "temporalk"), ("temporalk_7pt", "temporalk"), ("temporal2_7pt", "temporal2"),
             ("zmarch7", "zmarch"), ("sweep_direct", "direct"), ("box27_sep", "boxk"), ("box27_strip", "boxk"), ("boxk_27pt", "boxk"),
             ("copy_kernel", "copy_kernel"), ("fill_initial_kernel", "fill_initial_kernel"),
             ("plane_sums", "plane_sums"), ("tb2ds", "tb2ds"))
    for k, v in table:
        if k in name:
            return v
    return name[:40]


def main():
    tag = sys.argv[1]
    workload = sys.argv[2] if len(sys.argv) > 2 else "3d7pt_fp64_512cube_per_gpu"
    src = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    stats = {}
    for r in csv.DictReader(open(os.path.join(src, "trace", "run_kernel_stats.csv"))):
        stats[short(r["Name"])] = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]),
                                   "min_ns": float(r["MinNs"]), "max_ns": float(r["MaxNs"]), "name": r["Name"]}
    pmc = collections.defaultdict(dict)
    for counter in ("fetch", "write"):
        vals = collections.defaultdict(list)
        for r in csv.DictReader(open(os.path.join(src, counter, "run_counter_collection.csv"))):
            vals[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
        for k, v in vals.items():
            pmc[k][counter.upper() + "_SIZE_KiB"] = sum(v) / len(v)
    summary = {"tag": tag, "kernels": {}}
    for k, st in stats.items():
        ent = dict(st)
        if k in pmc and "FETCH_SIZE_KiB" in pmc[k] and "WRITE_SIZE_KiB" in pmc[k]:
            f, w = pmc[k]["FETCH_SIZE_KiB"], pmc[k]["WRITE_SIZE_KiB"]
            ent.update(FETCH_SIZE_KiB=f, WRITE_SIZE_KiB=w,
                       hbm_read_bytes=2 * f * 1024, hbm_write_bytes=w * 1024,
                       hbm_bytes_per_launch=(2 * f + w) * 1024,
                       actual_GBps=(2 * f + w) * 1024 / (st["avg_ns"] * 1e-9) / 1e9)
        summary["kernels"][k] = ent
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"),
                os.path.join(ROOT, "profiles", f"{tag}_kernel_stats.csv"))
    json.dump(summary, open(os.path.join(ROOT, "profiles", f"{tag}_summary.json"), "w"), indent=1)
    tpath = os.path.join(ROOT, "profiles", "traffic.json")
    table = json.load(open(tpath)) if os.path.exists(tpath) else {}
    sys.path.insert(0, ROOT)
    from bench import kernel_source_sha  # the sources the profiled library was built from
    for k, ent in summary["kernels"].items():
        if "hbm_bytes_per_launch" in ent and k in ("temporalk", "temporal2", "zmarch", "direct", "boxk", "tb2ds"):
            table.setdefault(workload, {})[k] = {"hbm_bytes_per_launch": round(ent["hbm_bytes_per_launch"]),
                                                 "source": f"profiles/{tag}_summary.json",
                                                 "kernel": ent["name"],
                                                 "kernel_source_sha": kernel_source_sha(k)}
    json.dump(table, open(tpath, "w"), indent=1)
    for k, ent in summary["kernels"].items():
        print(k, {x: round(y, 1) if isinstance(y, float) else y for x, y in ent.items() if x != "name"})


if __name__ == "__main__":
    main()
