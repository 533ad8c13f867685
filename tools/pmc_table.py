"""Summarise tools/pmc_variants.sh output: per variant, the per-launch mean of
every counter for the kernels whose name matches a pattern, plus derived
figures (HBM bytes with the gfx950 FETCH_SIZE x2 correction of
MI355X_MICROARCH.md §HBM, wait / VALU / LDS fractions of wave cycles).
usage: python tools/pmc_table.py <tag> [kernel-substring ...]"""
import collections
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    tag = sys.argv[1]
    pats = sys.argv[2:] or ["temporalk_7pt", "tkstrip_7pt", "boxk_27pt", "box27", "zmarch7", "temporal2_7pt"]
    base = os.path.join(ROOT, "gpurun_out", f"pmc_{tag}")
    out = {}
    for vdir in sorted(glob.glob(os.path.join(base, "v*")), key=lambda p: int(os.path.basename(p)[1:].split(".")[0]) if os.path.isdir(p) else 0):
        if not os.path.isdir(vdir):
            continue
        env = open(vdir + ".env").read().strip() if os.path.exists(vdir + ".env") else ""
        vals = collections.defaultdict(lambda: collections.defaultdict(list))
        durs = collections.defaultdict(list)
        for f in glob.glob(os.path.join(vdir, "p*", "run_counter_collection.csv")):
            for r in csv.DictReader(open(f)):
                k = next((p for p in pats if p in r["Kernel_Name"]), None)
                if not k:
                    continue
                vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
                durs[k].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
        for k, cs in vals.items():
            m = {c: sum(v) / len(v) for c, v in cs.items()}
            d = {}
            if "FETCH_SIZE" in m:
                d["hbm_read_GB"] = 2 * m["FETCH_SIZE"] * 1024 / 1e9
            if "WRITE_SIZE" in m:
                d["hbm_write_GB"] = m["WRITE_SIZE"] * 1024 / 1e9
            wc = m.get("SQ_WAVE_CYCLES")
            if wc:
                for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                          "SQ_ACTIVE_INST_LDS"):
                    if c in m:
                        d[c.replace("SQ_", "").lower() + "_frac"] = round(m[c] / wc, 3)
            if "SQ_BUSY_CYCLES" in m and "GRBM_GUI_ACTIVE" in m:
                pass
            d["mean_dispatch_us(profiled)"] = round(sum(durs[k]) / len(durs[k]) / 1e3, 1)
            out.setdefault(env or os.path.basename(vdir), {})[k] = {"counters": m, "derived": d}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
