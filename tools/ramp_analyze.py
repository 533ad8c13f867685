#!/usr/bin/env python3
"""Per-phase launch durations of tools/ramp_probe.py's kernel trace.

    tools/ramp_analyze.py gpurun_out/<tag>/ramp/run_kernel_trace.csv

Phases are split by the probe's 16-byte marker copies (copy_kernel with a
one-workgroup grid); prints each phase's K-step launch durations (us) in
order, with their mean over the first 10 and the rest."""
import csv
import sys


def main(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    phases, cur = [], []
    for r in rows:
        name, grid = r["Kernel_Name"], int(r.get("Grid_Size_X") or 0)
        dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        if "copy_kernel" in name and grid <= 256:
            phases.append(cur)
            cur = []
        elif "tkstrip" in name:
            cur.append(dur)
    phases.append(cur)
    labels = ["pre", "A start (prepare + 60 launches)", "B after 0.3 s idle", "C re-filled reference IC",
              "D random interior", "E after 60 ms of copies", "post"]
    for i, ph in enumerate(phases):
        if not ph:
            continue
        head, tail = ph[:10], ph[10:]
        lab = labels[i] if i < len(labels) else f"phase {i}"
        mh = sum(head) / len(head)
        mt = sum(tail) / len(tail) if tail else float("nan")
        print(f"{lab}: {len(ph)} launches, first 10 mean {mh:.1f} us, rest mean {mt:.1f} us")
        print("   " + " ".join(f"{d:.0f}" for d in ph))


if __name__ == "__main__":
    main(sys.argv[1])
