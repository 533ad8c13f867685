"""Do the slab round's launches overlap?  Reads a rocprofv3 kernel trace
(run_kernel_trace.csv) and reports, per interior K-step launch, how much of
the boundary launches of the same round ran concurrently with it.
usage: python tools/overlap_check.py <trace.csv>"""
import csv
import sys


def main():
    rows = [r for r in csv.DictReader(open(sys.argv[1])) if "tkstrip" in r["Kernel_Name"] or "temporalk" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Grid_Size_X"]), r.get("Queue_Id", "?"),
           r.get("Stream_Id", "?")) for r in rows]
    big = max(e[2] for e in ev)
    for i, (s, e, g, q, st) in enumerate(ev[:40]):
        kind = "interior" if g == big else "boundary"
        print(f"{kind:8s} start {(s - ev[0][0]) / 1e3:10.1f} us  dur {(e - s) / 1e3:8.1f} us  grid {g:8d} queue {q} stream {st}")


if __name__ == "__main__":
    main()
