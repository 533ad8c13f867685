#!/usr/bin/env python3
"""Per-round timeline of a slab job from a rocprofv3 kernel trace.

    python tools/slab_timeline.py <run_kernel_trace.csv> [--last 12]

Prints the last kernels of the run (the strip / box launches, RCCL's kernels,
face waits and copies longer than a few microseconds) with start / end /
duration relative to the first of them and the queue, then per exchange
kernel (RCCL's, or the copies of a copy exchange) how much of its time ran
beside a stencil launch -- the overlap the round form is meant to give -- and
the stencil launches' durations with and without an exchange beside them."""
import argparse
import csv


def load(path):
    rows = list(csv.DictReader(open(path)))
    out = []
    for r in rows:
        name = r["Kernel_Name"]
        kind = ("stencil" if ("tkstrip" in name or "box27" in name or "zmarch" in name or "temporal" in name)
                else "rccl" if "rccl" in name.lower() or "nccl" in name.lower()
                else "wait" if "wait_counters" in name
                else "copy" if "copyBuffer" in name
                else None)
        if kind is None:
            continue
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        out.append(dict(kind=kind, name=name, s=s, e=e, q=r["Queue_Id"], grid=int(r["Grid_Size_X"])))
    out.sort(key=lambda k: k["s"])
    return out


def overlap(a, b):
    return max(0, min(a["e"], b["e"]) - max(a["s"], b["s"]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--last", type=int, default=14)
    ap.add_argument("--window", type=float, default=0.0, help="only kernels in the last W ms of the run (0: all)")
    args = ap.parse_args()
    ks = load(args.trace)
    if args.window > 0:
        # the job's last rounds: the window ends with the last exchange kernel
        # (a check grid may run after the job)
        exk = [k for k in ks if k["kind"] in ("rccl", "wait")] or ks
        end = max(k["e"] for k in exk) + 2e6
        ks = [k for k in ks if end - args.window * 1e6 <= k["s"] <= end]
    # drop tiny copies (the fill's and the plane copies' housekeeping)
    ks = [k for k in ks if not (k["kind"] == "copy" and k["e"] - k["s"] < 5000)]
    t0 = ks[-args.last]["s"] if len(ks) >= args.last else ks[0]["s"]
    print(f"{'start ms':>10} {'end ms':>10} {'dur ms':>8}  queue  kernel")
    for k in ks[-args.last:]:
        print(f"{(k['s'] - t0) / 1e6:10.3f} {(k['e'] - t0) / 1e6:10.3f} {(k['e'] - k['s']) / 1e6:8.3f}  q{k['q']:<4}  "
              f"{k['kind']:7s} {k['name'][:48]} grid={k['grid']}")
    st = [k for k in ks if k["kind"] == "stencil"]
    ex = [k for k in ks if k["kind"] in ("rccl", "copy")]
    if ex:
        tot = sum(k["e"] - k["s"] for k in ex)
        beside = sum(min(k["e"] - k["s"], sum(overlap(k, s) for s in st)) for k in ex)
        print(f"exchange kernels: {len(ex)}, {tot / 1e6:.3f} ms in all, {100.0 * beside / max(1, tot):.1f} % of it beside a "
              "stencil launch")
    big = [s for s in st if s["e"] - s["s"] > 1e6]  # launches over 1 ms (the interior / pass launches)
    if big:
        with_ex = [s for s in big if any(overlap(s, k) > 0 for k in ex)]
        without = [s for s in big if s not in with_ex]
        avg = lambda v: sum(k["e"] - k["s"] for k in v) / max(1, len(v)) / 1e6
        print(f"stencil launches > 1 ms: {len(big)}; with an exchange beside: {len(with_ex)} avg {avg(with_ex):.3f} ms; "
              f"without: {len(without)} avg {avg(without):.3f} ms")


if __name__ == "__main__":
    main()
