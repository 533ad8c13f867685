#!/usr/bin/env python3
"""Tabulate a tools/gpu/lease.sh pitchscan log: per plane width the best Gcell/s of the raw pitch
(STENCIL_ROW_RULE=0), +128 B, +2 KiB and the product's own padding (the row-pitch rule).
usage: python tools/pitch_table.py <pitchscan_<dtype>.txt> [...]"""
import collections
import re
import sys

PAT = re.compile(r"STENCIL_ROW_RULE=(\d) pad (\d+): \S+ star r1 naive (fp32|fp64) (\d+)x(\d+)x(\d+) \d+ sweeps: "
                 r"best [\d.]+ ms, ([\d.]+) Gcell/s")


def raw_pitch(nx, es):
    align = 128 // es
    return ((align + nx + 1 + align - 1) // align * align) * es  # origin_x = align for r = 1


def rule_pitch(p):
    return p + (128 if p < 65536 else 2048) if p >= 32768 and p % 32768 <= 256 else p


for path in sys.argv[1:]:
    res = collections.defaultdict(list)
    for line in open(path):
        m = PAT.match(line)
        if m:
            res[(m.group(3), int(m.group(4)), int(m.group(5)), m.group(1), int(m.group(2)))].append(float(m.group(7)))
    print(f"{path}\n{'dtype':5} {'plane':>12} {'raw pitch':>9} | {'raw':>6} {'+128B':>6} {'+2KiB':>6} | {'product':>7} pitch")
    for dt, nx, ny in sorted({k[:3] for k in res}):
        es = 8 if dt == "fp64" else 4
        g = lambda rule, pad: max(res.get((dt, nx, ny, rule, pad), [0.0]))
        p = raw_pitch(nx, es)
        print(f"{dt:5} {nx:>6}x{ny:<5} {p:9d} | {g('0', 0):6.0f} {g('0', 128 // es):6.0f} {g('0', 2048 // es):6.0f} | "
              f"{g('1', 0):7.0f} {rule_pitch(p)}")
