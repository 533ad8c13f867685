#!/usr/bin/env python3
"""Counterpart of the reference's experiment sweep (run_expr.py:6-43).

Same sweep (block sizes x iteration counts, n = 8 * block size), same stdout
regex, same CSV columns ("Block Size", "Iteration", one column per method, ms
with 3 decimals).  Differences, on purpose: no bsub (the binary runs on the
local GPU), the current CLI flags (-s for the size; the reference passes the
stale "-m <size> ... -w 1"), and the methods are named
explicitly (the reference relied on a removed default).

usage: python run_expr.py [--methods M ...] [--iterations I ...] [--block-sizes B ...] [--out output.csv]
"""
import argparse
import csv
import os
import re
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
PATTERN = r'The average time taken by (.*) method is (.*)ms for \d+ iterations\.'  # run_expr.py:9

BLOCK_SIZES = [8, 16, 32, 48, 50, 64, 72, 88, 100, 120]                  # run_expr.py:6
ITERATIONS = [1, 10, 100, 1000, 5000, 10000, 50000, 100000]              # run_expr.py:7


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--methods", nargs="+", default=["DMA", "DMAStaticUnroll", "DMASlavePack", "RMA", "HIP", "CPU"])
    ap.add_argument("--cpu-max-iterations", type=int, default=1000,
                    help="run the CPU method (the reference's naive loop on the host, single-threaded) only up to "
                         "this many iterations: at 100000 iterations of a 960^2 grid it alone takes minutes")
    ap.add_argument("--block-sizes", nargs="+", type=int, default=BLOCK_SIZES)
    ap.add_argument("--iterations", nargs="+", type=int, default=ITERATIONS)
    ap.add_argument("--repeat", type=int, default=1)
    ap.add_argument("--binary", default=os.path.join(HERE, "build", "bin", "stencil_main"))
    ap.add_argument("--out", default="output.csv")
    args = ap.parse_args()

    outputs = []
    for block_size in args.block_sizes:
        for iteration in args.iterations:
            matrix_size = block_size * 8
            methods = [m for m in args.methods if m != "CPU" or iteration <= args.cpu_max_iterations]
            command = [args.binary, "-s", str(matrix_size), "-b", str(block_size), "-i", str(iteration),
                       "-R", str(args.repeat), "-m", *methods]
            print(f'----------- block size: {block_size}, iteration: {iteration} -----------')
            result = subprocess.run(command, capture_output=True, text=True)
            output = result.stdout.strip()
            print(output)
            if result.returncode != 0:
                print(result.stderr.strip())
            row = {'Block Size': block_size, 'Iteration': iteration}
            for match in re.finditer(PATTERN, output):
                method, time = match.groups()
                row[method] = f"{float(time):.3f}"
            outputs.append(row)

    with open(args.out, 'w', newline='') as f:
        # columns of every row, first-seen order (a method dropped from some
        # rows -- CPU past --cpu-max-iterations -- leaves those cells empty)
        fields = list(dict.fromkeys(k for row in outputs for k in row))
        writer = csv.DictWriter(f, fieldnames=fields)
        writer.writeheader()
        writer.writerows(outputs)


if __name__ == "__main__":
    main()
