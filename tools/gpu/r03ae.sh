#!/bin/bash
# round 3, call ae: the box file under gcn-max-memory-clause vs default on deep grids (time_lib: AUTO whole-job
# sweeps from the reference initial condition), alternating, separate processes
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/r03ae_box_mc.txt
: > $O
t() { timeout -k 10 300 python3 tools/time_lib.py build/variants/lib_$1.so "${@:2}" >> $O 2>/dev/null; }
for rep in 1 2; do
  for v in boxbase boxmc; do
    t $v box fp64 2048 2048 2048 8 2 || exit 1
    t $v box fp64 2048 2048 1024 16 2 || exit 1
    t $v box fp64 1024 1024 2048 32 2 || exit 1
    t $v box fp32 2048 2048 1024 16 2 || exit 1
  done
done
