#!/bin/bash
# round 3, call ap: the box file under other scheduler options at C5 (2048^3 fp64, time_lib: AUTO whole-job
# sweeps), alternating, separate processes
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/r03ap_box_sched.txt
: > $O
for rep in 1 2; do
  for v in bxbase bxnounc bxaa bxnocl; do
    timeout -k 10 300 python3 tools/time_lib.py build/variants/lib_$v.so box fp64 2048 2048 2048 8 2 >> $O 2>/dev/null || exit 1
  done
done
