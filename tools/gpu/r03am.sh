#!/bin/bash
# round 3, call am: the 2D kernels' file (kernels_tb2d.hip: tb2ds, C1's kernel) under the machine schedulers,
# C1 = 1024^2 fp64 100 sweeps and fp32 (AUTO), alternating, separate processes
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/r03am_tb2d_sched.txt
: > $O
for rep in 1 2; do
  for v in tbase tilp tmc titer; do
    timeout -k 10 120 python3 tools/time_lib.py build/variants/lib_$v.so star fp64 1024 1024 0 100 20 >> $O 2>/dev/null || exit 1
    timeout -k 10 120 python3 tools/time_lib.py build/variants/lib_$v.so star fp32 1024 1024 0 100 20 >> $O 2>/dev/null || exit 1
  done
done
