#!/bin/bash
# round 3, call aa: scheduler variants across shapes (tools/time_lib.py: AUTO's whole-job sweeps from the
# reference initial condition, device time), alternating libraries in separate processes
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/r03aa_sched_shapes.txt
: > $O
t() { timeout -k 10 200 python3 tools/time_lib.py build/variants/lib_$1.so "${@:2}" >> $O 2>/dev/null; }
for rep in 1 2; do
  for v in base maxilp; do
    t $v star fp64 512 512 512 200 || exit 1
    t $v star fp64 1024 1024 1024 40 || exit 1
    t $v star fp64 2048 2048 512 40 || exit 1
    t $v star fp32 512 512 512 200 || exit 1
    t $v star fp32 2048 2048 512 50 || exit 1
  done
  for v in boxbase boxmemclause; do
    t $v box fp64 512 512 512 96 || exit 1
    t $v box fp64 1024 1024 1024 24 || exit 1
    t $v box fp64 2048 2048 256 24 || exit 1
    t $v box fp32 2048 2048 256 24 || exit 1
  done
done
