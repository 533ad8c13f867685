#!/bin/bash
# round 3, call an: kernels_tb2d.hip under gcn-max-ilp vs default on the other 2D shapes (radius 2 and 3, the DMA
# order, a one-workgroup grid), alternating, separate processes
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/r03an_tb2d_sched.txt
: > $O
for rep in 1 2; do
  for v in tbase tilp; do
    TL_RADIUS=2 timeout -k 10 120 python3 tools/time_lib.py build/variants/lib_$v.so star fp64 1024 1024 0 100 20 >> $O 2>/dev/null || exit 1
    TL_RADIUS=3 timeout -k 10 120 python3 tools/time_lib.py build/variants/lib_$v.so star fp64 1024 1024 0 100 20 >> $O 2>/dev/null || exit 1
    TL_ORDER=dma timeout -k 10 120 python3 tools/time_lib.py build/variants/lib_$v.so star fp32 1024 1024 0 100 20 >> $O 2>/dev/null || exit 1
    timeout -k 10 120 python3 tools/time_lib.py build/variants/lib_$v.so star fp64 64 64 0 1000 20 >> $O 2>/dev/null || exit 1
    timeout -k 10 120 python3 tools/time_lib.py build/variants/lib_$v.so star fp64 4096 4096 0 100 5 >> $O 2>/dev/null || exit 1
  done
done
