#!/bin/bash
# round 3, call aq: the box file without the unclustered high-RP reschedule stage vs default on other box shapes
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/r03aq_box_nounc.txt
: > $O
for rep in 1 2; do
  for v in bxbase bxnounc; do
    timeout -k 10 200 python3 tools/time_lib.py build/variants/lib_$v.so box fp64 512 512 512 96 3 >> $O 2>/dev/null || exit 1
    timeout -k 10 200 python3 tools/time_lib.py build/variants/lib_$v.so box fp64 1024 1024 1024 24 3 >> $O 2>/dev/null || exit 1
    timeout -k 10 200 python3 tools/time_lib.py build/variants/lib_$v.so box fp32 2048 2048 256 24 3 >> $O 2>/dev/null || exit 1
    timeout -k 10 200 python3 tools/time_lib.py build/variants/lib_$v.so box fp32 512 512 512 96 3 >> $O 2>/dev/null || exit 1
  done
done
