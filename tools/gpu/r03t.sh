#!/bin/bash
# round 3, call t: the pre-round-3 box order's fp32 probe shapes, SLP build at full -O3, with and without
# LLVM's GCN DPP Combine pass (-mllvm -amdgpu-dpp-combine=false); reference = the no-SLP build (96RRNN)
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/r03t_slp_dppcombine_old.txt
: > $O
for v in o999999 odppoff; do
  for k in 1 2 3; do
    timeout -k 10 120 python3 -u tools/slp_bisect.py build/slp_old/libdbg_$v.so $k --ref-cfg 960808 950808 >> $O 2>&1 || exit 1
  done
  for k in 3 4; do
    timeout -k 10 120 python3 -u tools/slp_bisect.py build/slp_old/libdbg_$v.so $k --ref-cfg 960408 950408 >> $O 2>&1 || exit 1
  done
done
