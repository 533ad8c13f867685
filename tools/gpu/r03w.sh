#!/bin/bash
# round 3, call w: the 7-point strip kernel's interior fast path three ways -- a second copy of the step (default,
# FP = 1), none (710708), a wave-uniform branch around each select in one step body (730708) -- parity, then the
# bench's own workload (C2 1000 sweeps, NS 2048^3) alternating runs in separate processes
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "tkstrip_chunking and (730708 or 710708)" > gpurun_out/r03w_fp_parity.txt 2>&1 || exit 1
O=gpurun_out/r03w_fastpath_bench.txt
: > $O
for rep in 1 2; do
  for cfg in 1 710708 730708; do
    echo "STENCIL_TK_STRIP=$cfg C2" >> $O
    STENCIL_TK_STRIP=$cfg timeout -k 10 200 python3 bench.py --no-cpu-baseline >> $O 2>/dev/null || exit 1
  done
done
for cfg in 1 730708; do
  echo "STENCIL_TK_STRIP=$cfg NS" >> $O
  STENCIL_TK_STRIP=$cfg timeout -k 10 300 python3 bench.py --config NS --steps 40 --warmup 4 --no-cpu-baseline >> $O 2>/dev/null || exit 1
done
