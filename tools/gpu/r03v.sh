#!/bin/bash
# round 3, call v: the 7-point strip kernel's interior fast path (default) against the same shape without it
# (debug cfg 710708), on the bench's own workload (evolving field, stencil_iterate, 1000 sweeps), alternating
# runs in separate processes; NS (2048^3) likewise
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/r03v_fastpath_bench.txt
: > $O
for rep in 1 2; do
  for cfg in 1 710708; do
    echo "STENCIL_TK_STRIP=$cfg C2" >> $O
    STENCIL_TK_STRIP=$cfg timeout -k 10 200 python3 bench.py --no-cpu-baseline >> $O 2>/dev/null || exit 1
  done
done
for cfg in 1 710708; do
  echo "STENCIL_TK_STRIP=$cfg NS" >> $O
  STENCIL_TK_STRIP=$cfg timeout -k 10 300 python3 bench.py --config NS --steps 40 --warmup 4 --no-cpu-baseline >> $O 2>/dev/null || exit 1
done
