#!/bin/bash
# round 3, call ah: packed schedules for face-signalled slab launches -- the signal / slab tests, then the
# interior-rank rehearsal (loopback) and the single-process slab job rehearsal, packed vs equal chunks
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_slab.py \
  tests/test_gpu_slab_job.py > gpurun_out/r03ah_slab_tests.txt 2>&1 || exit 1
O=gpurun_out/r03ah_loopback.txt
: > $O
for rep in 1 2; do
  for p in 1 0; do
    echo "STENCIL_TK_PACK_SIG=$p loopback" >> $O
    STENCIL_TK_PACK_SIG=$p timeout -k 10 300 python3 bench.py --exchange loopback --steps 400 --warmup 20 --no-cpu-baseline >> $O 2>/dev/null || exit 1
  done
done
