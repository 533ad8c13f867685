#!/bin/bash
# round 3, call x: the product library with kernels_strip.hip compiled under different machine-scheduler
# choices (tools/lib_variants.sh; device-only -mllvm flags), the bench's C2 workload, alternating, 2 runs each
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/r03x_sched_bench.txt
: > $O
for rep in 1 2; do
  for t in base maxilp memclause iterilp nounclust nopostra; do
    echo "VARIANT $t C2" >> $O
    timeout -k 10 200 python3 tools/bench_lib.py build/variants/lib_$t.so --no-cpu-baseline >> $O 2>/dev/null || exit 1
  done
done
