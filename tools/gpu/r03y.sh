#!/bin/bash
# round 3, call y: scheduler variants beyond C2 -- the strip kernel (gcn-max-ilp) at NS 2048^3 and C3 4096^3 fp32
# (rolling), gcn-max-ilp + no clustered low-occupancy reschedule at C2, and the box kernel (gcn-max-memory-clause)
# at C5; alternating runs in separate processes
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/r03y_sched_bench.txt
: > $O
run() { echo "VARIANT $1" >> $O; L=$2; shift 2; timeout -k 10 300 python3 tools/bench_lib.py build/variants/lib_$L.so "$@" --no-cpu-baseline >> $O 2>/dev/null; }
for t in maxilp_nlo maxilp base; do run "$t C2" $t || exit 1; done
for t in base maxilp base maxilp; do run "$t NS" $t --config NS --steps 40 --warmup 4 || exit 1; done
for t in boxbase boxmemclause boxbase boxmemclause; do run "$t C5" $t --config C5 --steps 16 --warmup 4 || exit 1; done
for t in base maxilp; do run "$t C3" $t --config C3 --steps 20 --warmup 0 || exit 1; done
