#!/bin/bash
# round 3, call ad: second scheduler sweep -- variants of the max-ILP strip file at C2 (and C3's fp32 K = 5
# kernel shares the file), variants of the default strip file at NS; alternating, separate processes
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/r03ad_sched2.txt
: > $O
run() { echo "VARIANT $1" >> $O; L=$2; shift 2; timeout -k 10 300 python3 tools/bench_lib.py build/variants/lib_$L.so "$@" --no-cpu-baseline >> $O 2>/dev/null; }
for t in ilp ilp_aa ilp_nocl ilp_td ilp_bi ilp_post ilp; do run "$t C2" $t || exit 1; done
for rep in 1 2; do
  for t in m_base m_mc m_aa m_nocl m_td; do run "$t NS" $t --config NS --steps 40 --warmup 4 || exit 1; done
done
