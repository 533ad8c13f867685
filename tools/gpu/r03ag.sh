#!/bin/bash
# round 3, call ag: the face-signalled slab kernels (SIG, default strip file) under gcn-max-ilp vs default:
# the single-GPU interior-rank rehearsal (periodic halos by device copies), alternating, separate processes
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/r03ag_sig_sched.txt
: > $O
for rep in 1 2; do
  for t in sbase silp; do
    echo "VARIANT $t loopback" >> $O
    timeout -k 10 300 python3 tools/bench_lib.py build/variants/lib_$t.so --exchange loopback --steps 400 --warmup 20 --no-cpu-baseline >> $O 2>/dev/null || exit 1
  done
done
