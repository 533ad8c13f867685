#!/bin/bash
# round 3, call m: rocprof + PMC of the C5 bench on the new box kernel (traffic table), and the C5 interior-rank
# rehearsal (face-signalled 5 x 8 K = 4 rounds, periodic halos by device copies)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
bash $R/profiles/collect.sh r03z2_c5 --config C5 --steps 8 --warmup 0 --no-cpu-baseline > $R/gpurun_out/r03z2_c5_collect.log 2>&1 &&
cd $R && timeout -k 10 300 python3 bench.py --config C5 --exchange loopback --steps 32 --warmup 4 --no-cpu-baseline \
  > gpurun_out/r03m_bench_c5_loopback.json 2> gpurun_out/r03m_bench_c5_loopback.err
