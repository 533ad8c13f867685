#!/bin/bash
# round 3, call af: rocprof + PMC (FETCH / WRITE passes) of C2 and C3 on the final strip sources (max-ILP build)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
bash $R/profiles/collect.sh r03z4 --steps 100 --warmup 5 --no-cpu-baseline > $R/gpurun_out/r03z4_collect.log 2>&1 &&
bash $R/profiles/collect.sh r03z4_c3 --config C3 --steps 10 --warmup 0 --no-cpu-baseline > $R/gpurun_out/r03z4_c3_collect.log 2>&1
