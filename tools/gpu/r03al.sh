#!/bin/bash
# round 3, call al: rocprof + PMC of C2 (schedule pinned to the model's packed grid, STENCIL_TK_PACK=2) and C3 on
# the final sources
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
STENCIL_TK_PACK=2 bash $R/profiles/collect.sh r03z7 --steps 100 --warmup 5 --no-cpu-baseline > $R/gpurun_out/r03z7_collect.log 2>&1 &&
bash $R/profiles/collect.sh r03z7_c3 --config C3 --steps 10 --warmup 0 --no-cpu-baseline > $R/gpurun_out/r03z7_c3_collect.log 2>&1
