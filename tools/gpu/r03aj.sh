#!/bin/bash
# round 3, call aj: C2 rocprof + PMC with the schedule fixed to the model's choice (STENCIL_TK_PACK=2: packed at
# 512^3, as the timing trial picks in the plain bench runs; under --pmc the trial's timing is distorted and can
# pick the equal chunks, which r03z5's FETCH pass did)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
STENCIL_TK_PACK=2 bash $R/profiles/collect.sh r03z6 --steps 100 --warmup 5 --no-cpu-baseline > $R/gpurun_out/r03z6_collect.log 2>&1
