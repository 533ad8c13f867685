#!/bin/bash
# round 3, final profiles: rocprofv3 kernel trace + stats and FETCH/WRITE passes of the bench commands whose
# traffic the bench line reports (C2 default, C3 on one GPU, C5 on one GPU), on the final kernel sources
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
bash $R/profiles/collect.sh r03z --steps 100 --warmup 5 --no-cpu-baseline > $R/gpurun_out/r03z_collect.log 2>&1 &&
bash $R/profiles/collect.sh r03z_c3 --config C3 --steps 10 --warmup 0 --no-cpu-baseline > $R/gpurun_out/r03z_c3_collect.log 2>&1 &&
bash $R/profiles/collect.sh r03z_c5 --config C5 --steps 8 --warmup 0 --no-cpu-baseline > $R/gpurun_out/r03z_c5_collect.log 2>&1
