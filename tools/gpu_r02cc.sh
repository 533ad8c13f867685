#!/bin/bash
# C1 (1024^2 fp64 2D 5-point, 100 sweeps): kernel trace + SQ counters of the strip kernel tb2ds
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TUNE_DIMS=2 TUNE_SHAPE=1024,1024,1 TUNE_ITERS=100 TUNE_KERNEL=auto TUNE_DTYPE=fp64
timeout -k 10 200 python tools/tune.py 1024 '[{}]' || exit 1
bash tools/pmc_variants.sh c1 "STENCIL_DUMMY=0" || exit 1
python tools/pmc_table.py c1 tb2ds > gpurun_out/pmc_c1_table.json
cat gpurun_out/pmc_c1_table.json | head -60
