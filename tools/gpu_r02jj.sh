#!/bin/bash
# 8-cell x ring (48-cell output rows, aligned stores) vs the default 4-cell ring
# (the variant, STENCIL_TK_CFG=810708, and its checker were removed after this run)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=r02jj
timeout -k 10 120 python -u tools/xring_check.py > gpurun_out/${TAG}_check.log 2>&1 || { cat gpurun_out/${TAG}_check.log; exit 1; }
for s in 512,512,512 2048,2048,512 528,528,512; do
  echo "== shape $s" >> gpurun_out/${TAG}_ab.log
  TUNE_SHAPE=$s TUNE_ITERS=100 timeout -k 10 200 python -u tools/tune.py 512 '[{}, {"STENCIL_TK_CFG": 810708}, {"STENCIL_TK_PACK": 0}, {"STENCIL_TK_CFG": 810708, "STENCIL_TK_PACK": 0}]' >> gpurun_out/${TAG}_ab.log 2>&1 || exit 1
done
