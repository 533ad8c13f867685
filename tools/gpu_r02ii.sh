#!/bin/bash
# 512^3 fp64 K=4: packed chunk length sweep (STENCIL_TK_PACK_LC, model bypassed) vs equal chunks
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=r02ii
V='[{"STENCIL_TK_PACK": 0}, {"STENCIL_TK_PACK": 2}'
for lc in 100 128 150 171 200 215 230 245 256 280 300 342 400; do V="$V, {\"STENCIL_TK_PACK\": 2, \"STENCIL_TK_PACK_LC\": $lc}"; done
V="$V]"
TUNE_SHAPE=512,512,512 TUNE_ITERS=200 STENCIL_TK_VERBOSE=1 timeout -k 10 300 python -u tools/tune.py 512 "$V" 2>&1 | grep -v "^tkstrip" > gpurun_out/${TAG}_lc.log || exit 1
