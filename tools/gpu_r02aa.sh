#!/bin/bash
# Box fp64 K=3 vs K=4 around the AUTO threshold (planes of 1024^2 cells), and 768^2
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TUNE_STENCIL=box TUNE_DTYPE=fp64
for SH in 1024,1024,512 768,768,512 1536,1536,256; do
  for K in 3 4; do
    echo "== $SH K=$K"
    TUNE_ITERS=24 TUNE_SWEEPK=$K TUNE_SHAPE=$SH timeout -k 10 300 python tools/tune.py 512 '[{}]' || exit 1
  done
done
