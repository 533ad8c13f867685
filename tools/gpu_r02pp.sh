#!/bin/bash
# Box K=4 with E pinned (4 x 8 and 2 x 16 rows, both spill 21-30 VGPRs) against
# the default 3 x 8 K=4 strip: per-sweep time, interleaved in one process
# (the pinned variants, cfg 980xxx, were removed after this measurement: the
# script now times the default shape only)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TUNE_STENCIL=box TUNE_DTYPE=fp64 TUNE_SWEEPK=4
for SH in 2048,2048,256 2048,2048,2048 1024,1024,512; do
  IT=24; [ $SH = 2048,2048,2048 ] && IT=12
  echo "== fp64 $SH K=4"
  TUNE_ITERS=$IT TUNE_SHAPE=$SH timeout -k 10 300 python tools/tune.py 512 \
    '[{}, {"STENCIL_BOXK_CFG": "980408"}, {"STENCIL_BOXK_CFG": "980216"}, {"STENCIL_BOXK_CFG": "980312"}]' || exit 1
done
