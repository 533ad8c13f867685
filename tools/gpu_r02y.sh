#!/bin/bash
# Box strip: E pin on/off, interleaved in one process (tools/tune.py), default shapes
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TUNE_STENCIL=box
for SH in 2048,2048,256 512,512,512; do
  for K in 3 4; do
    echo "== fp64 $SH K=$K"
    TUNE_ITERS=24 TUNE_DTYPE=fp64 TUNE_SWEEPK=$K TUNE_SHAPE=$SH timeout -k 10 300 python tools/tune.py 512 '[{},{"STENCIL_BOXK_NOPIN":"1"},{"STENCIL_BOXK_CFG":"910408"},{"STENCIL_BOXK_CFG":"910408","STENCIL_BOXK_NOPIN":"1"}]' || exit 1
  done
  echo "== fp32 $SH K=3"
  TUNE_ITERS=24 TUNE_DTYPE=fp32 TUNE_SWEEPK=3 TUNE_SHAPE=$SH timeout -k 10 300 python tools/tune.py 512 '[{},{"STENCIL_BOXK_NOPIN":"1"}]' || exit 1
done
