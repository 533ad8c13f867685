#!/bin/bash
# Box: K = 3 (sweepk) with narrower lanes vs the default pairs (tools/tune.py)
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TUNE_STENCIL=box TUNE_ITERS=24
for SH in 2048,2048,256 512,512,512; do
  echo "== fp64 $SH pairs (default)"
  TUNE_DTYPE=fp64 TUNE_KERNEL=temporal2 TUNE_SHAPE=$SH timeout -k 10 200 python tools/tune.py 512 '[{}]'
  echo "== fp64 $SH K=3"
  TUNE_DTYPE=fp64 TUNE_SWEEPK=3 TUNE_SHAPE=$SH timeout -k 10 200 python tools/tune.py 512 \
    '[{},{"STENCIL_BOXK_CFG":"10116"},{"STENCIL_BOXK_CFG":"10308"},{"STENCIL_BOXK_CFG":"10216"}]'
  echo "== fp32 $SH pairs (default)"
  TUNE_DTYPE=fp32 TUNE_KERNEL=temporal2 TUNE_SHAPE=$SH timeout -k 10 200 python tools/tune.py 512 '[{}]'
  echo "== fp32 $SH K=3"
  TUNE_DTYPE=fp32 TUNE_SWEEPK=3 TUNE_SHAPE=$SH timeout -k 10 200 python tools/tune.py 512 \
    '[{},{"STENCIL_BOXK_CFG":"20116"},{"STENCIL_BOXK_CFG":"20308"},{"STENCIL_BOXK_CFG":"20216"}]'
done
