#!/bin/bash
# Separable-sum box kernel (round 2): workgroup shapes and K, interleaved A/B (tools/tune.py)
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TUNE_STENCIL=box TUNE_ITERS=24
for DT in fp64 fp32; do
  for SH in 512,512,512 2048,2048,256; do
    echo "== $DT $SH pairs (K=2)"
    TUNE_DTYPE=$DT TUNE_KERNEL=temporal2 TUNE_SHAPE=$SH timeout -k 10 200 python tools/tune.py 512 \
      '[{},{"STENCIL_BOXK_CFG":"216"},{"STENCIL_BOXK_CFG":"208"},{"STENCIL_BOXK_CFG":"308"},{"STENCIL_BOXK_CFG":"408"},{"STENCIL_BOXK_CFG":"10116"},{"STENCIL_BOXK_CFG":"10216"},{"STENCIL_BOXK_CFG":"20116"}]'
    echo "== $DT $SH K=3 sweepk"
    TUNE_DTYPE=$DT TUNE_SWEEPK=3 TUNE_SHAPE=$SH timeout -k 10 200 python tools/tune.py 512 \
      '[{},{"STENCIL_BOXK_CFG":"208"},{"STENCIL_BOXK_CFG":"308"}]'
  done
done
