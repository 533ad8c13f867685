#!/bin/bash
# Box strip with pinned E row sums (fewer VGPRs): parity of every strip shape, then A/B of shapes per K
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_slab.py -k "box" -x -q --timeout 200 --timeout-method thread > gpurun_out/box_pin_tests.log 2>&1
rc=$?; tail -2 gpurun_out/box_pin_tests.log; [ $rc -eq 0 ] || exit $rc
export TUNE_STENCIL=box
for SH in 2048,2048,256 512,512,512; do
  echo "== fp64 $SH K=3"
  TUNE_ITERS=24 TUNE_DTYPE=fp64 TUNE_SWEEPK=3 TUNE_SHAPE=$SH timeout -k 10 300 python tools/tune.py 512 '[{},{"STENCIL_BOXK_CFG":"910408"},{"STENCIL_BOXK_CFG":"910216"},{"STENCIL_BOXK_CFG":"910312"},{"STENCIL_BOXK_CFG":"910508"}]' || exit 1
  echo "== fp64 $SH K=4"
  TUNE_ITERS=24 TUNE_DTYPE=fp64 TUNE_SWEEPK=4 TUNE_SHAPE=$SH timeout -k 10 300 python tools/tune.py 512 '[{},{"STENCIL_BOXK_CFG":"910408"}]' || exit 1
  echo "== fp32 $SH K=3"
  TUNE_ITERS=24 TUNE_DTYPE=fp32 TUNE_SWEEPK=3 TUNE_SHAPE=$SH timeout -k 10 300 python tools/tune.py 512 '[{}]' || exit 1
  echo "== fp32 $SH K=4"
  TUNE_ITERS=24 TUNE_DTYPE=fp32 TUNE_SWEEPK=4 TUNE_SHAPE=$SH timeout -k 10 300 python tools/tune.py 512 '[{}]' || exit 1
done
