#!/bin/bash
# Box: strip layout (box27_strip, cfg 9VRRNN) vs the interleaved default, K = 3 and pairs (tools/tune.py)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_slab.py -k "box_strip_shapes or box_sweepk_signal" -x -q --timeout 120 --timeout-method thread > gpurun_out/box_strip_tests.log 2>&1
rc=$?; tail -3 gpurun_out/box_strip_tests.log; [ $rc -eq 0 ] || exit $rc
export TUNE_STENCIL=box TUNE_ITERS=24
for SH in 2048,2048,256 512,512,512 2048,2048,2048; do
  [ $SH = 2048,2048,2048 ] && export TUNE_ITERS=6
  echo "== fp64 $SH K=3"
  TUNE_DTYPE=fp64 TUNE_SWEEPK=3 TUNE_SHAPE=$SH timeout -k 10 300 python tools/tune.py 512 \
    '[{},{"STENCIL_BOXK_CFG":"910408"},{"STENCIL_BOXK_CFG":"910308"},{"STENCIL_BOXK_CFG":"910312"},{"STENCIL_BOXK_CFG":"910212"},{"STENCIL_BOXK_CFG":"910216"}]' || exit 1
  echo "== fp32 $SH K=3"
  TUNE_DTYPE=fp32 TUNE_SWEEPK=3 TUNE_SHAPE=$SH timeout -k 10 300 python tools/tune.py 512 \
    '[{},{"STENCIL_BOXK_CFG":"920408"},{"STENCIL_BOXK_CFG":"920312"},{"STENCIL_BOXK_CFG":"920216"}]' || exit 1
  [ $SH = 2048,2048,2048 ] && continue
  echo "== fp64 $SH K=2"
  TUNE_DTYPE=fp64 TUNE_SWEEPK=2 TUNE_SHAPE=$SH timeout -k 10 200 python tools/tune.py 512 \
    '[{},{"STENCIL_BOXK_CFG":"910408"},{"STENCIL_BOXK_CFG":"910312"},{"STENCIL_BOXK_CFG":"910216"}]' || exit 1
  echo "== fp32 $SH K=2"
  TUNE_DTYPE=fp32 TUNE_SWEEPK=2 TUNE_SHAPE=$SH timeout -k 10 200 python tools/tune.py 512 \
    '[{},{"STENCIL_BOXK_CFG":"920408"},{"STENCIL_BOXK_CFG":"920312"},{"STENCIL_BOXK_CFG":"940208"}]' || exit 1
done
