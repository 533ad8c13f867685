#!/bin/bash
# saddr row offsets (row_off) in the strip / box kernels: full GPU suite, then the 7-point A/B of the fast path
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r02p.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests_r02p.log; [ $rc -eq 0 ] || exit $rc
export TUNE_ITERS=100
for SH in 512,512,512 2048,2048,512; do
  echo "== fp64 $SH"
  TUNE_DTYPE=fp64 TUNE_SHAPE=$SH timeout -k 10 300 python tools/tune.py 512 '[{},{"STENCIL_TK_FAST":"0"},{"STENCIL_TK_STRIP":"710708"}]' || exit 1
done
echo "== fp32 512^3"
TUNE_DTYPE=fp32 TUNE_SHAPE=512,512,512 timeout -k 10 300 python tools/tune.py 512 '[{}]' || exit 1
echo "== box fp64 / fp32 K=3 2048^2x256"
export TUNE_STENCIL=box TUNE_ITERS=24 TUNE_SWEEPK=3 TUNE_SHAPE=2048,2048,256
TUNE_DTYPE=fp64 timeout -k 10 300 python tools/tune.py 512 '[{},{"STENCIL_BOXK_CFG":"910408"}]' || exit 1
TUNE_DTYPE=fp32 timeout -k 10 300 python tools/tune.py 512 '[{}]' || exit 1
