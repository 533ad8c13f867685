#!/bin/bash
# 7-point strip: interior fast path (no ghost-cell selects) -- parity, then A/B of STENCIL_TK_FAST
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_slab.py -k "tkstrip or full_size_c2 or benched or temporalk or signalled or slab" -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_fast.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests_fast.log; [ $rc -eq 0 ] || exit $rc
export TUNE_ITERS=100
for SH in 512,512,512 2048,2048,512; do
  echo "== fp64 $SH"
  TUNE_DTYPE=fp64 TUNE_SHAPE=$SH timeout -k 10 300 python tools/tune.py 512 '[{"STENCIL_TK_FAST":"0"},{"STENCIL_TK_FAST":"1"}]' || exit 1
done
export TUNE_ITERS=20
echo "== fp64 2048^3 (NS)"
TUNE_DTYPE=fp64 TUNE_SHAPE=2048,2048,2048 timeout -k 10 300 python tools/tune.py 512 '[{"STENCIL_TK_FAST":"0"},{"STENCIL_TK_FAST":"1"}]' || exit 1
