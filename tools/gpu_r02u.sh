#!/bin/bash
# Box K=4 (strip 3x8): parity, then per-sweep time against the K=3 defaults
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "box_strip_shapes" -x -q --timeout 120 --timeout-method thread > gpurun_out/box_k4_tests.log 2>&1
rc=$?; tail -2 gpurun_out/box_k4_tests.log; [ $rc -eq 0 ] || exit $rc
export TUNE_STENCIL=box
for SH in 2048,2048,256 512,512,512 2048,2048,2048; do
  IT=24; [ $SH = 2048,2048,2048 ] && IT=12
  for DT in fp64 fp32; do
    echo "== $DT $SH K=3 default"
    TUNE_ITERS=$IT TUNE_DTYPE=$DT TUNE_SWEEPK=3 TUNE_SHAPE=$SH timeout -k 10 300 python tools/tune.py 512 '[{}]' || exit 1
    echo "== $DT $SH K=4"
    TUNE_ITERS=$IT TUNE_DTYPE=$DT TUNE_SWEEPK=4 TUNE_SHAPE=$SH timeout -k 10 300 python tools/tune.py 512 '[{}]' || exit 1
  done
done
