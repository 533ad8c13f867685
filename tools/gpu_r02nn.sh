#!/bin/bash
# next plane's loads issued row by row (SL) vs one burst at the end of the step
# (the SL variant was removed after this run: no gain)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=r02nn
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "tkstrip_chunking and (910708 or 930708 or 920708)" > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -2 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
for s in 512,512,512 2048,2048,512; do
  echo "== fp64 shape $s" >> gpurun_out/${TAG}_ab.log
  TUNE_SHAPE=$s TUNE_ITERS=100 timeout -k 10 200 python -u tools/tune.py 512 '[{}, {"STENCIL_TK_STRIP": 910708}, {"STENCIL_TK_STRIP": 710708}, {"STENCIL_TK_STRIP": 930708}]' >> gpurun_out/${TAG}_ab.log 2>&1 || exit 1
done
for s in 512,512,512 2048,2048,512; do
  echo "== fp32 shape $s" >> gpurun_out/${TAG}_ab.log
  TUNE_DTYPE=fp32 TUNE_SHAPE=$s TUNE_ITERS=100 timeout -k 10 200 python -u tools/tune.py 512 '[{}, {"STENCIL_TK_STRIP": 920708}]' >> gpurun_out/${TAG}_ab.log 2>&1 || exit 1
done
