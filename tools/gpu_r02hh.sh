#!/bin/bash
# measured packed-vs-equal schedule choice: parity tests, per-shape A/B, default bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=r02hh
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "schedule_choice or benched_kernel or packed" > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
for s in 504,512,512 256,256,256 448,448,448 512,512,512 400,400,400; do
  echo "== shape $s" >> gpurun_out/${TAG}_pick.log
  TUNE_SHAPE=$s TUNE_ITERS=200 STENCIL_TK_VERBOSE=1 timeout -k 10 120 python -u tools/tune.py 512 '[{}, {"STENCIL_TK_PACK": 2}, {"STENCIL_TK_PACK": 0}]' 2>&1 | grep -v "^tkstrip" >> gpurun_out/${TAG}_pick.log || exit 1
done
echo "== box" >> gpurun_out/${TAG}_pick.log
for s in 400,400,400 512,512,512 256,256,256; do
  echo "== box shape $s" >> gpurun_out/${TAG}_pick.log
  TUNE_STENCIL=box TUNE_SHAPE=$s TUNE_ITERS=60 STENCIL_TK_VERBOSE=1 timeout -k 10 120 python -u tools/tune.py 512 '[{}, {"STENCIL_BOXK_PACK": 2}, {"STENCIL_BOXK_PACK": 0}]' 2>&1 | grep -v "^tkstrip" >> gpurun_out/${TAG}_pick.log || exit 1
done
timeout -k 10 300 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit 1
cat gpurun_out/${TAG}_bench.json
