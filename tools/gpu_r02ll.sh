#!/bin/bash
# 7-point K=4 fp64 strip with 3 / 4 waves per SIMD (4 rows x 12 waves, 156 VGPRs;
# 3 rows x 16 waves, 125 VGPRs) vs the default 7 rows x 8 waves (252 VGPRs)
# (shapes 10412 / 10316 removed after this run: slower)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=r02ll
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "tkstrip_chunking and (10412 or 10316)" > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -2 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
for s in 512,512,512 2048,2048,512 504,480,512; do
  echo "== shape $s" >> gpurun_out/${TAG}_ab.log
  TUNE_SHAPE=$s TUNE_ITERS=100 timeout -k 10 200 python -u tools/tune.py 512 '[{}, {"STENCIL_TK_STRIP": 10412}, {"STENCIL_TK_STRIP": 10316}]' >> gpurun_out/${TAG}_ab.log 2>&1 || exit 1
done
