#!/bin/bash
# Packed schedule vs equal chunks vs the interior fast path, over shapes
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=r02gg
for s in 504,512,512 512,480,512 512,512,512 256,256,256 320,320,320 384,384,384 400,400,400 448,448,448 640,640,640 768,768,256; do
  echo "== shape $s" >> gpurun_out/${TAG}_pack.log
  TUNE_SHAPE=$s TUNE_ITERS=200 timeout -k 10 120 python -u tools/tune.py 512 '[{}, {"STENCIL_TK_PACK": 0}, {"STENCIL_TK_FAST": 0}, {"STENCIL_TK_PACK": 0, "STENCIL_TK_FAST": 1}]' >> gpurun_out/${TAG}_pack.log 2>&1 || exit 1
done
