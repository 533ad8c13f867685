#!/bin/bash
# Does the ragged last tile column / row cost the 512^3 bench time?  Same kernel,
# shapes that tile exactly (504 = 9 x 56 in x, 480 = 10 x 48 in y) vs 512.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=r02ff
for s in 512,512,512 504,512,512 512,480,512 504,480,512 560,528,512; do
  echo "== shape $s" >> gpurun_out/${TAG}_ragged.log
  TUNE_SHAPE=$s TUNE_ITERS=200 STENCIL_TK_VERBOSE=1 timeout -k 10 120 python -u tools/tune.py 512 '[{}, {"STENCIL_TK_PACK": 0}]' >> gpurun_out/${TAG}_ragged.log 2>&1 || exit 1
done
