# 512^3 fp64: default chunking vs 2 chunks (one round) vs 2 chunks + XCD-grouped order, two processes
set -o pipefail
V='[{}, {"STENCIL_TK_ZCHUNK": 256}, {"STENCIL_TK_ZCHUNK": 256, "STENCIL_TK_XCD": 1}, {"STENCIL_TK_XCD": 1}]'
for r in 1 2; do
  echo "== run $r 512^3 fp64"; TUNE_ITERS=100 timeout -k 5 200 python tools/tune.py 512 "$V" || exit 1
done
echo "== 1024^2x512 fp64"; TUNE_SHAPE=1024,1024,512 TUNE_ITERS=40 timeout -k 5 200 python tools/tune.py 512 "$V" || exit 1
echo "== 640^3 fp64"; TUNE_ITERS=40 timeout -k 5 200 python tools/tune.py 640 "$V" || exit 1
