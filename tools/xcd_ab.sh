# strip kernel: XCD-grouped block order (STENCIL_TK_XCD=1) vs the plain order, per z-chunking
set -o pipefail
V='[{}, {"STENCIL_TK_XCD": 1}, {"STENCIL_TK_ZCHUNK": 256}, {"STENCIL_TK_ZCHUNK": 256, "STENCIL_TK_XCD": 1}, {"STENCIL_TK_ZCHUNK": 128}, {"STENCIL_TK_ZCHUNK": 128, "STENCIL_TK_XCD": 1}]'
echo "== 512^3 fp64"; TUNE_ITERS=48 timeout -k 5 200 python tools/tune.py 512 "$V" || exit 1
echo "== 512^3 fp32"; TUNE_DTYPE=fp32 TUNE_ITERS=48 timeout -k 5 200 python tools/tune.py 512 "$V" || exit 1
echo "== 2048^2x512 fp64"; TUNE_SHAPE=2048,2048,512 TUNE_ITERS=16 timeout -k 5 200 python tools/tune.py 512 '[{}, {"STENCIL_TK_XCD": 1}]' || exit 1
