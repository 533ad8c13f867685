# z-chunk A/B of the strip kernel on the bench configs (per-GPU shapes)
set -o pipefail
V='[{}, {"STENCIL_TK_ZCHUNK": 512}, {"STENCIL_TK_ZCHUNK": 256}, {"STENCIL_TK_ZCHUNK": 171}, {"STENCIL_TK_ZCHUNK": 128}]'
echo "== 512^3 fp64"; timeout -k 5 120 python tools/tune.py 512 "$V" || exit 1
echo "== 512^3 fp32"; TUNE_DTYPE=fp32 timeout -k 5 120 python tools/tune.py 512 "$V" || exit 1
echo "== 2048x2048x512 fp64"; TUNE_SHAPE=2048,2048,512 TUNE_ITERS=20 timeout -k 5 200 python tools/tune.py 512 "$V" || exit 1
echo "== 1024^3 fp32"; TUNE_DTYPE=fp32 TUNE_ITERS=20 timeout -k 5 200 python tools/tune.py 1024 '[{}, {"STENCIL_TK_ZCHUNK": 1024}, {"STENCIL_TK_ZCHUNK": 512}, {"STENCIL_TK_ZCHUNK": 342}, {"STENCIL_TK_ZCHUNK": 256}]' || exit 1
