# 7-point fp64 K=4 strip kernel: input ring depth (NS planes, NS-2 in flight) x rows per wave
set -o pipefail
V='[{}, {"STENCIL_TK_STRIP": 510708}, {"STENCIL_TK_STRIP": 510608}, {"STENCIL_TK_STRIP": 610608}, {"STENCIL_TK_STRIP": 610508}]'
echo "== 512^3 fp64"; TUNE_ITERS=48 timeout -k 5 200 python tools/tune.py 512 "$V" || exit 1
echo "== 2048^2x512 fp64"; TUNE_SHAPE=2048,2048,512 TUNE_ITERS=16 timeout -k 5 200 python tools/tune.py 512 "$V" || exit 1
