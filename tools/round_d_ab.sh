# strip kernel chunk model: per-round cost D = 4 (default) vs 0 (rounds x (chunk + 2K) only)
set -o pipefail
V='[{}, {"STENCIL_TK_ROUND_D": 0}]'
echo "== 512^3 fp64"; TUNE_ITERS=100 timeout -k 5 200 python tools/tune.py 512 "$V" || exit 1
echo "== 512^3 fp32"; TUNE_DTYPE=fp32 TUNE_ITERS=100 timeout -k 5 200 python tools/tune.py 512 "$V" || exit 1
echo "== 2048^2x512 fp64"; TUNE_SHAPE=2048,2048,512 TUNE_ITERS=16 timeout -k 5 200 python tools/tune.py 512 "$V" || exit 1
echo "== 4096^2x1024 fp32"; TUNE_DTYPE=fp32 TUNE_SHAPE=4096,4096,1024 TUNE_ITERS=10 timeout -k 5 300 python tools/tune.py 512 "$V" || exit 1
echo "== 768^3 fp64"; TUNE_ITERS=24 timeout -k 5 200 python tools/tune.py 768 "$V" || exit 1
echo "== 256^3 fp64"; TUNE_ITERS=200 timeout -k 5 200 python tools/tune.py 256 "$V" || exit 1
