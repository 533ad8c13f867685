# A/B: the persistent 2D kernel (one launch per job) vs the K-step launches, C1 (1024^2, 100 iterations)
set -o pipefail
V='[{}, {"STENCIL_TB2DP": 1}, {"STENCIL_TB2DP": 1, "STENCIL_TB2DP_K": 4}, {"STENCIL_TB2DP": 1, "STENCIL_TB2DP_K": 12}, {"STENCIL_TB2DP": 1, "STENCIL_TB2DP_K": 16}]'
echo "== C1 fp64 naive"; TUNE_DIMS=2 TUNE_ITERS=100 timeout -k 5 120 python tools/tune.py 1024 "$V" || exit 1
echo "== C1r fp32 dma"; TUNE_DIMS=2 TUNE_ITERS=100 TUNE_DTYPE=fp32 TUNE_ORDER=dma timeout -k 5 120 python tools/tune.py 1024 "$V" || exit 1
echo "== 2048^2 fp64"; TUNE_DIMS=2 TUNE_ITERS=100 timeout -k 5 120 python tools/tune.py 2048 "$V" || exit 1
echo "== 512^2 fp64"; TUNE_DIMS=2 TUNE_ITERS=100 timeout -k 5 120 python tools/tune.py 512 "$V" || exit 1
