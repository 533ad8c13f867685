# 2D column kernel (one 64 x RYC region per wave, no LDS, no barrier) vs the default strips, C1
set -o pipefail
V='[{}, {"STENCIL_TB2D_CFG": 936404, "STENCIL_TB2D_K": 10}, {"STENCIL_TB2D_CFG": 936404, "STENCIL_TB2D_K": 14}, {"STENCIL_TB2D_CFG": 934804, "STENCIL_TB2D_K": 8}, {"STENCIL_TB2D_CFG": 936401, "STENCIL_TB2D_K": 12}, {"STENCIL_TB2D_CFG": 939604, "STENCIL_TB2D_K": 16}]'
echo "== C1 fp64 naive"; TUNE_DIMS=2 TUNE_ITERS=100 timeout -k 5 150 python tools/tune.py 1024 "$V" || exit 1
echo "== C1r fp32 dma"; TUNE_DIMS=2 TUNE_ITERS=100 TUNE_DTYPE=fp32 TUNE_ORDER=dma timeout -k 5 150 python tools/tune.py 1024 "$V" || exit 1
