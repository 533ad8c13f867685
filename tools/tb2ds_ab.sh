# C1 (1024^2, 100 iterations): register-strip region shapes x sweeps per launch
set -o pipefail
V='[{}, {"STENCIL_TB2D_K": 10}, {"STENCIL_TB2D_K": 12}, {"STENCIL_TB2D_K": 13}, {"STENCIL_TB2D_K": 14}, {"STENCIL_TB2D_K": 16}, {"STENCIL_TB2D_CFG": 92816, "STENCIL_TB2D_K": 16}, {"STENCIL_TB2D_CFG": 92816, "STENCIL_TB2D_K": 20}, {"STENCIL_TB2D_CFG": 92816, "STENCIL_TB2D_K": 24}]'
echo "== C1 fp64 naive"; TUNE_DIMS=2 TUNE_ITERS=100 timeout -k 5 150 python tools/tune.py 1024 "$V" || exit 1
echo "== C1r fp32 dma"; TUNE_DIMS=2 TUNE_ITERS=100 TUNE_DTYPE=fp32 TUNE_ORDER=dma timeout -k 5 150 python tools/tune.py 1024 "$V" || exit 1
echo "== 2048^2 fp64 naive"; TUNE_DIMS=2 TUNE_ITERS=100 timeout -k 5 150 python tools/tune.py 2048 "$V" || exit 1
echo "== 512^2 fp32 naive"; TUNE_DIMS=2 TUNE_ITERS=100 TUNE_DTYPE=fp32 timeout -k 5 150 python tools/tune.py 512 "$V" || exit 1
