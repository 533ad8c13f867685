# 2D fp64: 128 x 64 regions as 16 waves x 4 rows (default) vs 8 waves x 8 rows, sweeps per launch by the round rule
set -o pipefail
V='[{}, {"STENCIL_TB2D_CFG": 92808}]'
for n in 512 1024 2048 4096; do
  echo "== ${n}^2 fp64 naive"; TUNE_DIMS=2 TUNE_ITERS=100 timeout -k 5 150 python tools/tune.py $n "$V" || exit 1
  echo "== ${n}^2 fp64 dma"; TUNE_DIMS=2 TUNE_ITERS=100 TUNE_ORDER=dma timeout -k 5 150 python tools/tune.py $n "$V" || exit 1
done
