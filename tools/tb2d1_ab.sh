set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "2d or c1 or golden or cli or reference_abi" -x -q --timeout 120 --timeout-method thread 2>&1 | tail -2 || exit 1
V='[{}, {"STENCIL_TB2D_SINGLE": 0}]'
for n in 32 64 96 128; do
  echo "== ${n}^2 fp32 dma"; TUNE_DIMS=2 TUNE_ITERS=1000 TUNE_DTYPE=fp32 TUNE_ORDER=dma timeout -k 5 150 python tools/tune.py $n "$V" || exit 1
  echo "== ${n}^2 fp64 naive"; TUNE_DIMS=2 TUNE_ITERS=1000 timeout -k 5 150 python tools/tune.py $n "$V" || exit 1
done
