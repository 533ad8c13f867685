set -o pipefail
V='[{}, {"STENCIL_TB2D_CFG": 92416}]'
for n in 512 2048 4096; do
  echo "== ${n}^2 fp32 dma"; TUNE_DIMS=2 TUNE_ITERS=100 TUNE_DTYPE=fp32 TUNE_ORDER=dma timeout -k 5 150 python tools/tune.py $n "$V" || exit 1
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "2d or c1 or golden or cli or reference_abi" -x -q --timeout 120 --timeout-method thread 2>&1 | tail -2
