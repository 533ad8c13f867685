# 27-point box kernels: parity, then interleaved A/B of the 2-step BOXK shapes (tools/tune.py)
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_slab.py -k "box" -x -q --timeout 120 --timeout-method thread > gpurun_out/box_tests.log 2>&1 || { tail -30 gpurun_out/box_tests.log; exit 1; }
tail -1 gpurun_out/box_tests.log
export TUNE_STENCIL=box TUNE_ITERS=24 TUNE_KERNEL=temporal2
for DT in fp64 fp32; do
for SH in 512,512,512 2048,2048,256; do
  echo "== $DT $SH"
  TUNE_DTYPE=$DT TUNE_SHAPE=$SH timeout -k 10 200 python tools/tune.py 512 '[{},{"STENCIL_BOXK_CFG":"1116"},{"STENCIL_BOXK_CFG":"116"},{"STENCIL_BOXK_CFG":"1416"}]'
done
done
