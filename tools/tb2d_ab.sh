# 2D tile-resident kernels (kernels_tb2d.hip): parity, then A/B of region shapes and K (tools/tune.py)
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "tile_resident" -x -q --timeout 120 --timeout-method thread > gpurun_out/tb2d_tests.log 2>&1 || { tail -30 gpurun_out/tb2d_tests.log; exit 1; }
tail -1 gpurun_out/tb2d_tests.log
export TUNE_DIMS=2 TUNE_ITERS=100 TUNE_KERNEL=auto TUNE_SHAPE=1024,1024
for DT in fp64 fp32; do
  echo "== $DT 1024^2"
  TUNE_DTYPE=$DT timeout -k 10 200 python tools/tune.py 1024 '[{},{"STENCIL_TB2D_CFG":"92808"},{"STENCIL_TB2D_CFG":"92816"},{"STENCIL_TB2D_CFG":"94808"},{"STENCIL_TB2D_CFG":"92816","STENCIL_TB2D_K":"12"},{"STENCIL_TB2D_CFG":"92816","STENCIL_TB2D_K":"16"},{"STENCIL_TB2D_CFG":"94808","STENCIL_TB2D_K":"12"},{"STENCIL_TB2D_CFG":"92808","STENCIL_TB2D_K":"12"}]'
done
