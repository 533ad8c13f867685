# 27-point box fp64 shapes: rows per wave x waves (tools/tune.py, fused pairs)
set -e
export TUNE_STENCIL=box TUNE_ITERS=24 TUNE_KERNEL=temporal2 TUNE_DTYPE=fp64
for SH in 512,512,512 2048,2048,256; do
  echo "== fp64 $SH"
  TUNE_SHAPE=$SH timeout -k 10 200 python tools/tune.py 512 '[{},{"STENCIL_BOXK_CFG":"208"},{"STENCIL_BOXK_CFG":"308"},{"STENCIL_BOXK_CFG":"216"},{"STENCIL_BOXK_CFG":"212"},{"STENCIL_BOXK_CFG":"408"}]'
done
