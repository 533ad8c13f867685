# A/B of the 27-point box kernels (single sweep, 2-step BOXK shapes, 3-step BOXK shapes)
set -e
mkdir -p gpurun_out
export TUNE_STENCIL=box TUNE_ITERS=24
for DT in fp64 fp32; do
for SH in 512,512,512 2048,2048,256; do
  echo "== $DT shape $SH single"
  TUNE_DTYPE=$DT TUNE_SHAPE=$SH TUNE_KERNEL=auto timeout -k 10 120 python tools/tune.py 512 '[{}]'
  echo "== $DT shape $SH fused2"
  TUNE_DTYPE=$DT TUNE_SHAPE=$SH TUNE_KERNEL=temporal2 timeout -k 10 200 python tools/tune.py 512 '[{},{"STENCIL_BOXK_CFG":"208"},{"STENCIL_BOXK_CFG":"116"}]'
  echo "== $DT shape $SH sweepk3"
  TUNE_DTYPE=$DT TUNE_SHAPE=$SH TUNE_SWEEPK=3 TUNE_KERNEL=auto timeout -k 10 120 python tools/tune.py 512 '[{},{"STENCIL_BOXK_CFG":"208"}]'
done
done
