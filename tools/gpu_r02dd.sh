#!/bin/bash
# Box: packed longest-first z-chunk schedule for few-tile grids -- parity, then A/B (STENCIL_BOXK_PACK)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_slab.py tests/test_gpu_slab_job.py -k "box or slab_job" -x -q --timeout 200 --timeout-method thread > gpurun_out/box_pack_tests.log 2>&1
rc=$?; tail -2 gpurun_out/box_pack_tests.log; [ $rc -eq 0 ] || exit $rc
export TUNE_STENCIL=box STENCIL_TK_VERBOSE=1
for SH in 512,512,512 400,400,400 640,640,320; do
  for DT in fp64 fp32; do
    echo "== $DT $SH K=auto"
    TUNE_ITERS=24 TUNE_DTYPE=$DT TUNE_SHAPE=$SH timeout -k 10 300 python tools/tune.py 512 '[{},{"STENCIL_BOXK_PACK":"0"}]' 2> gpurun_out/pack_verbose_${DT}_$SH.log || exit 1
    grep -m2 "pack (family 1)" gpurun_out/pack_verbose_${DT}_$SH.log
  done
done
