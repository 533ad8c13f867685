# Wider strip regions (12 / 16 waves per workgroup: less y over-fetch, one
# workgroup per CU): parity of the new shapes, then interleaved A/B
# (tools/tune.py) against the defaults.
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "tkstrip_chunking and (10716 or 10712 or 10612 or 10512 or 20716 or 20712 or 20512)" -x -q --timeout 120 --timeout-method thread > gpurun_out/strip_wide_tests.log 2>&1 || { tail -30 gpurun_out/strip_wide_tests.log; exit 1; }
tail -2 gpurun_out/strip_wide_tests.log
export TUNE_KERNEL=temporalk TUNE_ITERS=60
echo "== fp64 512"
TUNE_DTYPE=fp64 timeout -k 10 300 python tools/tune.py 512 '[{},{"STENCIL_TK_STRIP":"10716"},{"STENCIL_TK_STRIP":"10712"},{"STENCIL_TK_STRIP":"10612"},{"STENCIL_TK_STEPS":"5","STENCIL_TK_STRIP":"10512"}]'
echo "== fp64 2048x2048x512"
TUNE_SHAPE=2048,2048,512 TUNE_ITERS=20 TUNE_DTYPE=fp64 timeout -k 10 300 python tools/tune.py 512 '[{},{"STENCIL_TK_STRIP":"10716"},{"STENCIL_TK_STRIP":"10712"}]'
echo "== fp32 2048x2048x512"
TUNE_SHAPE=2048,2048,512 TUNE_ITERS=20 TUNE_DTYPE=fp32 timeout -k 10 300 python tools/tune.py 512 '[{},{"STENCIL_TK_STEPS":"4"},{"STENCIL_TK_STEPS":"4","STENCIL_TK_STRIP":"20716"},{"STENCIL_TK_STEPS":"4","STENCIL_TK_STRIP":"20712"},{"STENCIL_TK_STEPS":"5","STENCIL_TK_STRIP":"20512"}]'
