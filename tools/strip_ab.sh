# strip-layout K-step kernel: parity, then interleaved A/B against the default (tools/tune.py)
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "tkstrip or temporalk" -x -q --timeout 120 --timeout-method thread > gpurun_out/strip_tests.log 2>&1 || { tail -30 gpurun_out/strip_tests.log; exit 1; }
tail -2 gpurun_out/strip_tests.log
export TUNE_KERNEL=temporalk TUNE_ITERS=48
echo "== fp64 512"
TUNE_DTYPE=fp64 timeout -k 10 300 python tools/tune.py 512 '[{},{"STENCIL_TK_STRIP":"1"},{"STENCIL_TK_STRIP":"10708","STENCIL_TK_STEPS":"4"},{"STENCIL_TK_STRIP":"10608","STENCIL_TK_STEPS":"4"},{"STENCIL_TK_STRIP":"10708","STENCIL_TK_STEPS":"4","STENCIL_TK_REMAP":"1"}]'
echo "== fp64 2048x2048x512"
TUNE_SHAPE=2048,2048,512 TUNE_ITERS=12 TUNE_DTYPE=fp64 timeout -k 10 300 python tools/tune.py 512 '[{},{"STENCIL_TK_STRIP":"1"},{"STENCIL_TK_STRIP":"10708","STENCIL_TK_STEPS":"4"}]'
echo "== fp32 512"
TUNE_DTYPE=fp32 timeout -k 10 300 python tools/tune.py 512 '[{},{"STENCIL_TK_STRIP":"1"},{"STENCIL_TK_STRIP":"20708","STENCIL_TK_STEPS":"4"}]'
