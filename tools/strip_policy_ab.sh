# Store/load cache policy of the strip K-step kernel: nontemporal output
# stores (default) vs plain stores (cfg 94) vs nontemporal input loads
# (cfg 95).  Parity of both, then interleaved A/B (tools/tune.py).
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "tkstrip_chunking and (4-94 or 4-95)" -x -q --timeout 120 --timeout-method thread > gpurun_out/strip_policy_tests.log 2>&1 || { tail -30 gpurun_out/strip_policy_tests.log; exit 1; }
tail -1 gpurun_out/strip_policy_tests.log
export TUNE_KERNEL=temporalk TUNE_ITERS=60 STENCIL_TK_STEPS=4
echo "== fp64 512"
TUNE_DTYPE=fp64 timeout -k 10 300 python tools/tune.py 512 '[{},{"STENCIL_TK_STRIP":"94"},{"STENCIL_TK_STRIP":"95"}]'
echo "== fp64 2048x2048x512"
TUNE_SHAPE=2048,2048,512 TUNE_ITERS=20 TUNE_DTYPE=fp64 timeout -k 10 300 python tools/tune.py 512 '[{},{"STENCIL_TK_STRIP":"94"},{"STENCIL_TK_STRIP":"95"}]'
echo "== fp32 2048x2048x512 (K = 4)"
TUNE_SHAPE=2048,2048,512 TUNE_ITERS=20 TUNE_DTYPE=fp32 timeout -k 10 300 python tools/tune.py 512 '[{},{"STENCIL_TK_STRIP":"94"},{"STENCIL_TK_STRIP":"95"}]'
