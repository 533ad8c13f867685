# STENCIL_TK_PACK: parity (small shapes through the tkstrip tests, full
# sizes through tools/pack_check.py), then interleaved A/B (tools/tune.py).
set -e
mkdir -p gpurun_out
STENCIL_TK_PACK=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "tkstrip_chunking and -0-" -x -q --timeout 120 --timeout-method thread > gpurun_out/pack_tests.log 2>&1 || { tail -30 gpurun_out/pack_tests.log; exit 1; }
tail -1 gpurun_out/pack_tests.log
timeout -k 10 200 python tools/pack_check.py
export TUNE_KERNEL=temporalk TUNE_ITERS=60
echo "== fp64 512"
TUNE_DTYPE=fp64 timeout -k 10 300 python tools/tune.py 512 '[{},{"STENCIL_TK_PACK":"1"}]'
echo "== fp64 2048x2048x512"
TUNE_SHAPE=2048,2048,512 TUNE_ITERS=20 TUNE_DTYPE=fp64 timeout -k 10 300 python tools/tune.py 512 '[{},{"STENCIL_TK_PACK":"1"}]'
echo "== fp32 512"
TUNE_DTYPE=fp32 timeout -k 10 300 python tools/tune.py 512 '[{},{"STENCIL_TK_PACK":"1"}]'
