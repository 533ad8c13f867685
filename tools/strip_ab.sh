# strip-layout K-step kernel: parity, then interleaved A/B (tools/tune.py)
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "tkstrip" -x -q --timeout 120 --timeout-method thread > gpurun_out/strip_tests.log 2>&1 || { tail -30 gpurun_out/strip_tests.log; exit 1; }
tail -2 gpurun_out/strip_tests.log
export TUNE_KERNEL=temporalk TUNE_ITERS=60
for DT in fp64 fp32; do
echo "== $DT 512"
TUNE_DTYPE=$DT timeout -k 10 300 python tools/tune.py 512 '[{},{"STENCIL_TK_STEPS":"5"},{"STENCIL_TK_STEPS":"5","STENCIL_TK_STRIP":"10608"},{"STENCIL_TK_STEPS":"5","STENCIL_TK_STRIP":"20608"}]'
echo "== $DT 2048x2048x512"
TUNE_SHAPE=2048,2048,512 TUNE_ITERS=20 TUNE_DTYPE=$DT timeout -k 10 300 python tools/tune.py 512 '[{},{"STENCIL_TK_STEPS":"5"}]'
done
