# strip-layout K-step kernel: parity, then interleaved A/B (tools/tune.py)
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_slab.py -k "tkstrip or temporalk or slab" -x -q --timeout 120 --timeout-method thread > gpurun_out/strip_tests.log 2>&1 || { tail -30 gpurun_out/strip_tests.log; exit 1; }
tail -2 gpurun_out/strip_tests.log
export TUNE_KERNEL=temporalk TUNE_ITERS=48
for DT in fp64 fp32; do
echo "== $DT 512"
TUNE_DTYPE=$DT timeout -k 10 300 python tools/tune.py 512 '[{},{"STENCIL_TK_BALANCE":"0"},{"STENCIL_TK_STEPS":"3"}]'
echo "== $DT 2048x2048x512"
TUNE_SHAPE=2048,2048,512 TUNE_ITERS=12 TUNE_DTYPE=$DT timeout -k 10 300 python tools/tune.py 512 '[{},{"STENCIL_TK_BALANCE":"0"}]'
done
