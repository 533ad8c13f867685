set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "tile_resident or c1_1024" -x -q --timeout 120 --timeout-method thread > gpurun_out/tb2d_tests2.log 2>&1 || { tail -30 gpurun_out/tb2d_tests2.log; exit 1; }
tail -1 gpurun_out/tb2d_tests2.log
cd /tmp && export TMPDIR=/tmp
CONFIGS_CPU=0 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_c1 -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_configs.py c1prof C1 C1r > $GRAFT_REPO_ROOT/gpurun_out/c1prof.log 2>&1
grep -v amdgpu $GRAFT_REPO_ROOT/gpurun_out/c1prof.log | tail -3
cat $GRAFT_REPO_ROOT/gpurun_out/prof_c1/run_kernel_stats.csv | cut -c1-250
