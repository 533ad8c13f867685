#!/bin/bash
# stencil_prepare on the GPU (test + bench with --warmup 0: the schedule trial stays outside the timed region) + CLI warm-up
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=r02mm
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "prepare or schedule_choice or benched_kernel or cli" > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -2 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --warmup 0 --no-cpu-baseline > gpurun_out/${TAG}_bench_w0.json 2> gpurun_out/${TAG}_bench_w0.err || exit 1
timeout -k 10 120 ./build/bin/stencil_main -s 512 -b 64 -i 100 -m HIP --dims 3 > gpurun_out/${TAG}_cli3d.log 2>&1 || exit 1
cat gpurun_out/${TAG}_bench_w0.json; cat gpurun_out/${TAG}_cli3d.log
