#!/bin/bash
# round 3, call g: the fill fix (> 2^32 elements) -- rolling tests incl. C3 at full size, diag 2, C3 bench on one GPU
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/test_gpu_rolling.py \
  > gpurun_out/r03g_rolling_tests.txt 2>&1
timeout -k 10 420 python3 -u tools/rolling_diag2.py > gpurun_out/r03g_rolling_diag2.txt 2>&1 &&
timeout -k 10 400 python3 bench.py --config C3 --steps 200 --warmup 5 --no-cpu-baseline > gpurun_out/r03g_bench_c3.json 2> gpurun_out/r03g_bench_c3.err
