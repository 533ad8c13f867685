#!/bin/bash
# round 3, call o: C3 and C4 at full size on one GPU (rolling grid) -- tests and bench lines; box K = 5 parity
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_rolling.py \
  tests/test_gpu_parity.py -k "full_size_on_one_gpu or box_strip_shapes" > gpurun_out/r03o_tests.txt 2>&1 &&
timeout -k 10 300 python3 bench.py --config C4 --steps 40 --warmup 4 --no-cpu-baseline > gpurun_out/r03o_bench_c4.json 2> gpurun_out/r03o_bench_c4.err &&
timeout -k 10 400 python3 bench.py --config C3 --steps 20 --warmup 0 --no-cpu-baseline > gpurun_out/r03o_bench_c3.json 2> gpurun_out/r03o_bench_c3.err
