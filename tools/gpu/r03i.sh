#!/bin/bash
# round 3, call i: rank-mode slab job (C-ABI), box with the fast path compiled out, C5 / C2 benches
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_slab_job.py \
  > gpurun_out/r03i_slab_tests.txt 2>&1 &&
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "box" \
  > gpurun_out/r03i_box_parity.txt 2>&1 &&
timeout -k 10 300 python3 bench.py --config C5 --steps 32 --warmup 4 --no-cpu-baseline > gpurun_out/r03i_bench_c5.json 2> gpurun_out/r03i_bench_c5.err &&
timeout -k 10 300 python3 bench.py --no-cpu-baseline > gpurun_out/r03i_bench.json 2> gpurun_out/r03i_bench.err || exit 1
