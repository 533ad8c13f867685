#!/bin/bash
# round 3, call b: rolling grid (one resident grid) parity + C3 on one GPU; single-process slab bench rehearsal;
# the packed-schedule rework (lazy stream-ordered upload, kernel-keyed cache) and the debug-knob library
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu \
  tests/test_gpu_rolling.py tests/test_gpu_slab_job.py -k "rolling or c3 or bench_single or distinct" \
  > gpurun_out/r03b_tests.txt 2>&1 &&
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "schedule_choice or prepare_leaves or packed_schedule or benched_kernel or tkstrip_chunking" \
  > gpurun_out/r03b_tests2.txt 2>&1 &&
timeout -k 10 300 python3 bench.py --config C3 --steps 100 --warmup 5 --no-cpu-baseline > gpurun_out/r03b_bench_c3.json 2> gpurun_out/r03b_bench_c3.err &&
timeout -k 10 300 python3 bench.py --gpus 2 --share-device --exchange copy --steps 200 --warmup 10 > gpurun_out/r03b_bench_slabjob_share.json 2> gpurun_out/r03b_bench_slabjob_share.err
