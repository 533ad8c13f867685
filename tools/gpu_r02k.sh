#!/bin/bash
# Round 2: box strip defaults -- box parity suites, C5 bench on one GPU, C5 interior-rank (loopback) per SIG shape
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=r02k
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_slab.py tests/test_gpu_slab_job.py -k "box or slab_job or multi_gpu" -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_box_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests_box_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --config C5 --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/bench_c5_$TAG.json 2> gpurun_out/bench_c5_$TAG.err || { echo "bench C5 failed"; tail gpurun_out/bench_c5_$TAG.err; exit 1; }
cat gpurun_out/bench_c5_$TAG.json
for C in 0 910408 910308; do
  STENCIL_BOXK_SIG_CFG=$C timeout -k 10 300 python -u bench.py --exchange loopback --config C5 --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/bench_c5_loopback_sig${C}_$TAG.json 2> gpurun_out/bench_c5_loopback_sig${C}_$TAG.err || { echo "bench C5 loopback $C failed"; tail gpurun_out/bench_c5_loopback_sig${C}_$TAG.err; exit 1; }
  echo "SIG_CFG=$C"; cat gpurun_out/bench_c5_loopback_sig${C}_$TAG.json
done
