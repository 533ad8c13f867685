#!/bin/bash
# Full GPU suite on the strip-box defaults; C5 interior-rank with the strip SIG default; fp32 box interior rank
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=r02n
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --exchange loopback --config C5 --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/bench_c5_loopback_$TAG.json 2> gpurun_out/bench_c5_loopback_$TAG.err || { echo "C5 loopback failed"; tail gpurun_out/bench_c5_loopback_$TAG.err; exit 1; }
cat gpurun_out/bench_c5_loopback_$TAG.json | cut -c1-400
