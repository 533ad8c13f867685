#!/bin/bash
# Round-2 first GPU pass: race demonstration, GPU suite, default bench, rocprof of the bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/race_check.py > gpurun_out/race_check.log 2>&1 || { echo "race_check rc=$?"; exit 1; }
cat gpurun_out/race_check.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -5 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench rc=$?"; exit 1; }
cat gpurun_out/bench.json
bash profiles/collect.sh r02a --steps 1000 --warmup 20 --no-cpu-baseline || exit 1
