#!/bin/bash
# Round 2: full GPU suite after the box rewrite and the C++ slab jobs; benches of C2, C5, NS; box A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -15 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err || { echo "bench C2 rc=$?"; exit 1; }
cat gpurun_out/bench_c2.json
timeout -k 10 300 python -u bench.py --config C5 --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err || { echo "bench C5 rc=$?"; exit 1; }
cat gpurun_out/bench_c5.json
timeout -k 10 400 python -u bench.py --config NS --steps 40 --warmup 4 --no-cpu-baseline > gpurun_out/bench_ns.json 2> gpurun_out/bench_ns.err || { echo "bench NS rc=$?"; exit 1; }
cat gpurun_out/bench_ns.json
