#!/bin/bash
# round-2 tree after the box clean-up: full GPU suite, smoke, C5 rocprof (traffic table), default bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=r02z
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?; tail -2 gpurun_out/gpu_tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" 2>&1 | grep smoke || exit 1
bash profiles/collect.sh ${TAG}_c5 --config C5 --steps 16 --warmup 4 --no-cpu-baseline || exit 1
timeout -k 10 300 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench failed"; tail gpurun_out/bench_$TAG.err; exit 1; }
cut -c1-200 gpurun_out/bench_$TAG.json
