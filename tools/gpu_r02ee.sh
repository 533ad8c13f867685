#!/bin/bash
# rocprof evidence for the current kernel sources (C2 default bench, C5), full GPU suite, default bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=r02ee
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?; tail -2 gpurun_out/gpu_tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
bash profiles/collect.sh $TAG --steps 1000 --warmup 20 --no-cpu-baseline || exit 1
bash profiles/collect.sh ${TAG}_c5 --config C5 --steps 16 --warmup 4 --no-cpu-baseline || exit 1
