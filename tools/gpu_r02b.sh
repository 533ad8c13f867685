#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "box or golden or slab" --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_box.log 2>&1
rc=$?; tail -5 gpurun_out/gpu_tests_box.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 bash tools/box_r02_ab.sh > gpurun_out/box_ab.log 2>&1; rc=$?; cat gpurun_out/box_ab.log; exit $rc
