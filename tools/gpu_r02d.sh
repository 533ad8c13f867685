#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 120 ./tools/zmarch_pattern_bench > gpurun_out/pattern.log 2>&1; rc=$?; cat gpurun_out/pattern.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 bash tools/box_r02_ab.sh > gpurun_out/box_ab2.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/box_ab2.log; [ $rc -eq 0 ] || exit $rc
bash profiles/collect.sh r02d_c5 --config C5 --steps 10 --warmup 2 --no-cpu-baseline || exit 1
