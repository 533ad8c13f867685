#!/bin/bash
# round-2 final tree: smoke, default bench, rocprof of C5 (box K=4) for the traffic table, config table
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=r02w
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { echo "smoke failed"; cat gpurun_out/smoke_$TAG.log; exit 1; }
grep smoke gpurun_out/smoke_$TAG.log
bash profiles/collect.sh ${TAG}_c5 --config C5 --steps 16 --warmup 4 --no-cpu-baseline || exit 1
timeout -k 10 500 python tools/bench_configs.py $TAG > gpurun_out/configs_$TAG.log 2>&1 || { echo "configs failed"; tail -20 gpurun_out/configs_$TAG.log; exit 1; }
grep -v amdgpu.ids gpurun_out/configs_$TAG.log | tail -12
timeout -k 10 300 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench failed"; tail gpurun_out/bench_$TAG.err; exit 1; }
cut -c1-200 gpurun_out/bench_$TAG.json
