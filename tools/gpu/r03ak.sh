#!/bin/bash
# round 3, call ak: final tree -- whole GPU suite, smoke, bench lines (C2 default, NS, C3, C5, interior-rank rehearsal)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 1000 python3 -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests \
  > gpurun_out/r03ak_gpu_tests.txt 2>&1 || exit 1
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03ak_smoke.log 2>&1 &&
timeout -k 10 300 python3 bench.py > gpurun_out/r03ak_bench.json 2> gpurun_out/r03ak_bench.err &&
timeout -k 10 300 python3 bench.py --config NS --steps 40 --warmup 4 --no-cpu-baseline > gpurun_out/r03ak_bench_ns.json 2>> gpurun_out/r03ak_bench.err &&
timeout -k 10 300 python3 bench.py --config C3 --steps 20 --warmup 0 --no-cpu-baseline > gpurun_out/r03ak_bench_c3.json 2>> gpurun_out/r03ak_bench.err &&
timeout -k 10 300 python3 bench.py --config C5 --steps 32 --warmup 4 --no-cpu-baseline > gpurun_out/r03ak_bench_c5.json 2>> gpurun_out/r03ak_bench.err &&
timeout -k 10 300 python3 bench.py --exchange loopback --steps 400 --warmup 20 --no-cpu-baseline > gpurun_out/r03ak_bench_loopback.json 2>> gpurun_out/r03ak_bench.err
