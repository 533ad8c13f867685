#!/bin/bash
# round 3, call ar: final tree with the box file's scheduler option -- whole GPU suite, smoke, C5 bench, C5 rocprof+PMC
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 1000 python3 -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests \
  > gpurun_out/r03ar_gpu_tests.txt 2>&1 || exit 1
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03ar_smoke.log 2>&1 &&
timeout -k 10 300 python3 bench.py --config C5 --steps 32 --warmup 4 --no-cpu-baseline > gpurun_out/r03ar_bench_c5.json 2> gpurun_out/r03ar_bench.err || exit 1
bash $R/profiles/collect.sh r03z8_c5 --config C5 --steps 8 --warmup 0 --no-cpu-baseline > $R/gpurun_out/r03z8_c5_collect.log 2>&1
