#!/bin/bash
# round 3, call ai: final tree -- whole GPU suite, smoke, C2 bench, then rocprof + PMC of C2 and C3
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 1000 python3 -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests \
  > gpurun_out/r03ai_gpu_tests.txt 2>&1 || exit 1
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03ai_smoke.log 2>&1 &&
timeout -k 10 300 python3 bench.py > gpurun_out/r03ai_bench.json 2> gpurun_out/r03ai_bench.err || exit 1
bash $R/profiles/collect.sh r03z5 --steps 100 --warmup 5 --no-cpu-baseline > $R/gpurun_out/r03z5_collect.log 2>&1 &&
bash $R/profiles/collect.sh r03z5_c3 --config C3 --steps 10 --warmup 0 --no-cpu-baseline > $R/gpurun_out/r03z5_c3_collect.log 2>&1
