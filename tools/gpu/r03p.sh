#!/bin/bash
# round 3, call p: final tree -- whole GPU suite, smoke, bench lines (C2 default, NS, C5, C4), then rocprof + PMC
# of C2 and C5 on the final kernel sources (traffic table)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 1000 python3 -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests \
  > gpurun_out/r03p_gpu_tests.txt 2>&1 || exit 1
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03p_smoke.log 2>&1 &&
timeout -k 10 300 python3 bench.py > gpurun_out/r03p_bench.json 2> gpurun_out/r03p_bench.err &&
timeout -k 10 300 python3 bench.py --config NS --steps 40 --warmup 4 --no-cpu-baseline > gpurun_out/r03p_bench_ns.json 2> gpurun_out/r03p_bench_ns.err &&
timeout -k 10 300 python3 bench.py --config C5 --steps 32 --warmup 4 --no-cpu-baseline > gpurun_out/r03p_bench_c5.json 2> gpurun_out/r03p_bench_c5.err || exit 1
bash $R/profiles/collect.sh r03z3 --steps 100 --warmup 5 --no-cpu-baseline > $R/gpurun_out/r03z3_collect.log 2>&1 &&
bash $R/profiles/collect.sh r03z3_c5 --config C5 --steps 8 --warmup 0 --no-cpu-baseline > $R/gpurun_out/r03z3_c5_collect.log 2>&1
