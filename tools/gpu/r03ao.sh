#!/bin/bash
# round 3, call ao: final tree with the 2D kernel file under gcn-max-ilp -- whole GPU suite, smoke, C1 timing
# through the product library, C2 bench
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 1000 python3 -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests \
  > gpurun_out/r03ao_gpu_tests.txt 2>&1 || exit 1
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03ao_smoke.log 2>&1 || exit 1
for dt in fp64 fp32; do
  timeout -k 10 120 python3 tools/time_lib.py stencil_amd/libstencil_hip.so star $dt 1024 1024 0 100 20 >> gpurun_out/r03ao_c1.txt 2>/dev/null || exit 1
done
timeout -k 10 300 python3 bench.py > gpurun_out/r03ao_bench.json 2> gpurun_out/r03ao_bench.err
