#!/bin/bash
# Final-tree evidence after the measured schedule choice: full GPU suite, smoke,
# rocprof + PMC of the default C2 bench and of C5, default bench line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=r02kk
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?; tail -2 gpurun_out/gpu_tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { cat gpurun_out/${TAG}_smoke.log; exit 1; }
bash profiles/collect.sh $TAG --steps 1000 --warmup 20 --no-cpu-baseline || exit 1
bash profiles/collect.sh ${TAG}_c5 --config C5 --steps 16 --warmup 4 --no-cpu-baseline || exit 1
timeout -k 10 300 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit 1
cat gpurun_out/${TAG}_bench.json
