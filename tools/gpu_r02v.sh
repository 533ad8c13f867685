#!/bin/bash
# Box K=4 default for fp64 large planes: full GPU suite, C5 bench (one GPU), C5 interior rank (loopback, SIG K=4)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=r02v
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
for X in "" "--exchange loopback"; do
  timeout -k 10 300 python -u bench.py --config C5 --steps 32 --warmup 4 --no-cpu-baseline $X > gpurun_out/bench_c5${X// /}_$TAG.json 2> gpurun_out/bench_c5_$TAG.err || { echo "C5 $X failed"; tail gpurun_out/bench_c5_$TAG.err; exit 1; }
  python - gpurun_out/bench_c5${X// /}_$TAG.json <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(d["config"]["parallelism"], d["value"], d["roofline"]["mean_launch_ms"], d["roofline"]["frac"], d["roofline"].get("copy_kernel_GBps"))
PY
done
