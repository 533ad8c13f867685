#!/bin/bash
# After the box K threshold change: full GPU suite, NS proxy bench, C5 bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=r02bb
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?; tail -2 gpurun_out/gpu_tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --config NS --steps 40 --warmup 4 --no-cpu-baseline > gpurun_out/bench_ns_$TAG.json 2> gpurun_out/bench_ns_$TAG.err || { echo "NS failed"; tail gpurun_out/bench_ns_$TAG.err; exit 1; }
timeout -k 10 300 python -u bench.py --config C5 --steps 32 --warmup 4 --no-cpu-baseline > gpurun_out/bench_c5_$TAG.json 2> gpurun_out/bench_c5_$TAG.err || { echo "C5 failed"; tail gpurun_out/bench_c5_$TAG.err; exit 1; }
for f in ns c5; do python - gpurun_out/bench_${f}_$TAG.json <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r=d["roofline"]; print(d["config"]["workload"][:40], d["value"], r["frac"], r["mean_launch_ms"], r.get("traffic_GBps"), r.get("copy_kernel_GBps"))
PY
done
