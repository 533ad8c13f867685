#!/bin/bash
# strip 7-point fast path (no saddr), box saddr: strip/box suites, default bench, fast off/on bench A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=r02q
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_slab.py tests/test_gpu_slab_job.py -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?; tail -2 gpurun_out/gpu_tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
for F in 1 0 1 0; do
  STENCIL_TK_FAST=$F timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_fast${F}_$TAG.json 2> gpurun_out/bench_fast${F}_$TAG.err || { echo "bench failed"; tail gpurun_out/bench_fast${F}_$TAG.err; exit 1; }
  python - $F gpurun_out/bench_fast${F}_$TAG.json <<'PY'
import json,sys
d=json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print("fast", sys.argv[1], "value", d["value"], "launch_ms", d["roofline"]["mean_launch_ms"], "frac", d["roofline"]["frac"], "copy", d["roofline"].get("copy_kernel_GBps"))
PY
done
