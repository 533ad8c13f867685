#!/bin/bash
# rocprof evidence of the current default bench (C2) and of the C5 bench on one GPU (box strip)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash profiles/collect.sh r02t --steps 1000 --warmup 20 --no-cpu-baseline || exit 1
bash profiles/collect.sh r02t_c5 --config C5 --steps 12 --warmup 3 --no-cpu-baseline || exit 1
timeout -k 10 300 python -u bench.py > gpurun_out/bench_r02t.json 2> gpurun_out/bench_r02t.err || { echo "bench failed"; tail gpurun_out/bench_r02t.err; exit 1; }
cut -c1-300 gpurun_out/bench_r02t.json
