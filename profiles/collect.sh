#!/bin/bash
# Collect the rocprofv3 evidence for bench.py on one MI355X (run under gpurun).
# Kernel trace + stats, then FETCH_SIZE and WRITE_SIZE in separate --pmc passes
# (TCC slot limits; never combined with sys/runtime traces).
#   usage: profiles/collect.sh <tag> [bench args...]
set -u
TAG=${1:-run}; shift || true
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
ARGS=("$@")
[ ${#ARGS[@]} -eq 0 ] && ARGS=(--steps 100 --warmup 5 --no-cpu-baseline)
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 "$ROOT/bench.py" "${ARGS[@]}" > "$OUT/trace.log" 2>&1 || { echo "trace failed rc=$?"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- \
    python3 "$ROOT/bench.py" "${ARGS[@]}" > "$OUT/fetch.log" 2>&1 || { echo "fetch pass failed rc=$?"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- \
    python3 "$ROOT/bench.py" "${ARGS[@]}" > "$OUT/write.log" 2>&1 || { echo "write pass failed rc=$?"; exit 1; }
echo "profiles in $OUT"
