# rocprofv3 kernel trace of the face-signalled interior-rank rehearsal (RCCL send/recv to self)
set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out/prof_r01j_sig
mkdir -p "$OUT" && cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 "$GRAFT_REPO_ROOT/bench.py" --exchange nccl-self --steps 200 --warmup 8 > "$OUT/trace.log" 2>&1 || { echo "sig trace failed"; tail -5 "$OUT/trace.log"; exit 1; }
grep metric "$OUT/trace.log" | head -1
