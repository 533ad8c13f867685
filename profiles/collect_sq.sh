#!/bin/bash
# SQ/LDS counter passes for one kernel configuration (run under gpurun).
#   usage: profiles/collect_sq.sh <tag> [tune.py args...]
#   PROG=bench.py profiles/collect_sq.sh <tag> [bench.py args...]   (any repo-relative python program)
set -u
TAG=${1:-sq}; shift || true
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/sq_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
ARGS=("$@")
PROG=${PROG:-tools/tune.py}
[ ${#ARGS[@]} -eq 0 ] && [ "$PROG" = tools/tune.py ] && ARGS=(512)
i=0
for P in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
         "SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT" \
         "TCC_HIT_sum TCC_MISS_sum SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" ; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $P --output-format csv -d "$OUT/p$i" -o run -- \
      python3 "$ROOT/$PROG" "${ARGS[@]}" > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed rc=$?"; tail -5 "$OUT/p$i.log"; exit 1; }
done
echo "ok $OUT"
