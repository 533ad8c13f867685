#!/bin/bash
# L2 <-> fabric pressure counters for the strip kernel and the copy kernel
# (tools/tune.py 512 runs both): credit stalls, outstanding-request levels,
# TCC busy / tag stalls.  One counter group per rocprofv3 pass.
set -u
TAG=${1:-fabric}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/pmc_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
export TUNE_ITERS=${TUNE_ITERS:-12}
i=0
for P in "TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum GRBM_GUI_ACTIVE" \
         "TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" \
         "TCC_BUSY_sum TCC_CYCLE_sum TCC_TAG_STALL_sum TCC_EA0_WRREQ_STALL_sum" \
         "TCC_EA0_WRREQ_LEVEL_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_DRAM_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d "$OUT/p$i" -o run -- \
      python3 "$ROOT/tools/tune.py" 512 '[{}]' > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed rc=$?"; tail -5 "$OUT/p$i.log"; exit 1; }
done
echo "ok $OUT"
