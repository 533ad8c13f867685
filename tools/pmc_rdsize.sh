#!/bin/bash
# Read-request sizes at the L2 -> fabric interface (strip kernel and copy kernel, tools/tune.py 512)
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/pmc_rdsize
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
export TUNE_ITERS=${TUNE_ITERS:-12}
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_sum \
    --output-format csv -d "$OUT/p1" -o run -- python3 "$ROOT/tools/tune.py" 512 '[{}]' > "$OUT/p1.log" 2>&1 || { echo "failed"; tail -5 "$OUT/p1.log"; exit 1; }
echo ok
