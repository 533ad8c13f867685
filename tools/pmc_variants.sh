#!/bin/bash
# PMC passes (one counter group per rocprofv3 run) over tools/tune.py for
# several kernel variants given as env assignments, e.g.
#   bash tools/pmc_variants.sh tag "STENCIL_TK_STRIP=0" "STENCIL_TK_STRIP=1"
# Writes gpurun_out/pmc_<tag>/<variant#>/p<pass>/...; tools/pmc_table.py summarises.
set -u
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/pmc_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
export TUNE_KERNEL=${TUNE_KERNEL:-temporalk} TUNE_ITERS=${TUNE_ITERS:-12}
v=0
for VAR in "$@"; do
  v=$((v+1))
  mkdir -p "$OUT/v$v"
  echo "$VAR" > "$OUT/v$v.env"
  i=0
  for P in "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT" \
           "TCC_HIT_sum TCC_MISS_sum SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"; do
    i=$((i+1))
    ( export $VAR; timeout -k 10 120 rocprofv3 --pmc $P --output-format csv -d "$OUT/v$v/p$i" -o run -- \
        python3 "$ROOT/tools/tune.py" 512 '[{}]' > "$OUT/v$v/p$i.log" 2>&1 ) || { echo "variant $v pass $i failed rc=$?"; tail -5 "$OUT/v$v/p$i.log"; exit 1; }
  done
done
echo "ok $OUT"
