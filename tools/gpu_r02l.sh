#!/bin/bash
# C5 on one GPU: bench per box shape (the interleaved 3x8, strip 2x16, strip 4x8, strip 3x8) and tune.py beside it
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=r02l
for C in 10308 910216 910408 910308 0; do
  STENCIL_BOXK_CFG=$C timeout -k 10 300 python -u bench.py --config C5 --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/bench_c5_cfg${C}_$TAG.json 2> gpurun_out/bench_c5_cfg${C}_$TAG.err || { echo "bench C5 $C failed"; tail gpurun_out/bench_c5_cfg${C}_$TAG.err; exit 1; }
  python - "$C" gpurun_out/bench_c5_cfg${C}_$TAG.json <<'PY'
import json,sys
d=json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print("cfg", sys.argv[1], "value", d["value"], "mean_launch_ms", d["roofline"]["mean_launch_ms"], "copy", d["roofline"].get("copy_kernel_GBps"))
PY
done
export TUNE_STENCIL=box TUNE_ITERS=6
TUNE_DTYPE=fp64 TUNE_SWEEPK=3 TUNE_SHAPE=2048,2048,2048 timeout -k 10 300 python tools/tune.py 512 \
    '[{"STENCIL_BOXK_CFG":"10308"},{"STENCIL_BOXK_CFG":"910216"},{"STENCIL_BOXK_CFG":"910408"},{"STENCIL_BOXK_CFG":"910308"}]' || exit 1
