#!/bin/bash
# bench N>1 path rehearsed on one GPU (2 and 3 ranks sharing it, host-staged gloo halos) with the bitwise global-grid check
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for N in 2 3; do
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 --master-port 2953$N \
      bench.py --gpus $N --exchange host --share-device --steps 40 --warmup 4 --no-cpu-baseline > gpurun_out/rehearse_check_$N.json 2> gpurun_out/rehearse_check_$N.err || { echo "rehearsal $N failed"; tail -20 gpurun_out/rehearse_check_$N.err; exit 1; }
  python - gpurun_out/rehearse_check_$N.json <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(d["n_gpus"], d["value"], d["config"]["rounds"], json.dumps(d.get("multi_gpu_check")))
PY
done
