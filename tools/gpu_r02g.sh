#!/bin/bash
# Round-2 config table + multi-rank rehearsals after the box K=3 default and fuse_steps fix
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=r02g
timeout -k 10 500 python tools/bench_configs.py $TAG > gpurun_out/configs_$TAG.log 2>&1 || { echo "configs failed"; tail -20 gpurun_out/configs_$TAG.log; exit 1; }
grep -v amdgpu.ids gpurun_out/configs_$TAG.log
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 \
    bench.py --gpus 2 --exchange host --share-device --steps 40 --warmup 4 --no-cpu-baseline > gpurun_out/rehearse_$TAG.json 2> gpurun_out/rehearse_$TAG.err || { echo "rehearsal failed"; tail -20 gpurun_out/rehearse_$TAG.err; exit 1; }
grep metric gpurun_out/rehearse_$TAG.json
for EX in loopback nccl-self; do
  timeout -k 10 300 python bench.py --exchange $EX --steps 400 --warmup 20 > gpurun_out/bench_${EX}_$TAG.json 2> gpurun_out/bench_${EX}_$TAG.err || { echo "bench $EX failed"; tail -20 gpurun_out/bench_${EX}_$TAG.err; exit 1; }
  cat gpurun_out/bench_${EX}_$TAG.json
done
timeout -k 10 300 python bench.py --exchange loopback --config C5 --steps 30 --warmup 3 > gpurun_out/bench_c5_loopback_$TAG.json 2> gpurun_out/bench_c5_loopback_$TAG.err || { echo "bench C5 loopback failed"; tail -20 gpurun_out/bench_c5_loopback_$TAG.err; exit 1; }
cat gpurun_out/bench_c5_loopback_$TAG.json
