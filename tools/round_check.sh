#!/bin/bash
# One GPU call: full GPU test suite, bench (N=1), every BASELINE config on one
# GPU, and a 2-rank rehearsal of the multi-GPU bench path on the one GPU
# (host-staged gloo exchange).  usage: bash tools/round_check.sh <tag>
set -u
TAG=${1:-check}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1 || { echo "GPU tests failed"; tail -30 gpurun_out/gpu_tests_$TAG.log; exit 1; }
tail -1 gpurun_out/gpu_tests_$TAG.log
timeout -k 10 240 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench failed"; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
timeout -k 10 400 python tools/bench_configs.py $TAG > gpurun_out/configs_$TAG.log 2>&1 || { echo "configs failed"; tail -20 gpurun_out/configs_$TAG.log; exit 1; }
grep -v amdgpu.ids gpurun_out/configs_$TAG.log
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 \
    bench.py --gpus 2 --exchange host --share-device --steps 40 --warmup 4 > gpurun_out/rehearse_$TAG.json 2> gpurun_out/rehearse_$TAG.err || { echo "rehearsal failed"; tail -20 gpurun_out/rehearse_$TAG.err; exit 1; }
grep metric gpurun_out/rehearse_$TAG.json
