#!/bin/bash
# final tree: full GPU suite, smoke, config table, NS and C5 bench lines, interior-rank
# (loopback, face-signalled) line, 2-rank shared-GPU rehearsal with the bitwise check,
# rocprof + PMC of the default C2 bench, default bench line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=r02oo
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?; tail -2 gpurun_out/gpu_tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { cat gpurun_out/smoke_$TAG.log; exit 1; }
timeout -k 10 600 python tools/bench_configs.py $TAG > gpurun_out/configs_$TAG.log 2>&1 || { tail -20 gpurun_out/configs_$TAG.log; exit 1; }
timeout -k 10 300 python -u bench.py --config NS --steps 40 --warmup 4 --no-cpu-baseline > gpurun_out/bench_ns_$TAG.json 2> gpurun_out/bench_ns_$TAG.err || exit 1
timeout -k 10 300 python -u bench.py --config C5 --steps 32 --warmup 4 --no-cpu-baseline > gpurun_out/bench_c5_$TAG.json 2> gpurun_out/bench_c5_$TAG.err || exit 1
timeout -k 10 300 python -u bench.py --exchange loopback --no-cpu-baseline > gpurun_out/bench_loopback_$TAG.json 2> gpurun_out/bench_loopback_$TAG.err || exit 1
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29532 \
    bench.py --gpus 2 --exchange host --share-device --steps 40 --warmup 4 --no-cpu-baseline > gpurun_out/rehearse_2_$TAG.json 2> gpurun_out/rehearse_2_$TAG.err || exit 1
bash profiles/collect.sh $TAG --steps 1000 --warmup 20 --no-cpu-baseline || exit 1
timeout -k 10 300 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit 1
for f in bench_ns bench_c5 bench_loopback rehearse_2 bench; do cut -c1-160 gpurun_out/${f}_$TAG.json; done
