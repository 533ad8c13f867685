#!/bin/bash
# round 4, call a: the launch-duration ramp (tools/ramp_probe.py under a kernel trace) + the driver's bench command
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/r04a
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r04a/ramp -o run -- \
  python3 $R/tools/ramp_probe.py > $R/gpurun_out/r04a/ramp.log 2>&1 || exit 1
cd $R
timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r04a/bench_driver.json 2> gpurun_out/r04a/bench_driver.err || exit 1
timeout -k 10 200 python3 bench.py --steps 1000 --warmup 20 --no-cpu-baseline > gpurun_out/r04a/bench_1000.json 2>> gpurun_out/r04a/bench_driver.err
