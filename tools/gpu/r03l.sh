#!/bin/bash
# round 3, call l: the whole GPU suite with the new box order and K = 4 5 x 8 box defaults; K = 3 vs 4 on small
# planes; C5 / C2 benches
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python3 -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests \
  > gpurun_out/r03l_gpu_tests.txt 2>&1 || exit 1
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03l_smoke.log 2>&1 &&
timeout -k 10 300 python3 bench.py --config C5 --steps 32 --warmup 4 --no-cpu-baseline > gpurun_out/r03l_bench_c5.json 2> gpurun_out/r03l_bench_c5.err || exit 1
R=INIT=reference
for dt in fp64 fp32; do
  for n in 256 384 512; do
    timeout -k 10 200 python3 -u tools/ab.py --shape box --dtype $dt --grid $n $n $n --steps 4 --reps 5 \
      --variant $R --variant $R,STEPS=3 >> gpurun_out/r03l_ab_box_k3k4.txt 2>&1 || exit 1
  done
done
timeout -k 10 300 python3 bench.py --no-cpu-baseline > gpurun_out/r03l_bench.json 2> gpurun_out/r03l_bench.err
