#!/bin/bash
# round 3, call k: the 3D box redefined as ((P(z-1) + P(z)) + P(z+1)) - centre (8 operations per cell and
# stage, 236 -> 146 VGPRs at 3 x 8 K = 4): box parity against the new oracle, taller shapes A/B, C5 bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_gpu_slab.py tests/test_gpu_slab_job.py -k "box" > gpurun_out/r03k_box_tests.txt 2>&1 || exit 1
R=INIT=reference
timeout -k 10 300 python3 -u tools/ab.py --shape box --dtype fp64 --grid 2048 2048 256 --steps 4 --reps 5 \
  --variant $R --variant $R,STENCIL_BOXK_CFG=910408 --variant $R,STENCIL_BOXK_CFG=910508 \
  --variant $R,STENCIL_BOXK_CFG=910216 --variant $R,STENCIL_BOXK_CFG=910608,STEPS=3 \
  --variant $R,STENCIL_BOXK_CFG=910312,STEPS=3 \
  > gpurun_out/r03k_ab_box64.txt 2>&1 &&
timeout -k 10 300 python3 -u tools/ab.py --shape box --dtype fp32 --grid 2048 2048 256 --steps 3 --reps 5 \
  --variant $R --variant $R,STENCIL_BOXK_CFG=920608 --variant $R,STENCIL_BOXK_CFG=920308,STEPS=4 \
  --variant $R,STENCIL_BOXK_CFG=920408,STEPS=4 --variant $R,STENCIL_BOXK_CFG=920508,STEPS=4 \
  > gpurun_out/r03k_ab_box32.txt 2>&1 &&
timeout -k 10 300 python3 -u tools/ab.py --shape box --dtype fp64 --grid 512 512 512 --steps 4 --reps 5 \
  --variant $R --variant $R,STENCIL_BOXK_CFG=910408 --variant $R,STENCIL_BOXK_CFG=910508 \
  --variant $R,STENCIL_BOXK_CFG=910408,STEPS=3 --variant $R,STENCIL_BOXK_CFG=910608,STEPS=3 \
  > gpurun_out/r03k_ab_box64_512.txt 2>&1 &&
timeout -k 10 300 python3 bench.py --config C5 --steps 32 --warmup 4 --no-cpu-baseline > gpurun_out/r03k_bench_c5.json 2> gpurun_out/r03k_bench_c5.err
