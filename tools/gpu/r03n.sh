#!/bin/bash
# round 3, call n: box K = 5 (4 x 8 rows, 238 VGPRs fp64 / 250 fp32) against K = 4 (5 x 8), per sweep
set -o pipefail
mkdir -p gpurun_out
R=INIT=reference
timeout -k 10 300 python3 -u tools/ab.py --shape box --dtype fp64 --grid 2048 2048 256 --steps 4 --reps 5 \
  --variant $R --variant $R,STENCIL_BOXK_CFG=910408,STEPS=5 > gpurun_out/r03n_ab_box_k5.txt 2>&1 &&
timeout -k 10 300 python3 -u tools/ab.py --shape box --dtype fp64 --grid 512 512 512 --steps 4 --reps 5 \
  --variant $R --variant $R,STENCIL_BOXK_CFG=910408,STEPS=5 >> gpurun_out/r03n_ab_box_k5.txt 2>&1 &&
timeout -k 10 300 python3 -u tools/ab.py --shape box --dtype fp32 --grid 2048 2048 256 --steps 4 --reps 5 \
  --variant $R --variant $R,STENCIL_BOXK_CFG=920408,STEPS=5 >> gpurun_out/r03n_ab_box_k5.txt 2>&1 &&
timeout -k 10 300 python3 -u tools/ab.py --shape box --dtype fp64 --grid 2048 2048 256 --steps 4 --reps 5 \
  --variant INIT=random --variant INIT=random,STENCIL_BOXK_CFG=910408,STEPS=5 >> gpurun_out/r03n_ab_box_k5.txt 2>&1
