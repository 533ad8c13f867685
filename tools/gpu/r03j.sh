#!/bin/bash
# round 3, call j: box sum order ((P(z-1) + P(z)) + P(z+1)) - centre (ORD = 1: 144 instead of 236 VGPRs at
# 3 x 8 K = 4, so 4 x 8 and 5 x 8 fit) against the default order, reference initial condition and random data
set -o pipefail
mkdir -p gpurun_out
R=INIT=reference
timeout -k 10 300 python3 -u tools/ab.py --shape box --dtype fp64 --grid 2048 2048 256 --steps 4 --reps 5 \
  --variant $R --variant $R,STENCIL_BOXK_CFG=4990308,NOCHECK=1 --variant $R,STENCIL_BOXK_CFG=4990408,NOCHECK=1 \
  --variant $R,STENCIL_BOXK_CFG=4990508,NOCHECK=1 --variant $R,STENCIL_BOXK_CFG=3990608,NOCHECK=1,STEPS=3 \
  --variant INIT=random --variant INIT=random,STENCIL_BOXK_CFG=4990508,NOCHECK=1 \
  > gpurun_out/r03j_ab_ord_box64.txt 2>&1 &&
timeout -k 10 300 python3 -u tools/ab.py --shape box --dtype fp32 --grid 2048 2048 256 --steps 3 --reps 5 \
  --variant $R --variant $R,STENCIL_BOXK_CFG=3980408,NOCHECK=1 --variant $R,STENCIL_BOXK_CFG=3980608,NOCHECK=1 \
  --variant $R,STENCIL_BOXK_CFG=4980408,NOCHECK=1,STEPS=4 --variant $R,STENCIL_BOXK_CFG=4980508,NOCHECK=1,STEPS=4 \
  > gpurun_out/r03j_ab_ord_box32.txt 2>&1 &&
timeout -k 10 300 python3 -u tools/ab.py --shape box --dtype fp64 --grid 512 512 512 --steps 4 --reps 5 \
  --variant $R --variant $R,STENCIL_BOXK_CFG=4990408,NOCHECK=1 --variant $R,STENCIL_BOXK_CFG=4990508,NOCHECK=1 \
  > gpurun_out/r03j_ab_ord_box64_512.txt 2>&1
