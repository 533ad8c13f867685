#!/bin/bash
# round 3, call u: x+ neighbour by ds_bpermute (BP) in the 7-point strip kernel -- parity, then interleaved A/B
# against the default shapes (fp64 512^3 and 2048^2 x 512 K = 4; fp32 4096^2 x 256 K = 5)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "tkstrip_chunking and (910708 or 920708 or 910508)" > gpurun_out/r03u_bp_parity.txt 2>&1 || exit 1
O=gpurun_out/r03u_ab_bp.txt
R=INIT=reference
timeout -k 10 200 python3 -u tools/ab.py --shape star --dtype fp64 --grid 512 512 512 --steps 4 --reps 7 \
  --variant $R --variant $R,STENCIL_TK_STRIP=910708 --variant $R,STENCIL_TK_STRIP=710708 \
  --variant $R,STENCIL_TK_STRIP=920708 > $O 2>&1 || exit 1
timeout -k 10 200 python3 -u tools/ab.py --shape star --dtype fp64 --grid 2048 2048 512 --steps 4 --reps 5 \
  --variant $R --variant $R,STENCIL_TK_STRIP=910708 >> $O 2>&1 || exit 1
timeout -k 10 200 python3 -u tools/ab.py --shape star --dtype fp32 --grid 4096 4096 256 --steps 5 --reps 5 \
  --variant $R --variant $R,STENCIL_TK_STRIP=910508 >> $O 2>&1 || exit 1
