#!/bin/bash
# round 3, call ac: NS (2048^3 fp64) through AUTO vs the default file's build forced (debug cfg 10708), alternating
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/r03ac_ns_route.txt
: > $O
for rep in 1 2; do
  echo "AUTO NS" >> $O
  timeout -k 10 300 python3 bench.py --config NS --steps 40 --warmup 4 --no-cpu-baseline >> $O 2>/dev/null || exit 1
  echo "STENCIL_TK_STRIP=10708 NS" >> $O
  STENCIL_TK_STRIP=10708 timeout -k 10 300 python3 bench.py --config NS --steps 40 --warmup 4 --no-cpu-baseline >> $O 2>/dev/null || exit 1
done
echo "verbose" >> $O
STENCIL_TK_VERBOSE=1 timeout -k 10 300 python3 bench.py --config NS --steps 8 --warmup 0 --no-cpu-baseline >> $O 2>&1 || exit 1
