#!/bin/bash
# round 3, call r: fp32 box probe (8 x 8 rows, K = 3) through debug-library variants that differ only in
# how the SLP-vectorised probe object was compiled (tools/slp_bisect.sh)
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/r03r_slp_bisect.txt
timeout -k 10 120 python3 -u tools/slp_bisect.py build/slp/libdbg_base.so 3 950808 960808 > $O 2>&1 || exit 1
for v in b17204 b17205 dppoff; do
  timeout -k 10 120 python3 -u tools/slp_bisect.py build/slp/libdbg_$v.so 3 950808 >> $O 2>&1 || exit 1
done
