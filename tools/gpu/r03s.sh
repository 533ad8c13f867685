#!/bin/bash
# round 3, call s: the fp32 box probe (8 x 8 rows, K = 3, SLP build) of the PRE-round-3 box order (tree 53ccc07)
# through debug libraries whose probe object stops the optimiser at successive opt-bisect limits
# (tools/slp_bisect.sh); reference = the same library's no-SLP build of the same source (cfg 960808)
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/r03s_slp_bisect_old.txt
: > $O
for n in 999999 16214 16215 16233 16405 16491 16502 16503 16515 16600; do
  timeout -k 10 120 python3 -u tools/slp_bisect.py build/slp_old/libdbg_o$n.so 3 --ref-cfg 960808 950808 >> $O 2>&1 || exit 1
done
