#!/bin/bash
# round 3, call f: which path is wrong at 4096^2 x 1024 (rolling vs two-grid); PMC bytes of the HL strip
# variants; the shipping kernels built with and without SLP vectorisation, timed in separate processes
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 420 python3 -u tools/rolling_diag2.py > gpurun_out/r03f_rolling_diag2.txt 2>&1
cd /tmp
for v in 1 820908; do
  for c in FETCH_SIZE WRITE_SIZE; do
    STENCIL_TK_STRIP=$v timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $R/gpurun_out/r03f_pmc_strip$v/$c -o run -- \
      python3 $R/tools/ab.py --shape star --dtype fp64 --grid 512 512 512 --steps 4 --reps 1 --launches 3 \
      > $R/gpurun_out/r03f_pmc_strip${v}_$c.log 2>&1 || exit 1
  done
done
for c in FETCH_SIZE WRITE_SIZE; do
  STENCIL_TK_STRIP=830708 timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $R/gpurun_out/r03f_pmc_strip830708/$c -o run -- \
    python3 $R/tools/ab.py --shape star --dtype fp64 --grid 512 512 512 --steps 5 --reps 1 --launches 3 \
    > $R/gpurun_out/r03f_pmc_strip830708_$c.log 2>&1 || exit 1
done
cd $R
ab() {  # tag, args
  tag=$1; shift
  timeout -k 10 300 python3 -u tools/ab.py "$@" --reps 5 > gpurun_out/r03f_slp_$tag.txt 2>&1
}
for lib in slp noslp; do
  if [ $lib = noslp ]; then cp build/stage_noslp/libstencil_hip.so build/stage_noslp/libstencil_hip_debug.so stencil_amd/; fi
  ab ${lib}_box32 --shape box --dtype fp32 --grid 2048 2048 256 --steps 3 &&
  ab ${lib}_star32 --shape star --dtype fp32 --grid 4096 4096 256 --steps 5 &&
  ab ${lib}_star64 --shape star --dtype fp64 --grid 512 512 512 --steps 4 &&
  ab ${lib}_box64 --shape box --dtype fp64 --grid 2048 2048 256 --steps 4 || exit 1
done
