#!/bin/bash
# round 3, call h: the whole GPU suite on the current tree, smoke, and the bench lines (C2 default, NS, C5, C3)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python3 -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests \
  > gpurun_out/r03h_gpu_tests.txt 2>&1 || exit 1
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03h_smoke.log 2>&1 &&
timeout -k 10 300 python3 bench.py > gpurun_out/r03h_bench.json 2> gpurun_out/r03h_bench.err &&
timeout -k 10 300 python3 bench.py --config NS --steps 40 --warmup 4 --no-cpu-baseline > gpurun_out/r03h_bench_ns.json 2> gpurun_out/r03h_bench_ns.err &&
timeout -k 10 300 python3 bench.py --config C5 --steps 32 --warmup 4 --no-cpu-baseline > gpurun_out/r03h_bench_c5.json 2> gpurun_out/r03h_bench_c5.err
# box shapes with the interior fast path and no SLP (4 x 8 at K = 4: 4 VGPRs spilled; fp32 3 x 8 K = 4 fits now)
timeout -k 10 300 python3 -u tools/ab.py --shape box --dtype fp64 --grid 2048 2048 256 --steps 4 --reps 5 \
  --variant STENCIL_BOXK_FAST=0 --variant STENCIL_BOXK_FAST=1 --variant STENCIL_BOXK_CFG=910408 \
  > gpurun_out/r03h_ab_box64_k4.txt 2>&1 &&
timeout -k 10 300 python3 -u tools/ab.py --shape box --dtype fp64 --grid 2048 2048 256 --steps 3 --reps 5 \
  --variant STENCIL_BOXK_CFG=0 --variant STENCIL_BOXK_CFG=910312 --variant STENCIL_BOXK_CFG=910408 \
  > gpurun_out/r03h_ab_box64_k3.txt 2>&1 &&
timeout -k 10 300 python3 -u tools/ab.py --shape box --dtype fp32 --grid 2048 2048 256 --steps 3 --reps 5 \
  --variant STENCIL_BOXK_FAST=0 --variant STENCIL_BOXK_FAST=1 --variant STENCIL_BOXK_CFG=920308,STEPS=4 --variant STENCIL_BOXK_CFG=920408,STEPS=4 \
  > gpurun_out/r03h_ab_box32.txt 2>&1
