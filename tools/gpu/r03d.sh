#!/bin/bash
# round 3, call d: LDS-history (HL) strip variants and XCD-patch box order, A/B in one process each,
# parity of the new shapes, and FETCH/WRITE of the box order variants
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "xcd_patch or (tkstrip_chunking and (810808 or 810708 or 810608 or 820908 or 830708 or 820608))" > gpurun_out/r03d_hl_parity.txt 2>&1 &&
timeout -k 10 300 python3 -u tools/ab.py --shape star --dtype fp64 --grid 512 512 512 --steps 4 --reps 7 \
  --variant STENCIL_TK_STRIP=1 --variant STENCIL_TK_STRIP=810708 --variant STENCIL_TK_STRIP=810808 --variant STENCIL_TK_STRIP=820908 \
  --variant STENCIL_TK_STRIP=1,STEPS=5 --variant STENCIL_TK_STRIP=810608,STEPS=5 --variant STENCIL_TK_STRIP=810708,STEPS=5 \
  --variant STENCIL_TK_STRIP=830708,STEPS=5 \
  > gpurun_out/r03d_ab_hl_512.txt 2>&1 &&
timeout -k 10 300 python3 -u tools/ab.py --shape star --dtype fp64 --grid 2048 2048 512 --steps 4 --reps 5 \
  --variant STENCIL_TK_STRIP=1 --variant STENCIL_TK_STRIP=810808 --variant STENCIL_TK_STRIP=820908 \
  --variant STENCIL_TK_STRIP=1,STEPS=5 --variant STENCIL_TK_STRIP=810608,STEPS=5 --variant STENCIL_TK_STRIP=830708,STEPS=5 \
  > gpurun_out/r03d_ab_hl_2048.txt 2>&1 &&
timeout -k 10 300 python3 -u tools/ab.py --shape star --dtype fp32 --grid 4096 4096 256 --steps 5 --reps 5 \
  --variant STENCIL_TK_STRIP=1 --variant STENCIL_TK_STRIP=820608 --variant STENCIL_TK_STRIP=830708 \
  > gpurun_out/r03d_ab_hl_fp32_4096.txt 2>&1 &&
timeout -k 10 300 python3 -u tools/ab.py --shape star --dtype fp64 --grid 512 512 512 --steps 4 --reps 5 \
  --variant STENCIL_TK_PACK=0 --variant STENCIL_TK_PACK=0,STENCIL_TK_XCD=2 --variant STENCIL_TK_PACK=0,STENCIL_TK_XCD=4 \
  --variant STENCIL_TK_PACK=1 > gpurun_out/r03d_ab_tk_xcd_512.txt 2>&1 &&
timeout -k 10 300 python3 -u tools/ab.py --shape star --dtype fp64 --grid 2048 2048 512 --steps 4 --reps 5 \
  --variant STENCIL_TK_XCD=0 --variant STENCIL_TK_XCD=2 --variant STENCIL_TK_XCD=4 --variant STENCIL_TK_XCD=8 \
  > gpurun_out/r03d_ab_tk_xcd_2048.txt 2>&1 &&
timeout -k 10 300 python3 -u tools/ab.py --shape box --dtype fp64 --grid 2048 2048 256 --steps 4 --reps 5 \
  --variant STENCIL_BOXK_XCD=0 --variant STENCIL_BOXK_XCD=2 --variant STENCIL_BOXK_XCD=4 --variant STENCIL_BOXK_XCD=8 \
  > gpurun_out/r03d_ab_box_xcd.txt 2>&1 &&
R=$GRAFT_REPO_ROOT; cd /tmp
for v in 0 4; do
  for c in FETCH_SIZE WRITE_SIZE; do
    STENCIL_BOXK_XCD=$v timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $R/gpurun_out/r03d_pmc_xcd$v/$c -o run -- \
      python3 $R/tools/ab.py --shape box --dtype fp64 --grid 2048 2048 256 --steps 4 --reps 1 --launches 2 \
      > $R/gpurun_out/r03d_pmc_xcd${v}_$c.log 2>&1 || exit 1
  done
done
cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 300 python3 -u tools/box_v1_diff.py fp32 3 950808 960808 950408 960408 > gpurun_out/r03d_box_v1_probe.txt 2>&1 &&
timeout -k 10 300 python3 -u tools/box_v1_diff.py fp32 1 950808 960808 >> gpurun_out/r03d_box_v1_probe.txt 2>&1 &&
timeout -k 10 300 python3 -u tools/box_v1_diff.py fp32 2 950808 960808 >> gpurun_out/r03d_box_v1_probe.txt 2>&1 &&
timeout -k 10 300 python3 -u tools/box_v1_diff.py fp32 4 950408 960408 >> gpurun_out/r03d_box_v1_probe.txt 2>&1
cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --exchange host --share-device --steps 40 --warmup 8 > gpurun_out/r03d_rehearse_2rank.json 2> gpurun_out/r03d_rehearse_2rank.err &&
timeout -k 10 300 python3 bench.py > gpurun_out/r03d_bench_default.json 2> gpurun_out/r03d_bench_default.err
