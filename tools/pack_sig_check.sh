# Packed schedule on face-signalled slab rounds: full GPU suite (signalled
# tests run with the table forced, STENCIL_TK_PACK=2), then the interior-rank
# rehearsals (RCCL to self, device-copy loopback) with and without packing.
set -e
mkdir -p gpurun_out
if [ "${SKIP_TESTS:-0}" != 1 ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_packsig.log 2>&1 || { tail -30 gpurun_out/gpu_tests_packsig.log; exit 1; }
tail -1 gpurun_out/gpu_tests_packsig.log
fi
for EX in nccl-self loopback; do
for P in 0 1; do
STENCIL_TK_PACK=$P timeout -k 10 240 python bench.py --exchange $EX --steps 400 --warmup 8 --no-cpu-baseline > gpurun_out/packsig_${EX}_$P.json 2> gpurun_out/packsig_${EX}_$P.err || { tail -20 gpurun_out/packsig_${EX}_$P.err; exit 1; }
python -c "import json,sys; d=json.loads([l for l in open('gpurun_out/packsig_${EX}_$P.json') if l.startswith('{')][-1]); print('$EX pack=$P', d['value'], d['roofline']['mean_launch_ms'], d['config']['rounds'])"
done
done
