set -o pipefail
mkdir -p gpurun_out
for ex in loopback nccl-self; do
  for sg in "" "--face-signal" "--no-signal"; do
    timeout -k 10 150 python bench.py --exchange $ex $sg --steps 600 --warmup 30 > gpurun_out/sig_${ex}${sg}.json 2> gpurun_out/sig_${ex}${sg}.err || exit 1
    echo "$ex $sg"; cat gpurun_out/sig_${ex}${sg}.json | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['config']['rounds'], d['roofline']['mean_launch_ms'], d['roofline']['frac'])"
  done
done
