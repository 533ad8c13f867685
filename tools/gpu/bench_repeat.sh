set -o pipefail
O=gpurun_out/r05af; mkdir -p $O
for i in 1 2 3 4 5; do
  timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_driver_$i.json 2>> $O/bench.err || exit 1
done
