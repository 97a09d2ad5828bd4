set -o pipefail
mkdir -p gpurun_out/lanes
for L in 4; do
  timeout -k 10 600 python bench.py --no-cpu-baseline --lanes $L > gpurun_out/lanes/b20_$L.log 2>&1 || { echo B20_FAILED $L; tail -30 gpurun_out/lanes/b20_$L.log; exit 1; }
  grep metric gpurun_out/lanes/b20_$L.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('n20 lanes', $L, round(d['value']/1e6,3), 'M c/s', round(d['ms_per_step'],2))"
done
for L in 4 6 8; do
  timeout -k 10 600 python bench.py --no-cpu-baseline --lanes $L --log-n 16 --steps 20 --warmup 3 > gpurun_out/lanes/b16_$L.log 2>&1 || { echo B16_FAILED $L; tail -30 gpurun_out/lanes/b16_$L.log; exit 1; }
  grep metric gpurun_out/lanes/b16_$L.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('n16 lanes', $L, round(d['value']/1e6,3), 'M c/s', round(d['ms_per_step'],2))"
done
