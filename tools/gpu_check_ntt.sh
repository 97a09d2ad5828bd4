set -o pipefail
bash tools/gpu_check.sh || exit 1
d=gpurun_out/check
for k in 20 23; do
  timeout -k 10 300 python bench.py --mode ntt --log-n $k --steps 20 --warmup 3 --no-cpu-baseline > $d/ntt$k.log 2>&1 || { echo NTT_BENCH_FAILED; tail -20 $d/ntt$k.log; exit 1; }
  grep '"metric"' $d/ntt$k.log | cut -c1-200
done
