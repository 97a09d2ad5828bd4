# constraints/s across circuit sizes 2^12..2^20 (default lanes / queues), one GPU
set -o pipefail
export TMPDIR=/tmp
summ='import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,3), "M/s", round(d["ms_per_step"],2), "ms/step", d["config"]["proofs_per_step"], "proofs/step")'
mkdir -p gpurun_out/sizes
for k in 12 14 16 18 20; do
  st=$([ $k -le 16 ] && echo "--steps 30 --warmup 3" || echo "--steps 5 --warmup 2")
  timeout -k 10 300 python bench.py --no-cpu-baseline --log-n $k $st > gpurun_out/sizes/k$k.log 2>&1 || { echo FAIL $k; tail -5 gpurun_out/sizes/k$k.log; exit 1; }
  echo -n "2^$k: "; grep '"metric"' gpurun_out/sizes/k$k.log | python3 -c "$summ"
done
for k in 16; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --log-n $k --lanes 16 --hw-queues 32 --steps 30 --warmup 3 > gpurun_out/sizes/k${k}_l16.log 2>&1 || { echo FAIL; exit 1; }
  echo -n "2^$k lanes 16: "; grep '"metric"' gpurun_out/sizes/k${k}_l16.log | python3 -c "$summ"
done
