set -o pipefail
export TMPDIR=/tmp
summ='import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,3), "M/s", round(d["ms_per_step"],2), "ms/step")'
for k in 16 20; do for L in 2 3 4 5; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --log-n $k --lanes $L > gpurun_out/lanes_${k}_$L.log 2>&1 || { echo FAIL; tail -5 gpurun_out/lanes_${k}_$L.log; exit 1; }
  echo -n "2^$k lanes $L: "; grep '"metric"' gpurun_out/lanes_${k}_$L.log | python3 -c "$summ"
done; done
