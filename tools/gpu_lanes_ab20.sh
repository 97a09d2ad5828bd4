set -o pipefail
summ='import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,3), "M/s", round(d["ms_per_step"],2), "ms/step")'
for rep in 1 2; do for cfg in "3 4" "8 16" "6 12"; do read l q <<< "$cfg"
  timeout -k 10 300 python bench.py --no-cpu-baseline --lanes $l --hw-queues $q --steps 8 --warmup 2 > gpurun_out/l_$l.log 2>&1 || { echo FAIL; tail -5 gpurun_out/l_$l.log; exit 1; }
  echo -n "2^20 lanes $l queues $q #$rep: "; grep '"metric"' gpurun_out/l_$l.log | python3 -c "$summ"
done; done
