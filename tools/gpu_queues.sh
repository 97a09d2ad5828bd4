# lanes x HIP hardware queues sweep (GPU_MAX_HW_QUEUES, box default 4)
set -o pipefail
if [ $# -gt 0 ]; then CFGLIST=("$@"); else CFGLIST=("4 3" "8 3" "8 4" "8 6"); fi
export TMPDIR=/tmp
summ='import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,3), "M/s", round(d["ms_per_step"],2), "ms/step")'
for k in 16 20; do
  st=$([ $k = 16 ] && echo "--steps 30 --warmup 3" || echo "--steps 5 --warmup 2")
  for cfg in "${CFGLIST[@]}"; do
    read q l <<< "$cfg"
    GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python bench.py --no-cpu-baseline --log-n $k --lanes $l $st > gpurun_out/q_${k}_${q}_$l.log 2>&1 || { echo FAIL; tail -5 gpurun_out/q_${k}_${q}_$l.log; exit 1; }
    echo -n "2^$k queues $q lanes $l: "; grep '"metric"' gpurun_out/q_${k}_${q}_$l.log | python3 -c "$summ"
  done
done
