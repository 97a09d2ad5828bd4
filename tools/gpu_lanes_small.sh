# lanes sweep at small sizes (2^12, 2^14, 2^16): default bench lines with --lanes L
# (hardware queues 2L, at most 32)
set -o pipefail
export TMPDIR=/tmp
d=gpurun_out/lanes_small; rm -rf $d; mkdir -p $d
summ='import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,3), "M/s", round(d["ms_per_step"],2), "ms/step", d["config"]["proofs_per_step"], "proofs/step")'
for k in ${SIZES:-12 14 16}; do
  for L in ${LANES:-12 16 24 32}; do
    q=$((2 * L)); [ $q -gt 32 ] && q=32
    timeout -k 10 300 python bench.py --no-cpu-baseline --log-n $k --lanes $L --hw-queues $q --steps 20 --warmup 3 > $d/k${k}_l$L.log 2>&1 || { echo FAIL $k $L; tail -5 $d/k${k}_l$L.log; exit 1; }
    echo -n "2^$k lanes $L (queues $q): "; grep '"metric"' $d/k${k}_l$L.log | python3 -c "$summ"
  done
done
