#!/bin/bash
# Proof-level A/B: the default bench line (2^20, 2^16; --no-cpu-baseline) for the default build
# and each variant library (PLK_LIB), interleaved twice.   usage: bash tools/gpu_ab_proof.sh <variant ...>
set -o pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/.."
d=gpurun_out/ab_proof; rm -rf $d; mkdir -p $d
summ='import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,3), "M/s", round(d["ms_per_step"],1), "ms/step")'
for rep in 1 2; do
  for k in 20 16; do
    for v in default "$@"; do
      if [ "$v" = default ]; then lib=""; else lib="$PWD/dusk-plonk_amd/libplk-$v.so"; fi
      PLK_LIB=$lib timeout -k 10 300 python3 bench.py --log-n $k --no-cpu-baseline > $d/p_${v}_${k}_$rep.log 2>&1 || { echo BENCH_FAILED $v $k; tail -20 $d/p_${v}_${k}_$rep.log; exit 1; }
      echo -n "2^$k $v #$rep: "; grep '"metric"' $d/p_${v}_${k}_$rep.log | python3 -c "$summ"
    done
  done
done
echo done
