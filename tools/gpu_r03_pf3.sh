#!/bin/bash
# PF variant at 3 waves/SIMD (libplk-pf3.so, -DPLK_NTT_PF_MINW=3) against PF off.
set -uo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/.."
O=gpurun_out/r03pf3
rm -rf $O; mkdir -p $O
summ='import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],4), "ms/step")'
for rep in 1 2; do
  for k in 20 23; do
    for cfg in "0 " "768 $PWD/dusk-plonk_amd/libplk-pf3.so" "1024 $PWD/dusk-plonk_amd/libplk-pf3.so"; do
      set -- $cfg; pf=$1; lib=${2:-}
      PLK_LIB=$lib PLK_NTT_PF=$pf timeout -k 10 300 python3 bench.py --mode ntt --log-n $k --steps 20 --warmup 3 --no-cpu-baseline > $O/ntt_${pf}_${k}_$rep.log 2>&1 || { echo NTT_BENCH_FAILED $pf; tail -20 $O/ntt_${pf}_${k}_$rep.log; exit 1; }
      echo -n "2^$k pf $pf #$rep: "; grep '"metric"' $O/ntt_${pf}_${k}_$rep.log | python3 -c "$summ"
    done
  done
done
echo done
