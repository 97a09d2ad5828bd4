#!/bin/bash
# Persistent software-pipelined NTT passes (PLK_NTT_PF = grid size): parity with PF on, then
# the standalone 2^20 / 2^23 lines for PF off / 256 / 512 / 768, twice (box drift).
set -uo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/.."
O=gpurun_out/r03pf
rm -rf $O; mkdir -p $O
PLK_NTT_PF=512 timeout -k 10 600 python3 -u -m pytest tests/test_ntt_gpu.py -x -q --timeout 300 --timeout-method thread -m gpu > $O/tests.log 2>&1 || { echo TESTS_FAILED; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
summ='import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],4), "ms/step exact", d.get("bit_exact_vs_oracle"))'
for rep in 1 2; do
  for k in 20 23; do
    for pf in 0 256 512 768; do
      PLK_NTT_PF=$pf timeout -k 10 300 python3 bench.py --mode ntt --log-n $k --steps 20 --warmup 3 --no-cpu-baseline > $O/ntt_${pf}_${k}_$rep.log 2>&1 || { echo NTT_BENCH_FAILED $pf; tail -20 $O/ntt_${pf}_${k}_$rep.log; exit 1; }
      echo -n "2^$k pf $pf #$rep: "; grep '"metric"' $O/ntt_${pf}_${k}_$rep.log | python3 -c "$summ"
    done
  done
done
echo done
