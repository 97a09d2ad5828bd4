#!/bin/bash
# Two-pass NTT plans (PLK_NTT_MAX_LR = 9 / 10: radix up to 2^9 / 2^10, one or two columns per
# workgroup) against the default radix cap 2^8: NTT + prover parity with the cap raised, the
# standalone lines at 2^17 / 2^18 / 2^20, and the 2^16 / 2^20 proofs.
set -uo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/.."
O=gpurun_out/r03lr
rm -rf $O; mkdir -p $O
PLK_NTT_MAX_LR=10 timeout -k 10 600 python3 -u -m pytest tests/test_ntt_gpu.py tests/test_prover_oracle.py -x -q --timeout 300 --timeout-method thread -m gpu > $O/tests.log 2>&1 || { echo TESTS_FAILED; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
summ='import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],4), "ms/step", round(d["value"]/1e6,3), "M/s")'
for rep in 1 2; do
  for k in 17 18 20; do
    for lr in 8 9 10; do
      PLK_NTT_MAX_LR=$lr timeout -k 10 300 python3 bench.py --mode ntt --log-n $k --steps 20 --warmup 3 --no-cpu-baseline > $O/ntt_${lr}_${k}_$rep.log 2>&1 || { echo NTT_BENCH_FAILED $lr; tail -20 $O/ntt_${lr}_${k}_$rep.log; exit 1; }
      echo -n "ntt 2^$k max_lr $lr #$rep: "; grep '"metric"' $O/ntt_${lr}_${k}_$rep.log | python3 -c "$summ"
    done
  done
done
for k in 16 20; do
  st=16; [ $k = 20 ] && st=6
  for lr in 8 10; do
    PLK_NTT_MAX_LR=$lr timeout -k 10 300 python3 bench.py --no-cpu-baseline --log-n $k --steps $st --warmup 2 > $O/b${k}_$lr.log 2>&1 || { echo BENCH_FAILED; tail -20 $O/b${k}_$lr.log; exit 1; }
    echo -n "prove 2^$k max_lr $lr: "; grep '"metric"' $O/b${k}_$lr.log | python3 -c "$summ"
  done
done
echo done
