#!/bin/bash
# Fewer dispatches for small proofs (single-dispatch scans / Ruffini, k_sort_small, the
# k_bitsum2 fold): every GPU test, then A/B against libplk-prev.so at 2^12 / 2^14 / 2^16,
# interleaved twice.
set -uo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/.."
O=gpurun_out/r03disp
rm -rf $O; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests/ -x -q --timeout 300 --timeout-method thread -m gpu > $O/pytest.log 2>&1 || { echo PYTEST_FAILED; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
summ='import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,3), "M/s", round(d["ms_per_step"],3), "ms/step")'
for rep in 1 2; do
  for k in 12 14 16 20; do
    for lib in new prev; do
      l=""; [ $lib = prev ] && l=$PWD/dusk-plonk_amd/libplk-prev.so
      st=16; [ $k = 20 ] && st=6
      PLK_LIB=$l timeout -k 10 300 python3 bench.py --no-cpu-baseline --log-n $k --steps $st --warmup 3 > $O/b${k}_${lib}_$rep.log 2>&1 || { echo BENCH_FAILED; tail -20 $O/b${k}_${lib}_$rep.log; exit 1; }
      echo -n "2^$k $lib #$rep: "; grep '"metric"' $O/b${k}_${lib}_$rep.log | python3 -c "$summ"
    done
  done
done
for k in 12 16; do
  for lib in new prev; do
    l=""; [ $lib = prev ] && l=$PWD/dusk-plonk_amd/libplk-prev.so
    PLK_LIB=$l timeout -k 10 300 python3 bench.py --mode msm --no-cpu-baseline --log-n $k --steps 20 --warmup 3 > $O/m${k}_$lib.log 2>&1 || { echo MSM_FAILED; tail -20 $O/m${k}_$lib.log; exit 1; }
    echo -n "lone msm 2^$k $lib: "; grep '"metric"' $O/m${k}_$lib.log | python3 -c "$summ"
  done
done
echo done
