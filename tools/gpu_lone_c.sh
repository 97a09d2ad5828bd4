#!/bin/bash
# Lone-MSM window sweep (bench.py --mode msm, PLK_MSM_C = the srs.hip choose_c override):
# which c a lone commit of 2^16 / 2^20 points wants, against the proof batches' choice.
# usage: bash tools/gpu_lone_c.sh "12 13 14 15 16 17" "15 16 17 18 20"
set -uo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/.."
d=gpurun_out/lonec; rm -rf $d; mkdir -p $d
summ='import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],4), "ms;", round(d["value"]/1e6,2), "M points/s")'
for rep in 1 2; do
  for c in ${1:-13 14 15 16 17}; do
    PLK_MSM_C=$c timeout -k 10 240 python3 bench.py --mode msm --log-n 16 --steps 20 --warmup 3 --no-cpu-baseline > $d/m16_${c}_$rep.log 2>&1 || { echo BENCH_FAILED 16 $c; tail -20 $d/m16_${c}_$rep.log; exit 1; }
    echo -n "2^16 c=$c #$rep: "; grep '"metric"' $d/m16_${c}_$rep.log | python3 -c "$summ"
  done
  for c in ${2:-16 17 18 20}; do
    PLK_MSM_C=$c timeout -k 10 240 python3 bench.py --mode msm --log-n 20 --steps 10 --warmup 2 --no-cpu-baseline > $d/m20_${c}_$rep.log 2>&1 || { echo BENCH_FAILED 20 $c; tail -20 $d/m20_${c}_$rep.log; exit 1; }
    echo -n "2^20 c=$c #$rep: "; grep '"metric"' $d/m20_${c}_$rep.log | python3 -c "$summ"
  done
done
echo done
