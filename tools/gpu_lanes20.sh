#!/bin/bash
# 2^20 default bench at 12 / 14 / 16 prover lanes (--lanes; hardware queues 2 x lanes <= 32),
# interleaved twice.
set -o pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/.."
d=gpurun_out/lanes20; rm -rf $d; mkdir -p $d
summ='import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,3), "M/s", round(d["ms_per_step"],1), "ms/step", d["config"]["parallelism"])'
for rep in ${REPS:-1 2}; do
  for L in ${LANES:-12 14 16}; do
    timeout -k 10 300 python3 bench.py --lanes $L --steps ${STEPS:-5} --no-cpu-baseline > $d/l${L}_$rep.log 2>&1 || { echo BENCH_FAILED $L; tail -20 $d/l${L}_$rep.log; exit 1; }
    echo -n "2^20 lanes=$L #$rep: "; grep '"metric"' $d/l${L}_$rep.log | python3 -c "$summ"
  done
done
echo done
