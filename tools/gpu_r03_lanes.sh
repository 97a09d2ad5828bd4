#!/bin/bash
# Lane-count sweep on the current code (2^20 and 2^16), default hardware queues (2 per lane).
set -uo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/.."
O=gpurun_out/r03lanes
rm -rf $O; mkdir -p $O
summ='import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,3), "M", round(d["ms_per_step"],2), "ms/step")'
for L in 6 8 10 12; do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 6 --warmup 2 --lanes $L > $O/b20_$L.log 2>&1 || { echo FAILED; tail -20 $O/b20_$L.log; exit 1; }
  echo -n "2^20 lanes $L: "; grep '"metric"' $O/b20_$L.log | python3 -c "$summ"
done
for L in 10 12 14 16; do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --log-n 16 --steps 16 --warmup 3 --lanes $L > $O/b16_$L.log 2>&1 || { echo FAILED; tail -20 $O/b16_$L.log; exit 1; }
  echo -n "2^16 lanes $L: "; grep '"metric"' $O/b16_$L.log | python3 -c "$summ"
done
for L in 12 16; do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --log-n 12 --steps 16 --warmup 3 --lanes $L > $O/b12_$L.log 2>&1 || { echo FAILED; tail -20 $O/b12_$L.log; exit 1; }
  echo -n "2^12 lanes $L: "; grep '"metric"' $O/b12_$L.log | python3 -c "$summ"
done
echo done
