#!/bin/bash
# Full GPU test suite, then the proof-size sweep (2^12..2^20) and the lone MSM / NTT lines.
set -uo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/.."
O=gpurun_out/r03full
rm -rf $O; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests/ -x -v --timeout 300 --timeout-method thread -m gpu > $O/pytest.log 2>&1 || { echo PYTEST_FAILED; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
summ='import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,3), "M/s", round(d["ms_per_step"],4), "ms/step")'
for k in 12 14 16 18 20; do
  st=16; [ $k = 20 ] && st=6; [ $k = 18 ] && st=10
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --log-n $k --steps $st --warmup 2 > $O/b$k.log 2>&1 || { echo BENCH_FAILED; tail -20 $O/b$k.log; exit 1; }
  echo -n "prove 2^$k: "; grep '"metric"' $O/b$k.log | python3 -c "$summ"
done
for m in ntt msm; do
  for k in 16 20; do
    timeout -k 10 300 python3 bench.py --mode $m --log-n $k --steps 20 --warmup 3 --no-cpu-baseline > $O/$m$k.log 2>&1 || { echo MODE_FAILED; tail -20 $O/$m$k.log; exit 1; }
    echo -n "$m 2^$k: "; grep '"metric"' $O/$m$k.log | python3 -c "$summ"
  done
done
echo done
