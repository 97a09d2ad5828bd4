#!/bin/bash
# Lone-MSM-only adaptive runs + single readback copy: MSM / prover parity, lone MSM lines,
# size sweep.
set -uo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/.."
O=gpurun_out/r03h
rm -rf $O; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 \
  || { echo TESTS_FAILED; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
summ='import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,3), "M", d["unit"], round(d["ms_per_step"],3), "ms/step")'
for k in 20 16; do
  timeout -k 10 300 python3 bench.py --mode msm --log-n $k --steps 20 --warmup 3 --no-cpu-baseline > $O/msm${k}.log 2>&1 || { echo MSM_FAILED; tail -20 $O/msm${k}.log; exit 1; }
  echo -n "msm 2^$k: "; grep '"metric"' $O/msm${k}.log | python3 -c "$summ"
done
for k in 12 14 16 18 20; do
  timeout -k 10 300 python3 bench.py --log-n $k --no-cpu-baseline --steps 10 --warmup 2 > $O/b$k.log 2>&1 || { echo BENCH_FAILED $k; tail -20 $O/b$k.log; exit 1; }
  echo -n "prove 2^$k: "; grep '"metric"' $O/b$k.log | python3 -c "$summ"
done
PLK_LIB=$PWD/dusk-plonk_amd/libplk-base.so timeout -k 10 300 python3 bench.py --log-n 16 --no-cpu-baseline --steps 10 --warmup 2 > $O/b16base.log 2>&1 || { echo BENCH_FAILED base; exit 1; }
echo -n "prove 2^16 base: "; grep '"metric"' $O/b16base.log | python3 -c "$summ"
echo done
