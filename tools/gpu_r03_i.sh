#!/bin/bash
# r(X) folded into the evaluation batch and the opening aggregate, the wire blinds in one
# launch, PI(X) direct: whole -m gpu suite, size sweep, and the NTT tile-size sweep
# (PLK_NTT_LE_MIN) at the small sizes.
set -uo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/.."
O=gpurun_out/r03i
rm -rf $O; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 \
  || { echo TESTS_FAILED; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
summ='import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,3), "M", d["unit"], round(d["ms_per_step"],3), "ms/step")'
for k in 12 14 16 18 20; do
  timeout -k 10 300 python3 bench.py --log-n $k --no-cpu-baseline --steps 10 --warmup 2 > $O/b$k.log 2>&1 || { echo BENCH_FAILED $k; tail -20 $O/b$k.log; exit 1; }
  echo -n "prove 2^$k: "; grep '"metric"' $O/b$k.log | python3 -c "$summ"
done
for le in 8 9 10; do
  for k in 12 14 16; do
    PLK_NTT_LE_MIN=$le timeout -k 10 300 python3 bench.py --log-n $k --no-cpu-baseline --steps 10 --warmup 2 > $O/le${le}_$k.log 2>&1 || { echo BENCH_FAILED le$le $k; tail -20 $O/le${le}_$k.log; exit 1; }
    echo -n "le_min $le prove 2^$k: "; grep '"metric"' $O/le${le}_$k.log | python3 -c "$summ"
  done
done
echo done
