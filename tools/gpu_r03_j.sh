#!/bin/bash
# Same-box A/B of the current library against libplk-prev.so (the last commit) at 2^20 /
# 2^16 / 2^12, interleaved twice, after the NTT / MSM / prover parity tests of the current one.
set -uo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/.."
O=gpurun_out/r03j
rm -rf $O; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests/test_ntt_gpu.py tests/test_msm_gpu.py tests/test_prover_oracle.py tests/test_prover_gpu.py tests/test_prover_lanes.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 \
  || { echo TESTS_FAILED; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
summ='import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,3), "M", round(d["ms_per_step"],3), "ms/step")'
for rep in 1 2; do
  for v in new prev; do
    if [ "$v" = new ]; then lib=""; else lib="$PWD/dusk-plonk_amd/libplk-prev.so"; fi
    for k in 20 16 12; do
      st=10; [ $k = 20 ] && st=8
      PLK_LIB=$lib timeout -k 10 300 python3 bench.py --log-n $k --no-cpu-baseline --steps $st --warmup 2 > $O/b${k}_${v}_$rep.log 2>&1 || { echo BENCH_FAILED $v $k; tail -20 $O/b${k}_${v}_$rep.log; exit 1; }
      echo -n "2^$k $v #$rep: "; grep '"metric"' $O/b${k}_${v}_$rep.log | python3 -c "$summ"
    done
  done
done
echo done
