#!/bin/bash
# Round 3: 13 x 30 Fp limbs. MSM / prover parity tests first, then the A/B of the new library
# against libplk-base.so (the committed 14 x 28 build) at 2^20 and 2^16 (interleaved, twice)
# and the lone 2^20 MSM line of both.
set -uo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/.."
O=gpurun_out/r03c
rm -rf $O; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_msm_gpu.py tests/test_field_gpu.py tests/test_prover_oracle.py tests/test_prover_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 \
  || { echo TESTS_FAILED; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
summ='import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(round(d["value"]/1e6,3), d["unit"], round(d["ms_per_step"],2), "ms/step", "adds/s", "%.3g" % r.get("point_adds_per_s", 0), "frac", round(r["frac"],3))'
for rep in 1 2; do
  for v in new base; do
    if [ "$v" = new ]; then lib=""; else lib="$PWD/dusk-plonk_amd/libplk-base.so"; fi
    PLK_LIB=$lib timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 8 --warmup 2 > $O/b20_${v}_$rep.log 2>&1 || { echo BENCH_FAILED $v; tail -20 $O/b20_${v}_$rep.log; exit 1; }
    echo -n "2^20 $v #$rep: "; grep '"metric"' $O/b20_${v}_$rep.log | python3 -c "$summ"
    PLK_LIB=$lib timeout -k 10 300 python3 bench.py --no-cpu-baseline --log-n 16 --steps 20 --warmup 3 > $O/b16_${v}_$rep.log 2>&1 || { echo BENCH16_FAILED $v; tail -20 $O/b16_${v}_$rep.log; exit 1; }
    echo -n "2^16 $v #$rep: "; grep '"metric"' $O/b16_${v}_$rep.log | python3 -c "$summ"
  done
done
for v in new base; do
  if [ "$v" = new ]; then lib=""; else lib="$PWD/dusk-plonk_amd/libplk-base.so"; fi
  PLK_LIB=$lib timeout -k 10 300 python3 bench.py --mode msm --steps 20 --warmup 3 --no-cpu-baseline > $O/msm_${v}.log 2>&1 || { echo MSM_FAILED $v; tail -20 $O/msm_${v}.log; exit 1; }
  echo -n "msm 2^20 $v: "; grep '"metric"' $O/msm_${v}.log | python3 -c "$summ"
done
echo done
