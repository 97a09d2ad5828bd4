#!/bin/bash
# MSM A/B: MSM parity tests on each variant library (PLK_LIB=dusk-plonk_amd/libplk-<v>.so),
# then lone-MSM lines (bench.py --mode msm) at 2^16 / 2^20 for the default build and each
# variant, interleaved twice so box drift cancels.   usage: bash tools/gpu_msm_ab.sh <variant ...>
set -o pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/.."
d=gpurun_out/msm_ab; rm -rf $d; mkdir -p $d
for v in "$@"; do
  PLK_LIB=$PWD/dusk-plonk_amd/libplk-$v.so timeout -k 10 600 python3 -u -m pytest tests/test_msm_gpu.py tests/test_msm_reduction_identity.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $d/tests_$v.log 2>&1 || { echo TESTS_FAILED $v; tail -30 $d/tests_$v.log; exit 1; }
  echo -n "$v tests: "; tail -1 $d/tests_$v.log
done
summ='import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],4), "ms;", round(d["value"]/1e6,2), "M points/s; exact", d.get("bit_exact_vs_oracle"))'
for rep in 1 2; do
  for k in 16 20; do
    for v in default "$@"; do
      if [ "$v" = default ]; then lib=""; else lib="$PWD/dusk-plonk_amd/libplk-$v.so"; fi
      PLK_LIB=$lib timeout -k 10 240 python3 bench.py --mode msm --log-n $k --steps 20 --warmup 3 --no-cpu-baseline > $d/m_${v}_${k}_$rep.log 2>&1 || { echo MSM_BENCH_FAILED $v $k; tail -20 $d/m_${v}_${k}_$rep.log; exit 1; }
      echo -n "2^$k $v #$rep: "; grep '"metric"' $d/m_${v}_${k}_$rep.log | python3 -c "$summ"
    done
  done
done
echo done
