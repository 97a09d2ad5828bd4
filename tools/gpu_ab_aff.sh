#!/bin/bash
# batch-affine pair levels: MSM + prover parity tests on the default build, then bench A/B
# at 2^20 and 2^16 against variants (libplk-<v>.so), interleaved
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
d=gpurun_out/abaff; rm -rf $d; mkdir -p $d
timeout -k 10 600 python3 -u -m pytest tests/test_msm_gpu.py tests/test_prover_oracle.py tests/test_prover_gpu.py -x -q --timeout 300 --timeout-method thread > $d/tests.log 2>&1 || { tail -40 $d/tests.log; exit 1; }
tail -2 $d/tests.log
summ='import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(round(d["value"]/1e6,3), "M/s", round(d["ms_per_step"],2), "ms/step; acc solo", round(r["avg_launch_ms"],3), "ms")'
for k in 20 16; do
  for v in default "$@"; do
    if [ "$v" = default ]; then lib=""; else lib="$PWD/dusk-plonk_amd/libplk-$v.so"; fi
    PLK_LIB=$lib timeout -k 10 300 python3 bench.py --no-cpu-baseline --log-n $k --steps 8 --warmup 2 > $d/bench_${v}_$k.log 2>&1 || { echo BENCH_FAILED $v; tail -20 $d/bench_${v}_$k.log; exit 1; }
    echo -n "2^$k $v: "; grep '"metric"' $d/bench_${v}_$k.log | python3 -c "$summ"
  done
done
