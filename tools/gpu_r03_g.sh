#!/bin/bash
# Adaptive run length: MSM / prover parity, lone-MSM lines at 2^20 and 2^16 (new vs base
# library), and the size sweep 2^12..2^20 of the default bench.
set -uo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/.."
O=gpurun_out/r03g
rm -rf $O; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_msm_gpu.py tests/test_prover_oracle.py tests/test_prover_gpu.py tests/test_bench.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 \
  || { echo TESTS_FAILED; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
summ='import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(round(d["value"]/1e6,3), "M", d["unit"], round(d["ms_per_step"],3), "ms/step")'
for k in 20 16; do
  for v in new base; do
    if [ "$v" = new ]; then lib=""; else lib="$PWD/dusk-plonk_amd/libplk-base.so"; fi
    PLK_LIB=$lib timeout -k 10 300 python3 bench.py --mode msm --log-n $k --steps 20 --warmup 3 --no-cpu-baseline > $O/msm${k}_${v}.log 2>&1 || { echo MSM_FAILED $v; tail -20 $O/msm${k}_${v}.log; exit 1; }
    echo -n "msm 2^$k $v: "; grep '"metric"' $O/msm${k}_${v}.log | python3 -c "$summ"
  done
done
for k in 12 14 16 18 20; do
  timeout -k 10 300 python3 bench.py --log-n $k --no-cpu-baseline --steps 10 --warmup 2 > $O/b$k.log 2>&1 || { echo BENCH_FAILED $k; tail -20 $O/b$k.log; exit 1; }
  echo -n "prove 2^$k: "; grep '"metric"' $O/b$k.log | python3 -c "$summ"
done
echo done
# lone-transform generations (PLK_NTT_WG_LDS: LDS floor per workgroup -> WGs per CU)
for lds in 0 54000 80000; do
  for k in 20 23; do
    PLK_NTT_WG_LDS=$lds timeout -k 10 200 python3 bench.py --mode ntt --log-n $k --steps 20 --warmup 3 --no-cpu-baseline > $O/ntt${k}_$lds.log 2>&1 || { echo NTT_FAILED; tail -20 $O/ntt${k}_$lds.log; exit 1; }
    echo -n "ntt 2^$k lds $lds: "; grep '"metric"' $O/ntt${k}_$lds.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(round(r["dft_ms"],4), round(r["idft_ms"],4), "ms dft/idft")'
  done
done
echo done2
