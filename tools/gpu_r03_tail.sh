#!/bin/bash
# MSM reduction tail with lazy additions: ubench, MSM parity tests, lone-MSM bench + trace,
# and a proof-throughput check at 2^12 / 2^16 / 2^20 against the previous library.
set -uo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/.."
O=gpurun_out/r03tail
rm -rf $O; mkdir -p $O
timeout -k 10 120 ./tools/ubench_tail > $O/ubench_tail.txt 2>&1 || { echo UBENCH_FAILED; cat $O/ubench_tail.txt; exit 1; }
cat $O/ubench_tail.txt
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_msm_gpu.py tests/test_msm_reduction_identity.py tests/test_prover_oracle.py > $O/pytest.log 2>&1 || { echo PYTEST_FAILED; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for k in 20 16; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/t$k -o run -- python3 bench.py --mode msm --log-n $k --steps 12 --warmup 3 --no-cpu-baseline > $O/m$k.log 2>&1 || { echo PROF_FAILED $k; tail -20 $O/m$k.log; exit 1; }
  echo "== lone MSM 2^$k"; grep -o '"ms_per_step": [0-9.]*' $O/m$k.log; grep -o '"bit_exact_vs_oracle": [a-z]*' $O/m$k.log
  python3 tools/msm_trace.py $O/t$k/run_kernel_trace.csv 8 | tee $O/msm_summary$k.txt
done
for rl in 65536; do
  PLK_RUN_LANES=$rl timeout -k 10 300 python3 bench.py --mode msm --log-n 20 --steps 12 --warmup 3 --no-cpu-baseline > $O/m20_rl$rl.log 2>&1 || { echo SWEEP_FAILED; tail -20 $O/m20_rl$rl.log; exit 1; }
  echo -n "lone 2^20 run lanes $rl: "; grep -o '"ms_per_step": [0-9.]*' $O/m20_rl$rl.log
done
summ='import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,3), "M", round(d["ms_per_step"],2), "ms/step")'
for k in 12 16 20; do
  st=16; [ $k = 20 ] && st=6
  for lib in new prev; do
    if [ $lib = prev ]; then cp dusk-plonk_amd/libplk.so $O/libplk-new.so; cp dusk-plonk_amd/libplk-prev.so dusk-plonk_amd/libplk.so; fi
    timeout -k 10 300 python3 bench.py --no-cpu-baseline --log-n $k --steps $st --warmup 2 > $O/b${k}_$lib.log 2>&1 || { echo BENCH_FAILED; tail -20 $O/b${k}_$lib.log; cp $O/libplk-new.so dusk-plonk_amd/libplk.so; exit 1; }
    if [ $lib = prev ]; then cp $O/libplk-new.so dusk-plonk_amd/libplk.so; fi
    echo -n "prove 2^$k $lib: "; grep '"metric"' $O/b${k}_$lib.log | python3 -c "$summ"
  done
done
echo done
