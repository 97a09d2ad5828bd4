# MSM change check: MSM + prover parity tests, standalone MSM lines (2^20, 2^16), default
# bench lines (2^20, 2^16), single-lane 2^20 breakdown
set -o pipefail
export TMPDIR=/tmp
d=gpurun_out/msmchk; rm -rf $d; mkdir -p $d
timeout -k 10 600 python -u -m pytest tests/test_msm_gpu.py tests/test_prover_gpu.py tests/test_prover_lanes.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $d/tests.log 2>&1 || { echo TESTS_FAILED; tail -40 $d/tests.log; exit 1; }
tail -1 $d/tests.log
for k in 20 16; do
  timeout -k 10 300 python bench.py --mode msm --log-n $k --steps 10 --warmup 2 --no-cpu-baseline > $d/msm$k.log 2>&1 || { echo MSM_BENCH_FAILED; tail -20 $d/msm$k.log; exit 1; }
  grep '"metric"' $d/msm$k.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("msm 2^'$k'", round(d["value"]/1e6,1), "M points/s", round(d["ms_per_step"],3), "ms")'
done
for k in 20 16; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --log-n $k $( [ $k = 16 ] && echo "--steps 20 --warmup 3" || echo "--steps 6 --warmup 2" ) > $d/b$k.log 2>&1 || { echo BENCH_FAILED; tail -20 $d/b$k.log; exit 1; }
  grep '"metric"' $d/b$k.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("prove 2^'$k'", round(d["value"]/1e6,3), "M/s", round(d["ms_per_step"],2), "ms/step")'
done
bash tools/gpu_bd20.sh
