# wide-bucket MSM path: MSM parity tests (incl. 2^20 vs the oracle), prover tests, then the
# single-lane 2^20 breakdown and the default bench line
set -o pipefail
export TMPDIR=/tmp
d=gpurun_out/wide; rm -rf $d; mkdir -p $d
timeout -k 10 600 python -u -m pytest tests/test_msm_gpu.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $d/msm_tests.log 2>&1 || { echo MSM_TESTS_FAILED; tail -40 $d/msm_tests.log; exit 1; }
tail -2 $d/msm_tests.log
timeout -k 10 600 python -u -m pytest tests/test_prover_gpu.py tests/test_prover_oracle.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $d/prover_tests.log 2>&1 || { echo PROVER_TESTS_FAILED; tail -40 $d/prover_tests.log; exit 1; }
tail -2 $d/prover_tests.log
bash tools/gpu_bd20.sh || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 6 --warmup 2 > $d/bench20.log 2>&1 || { echo BENCH_FAILED; tail -20 $d/bench20.log; exit 1; }
grep '"metric"' $d/bench20.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); s=d["roofline"].get("solo",{}); print(round(d["value"]/1e6,3), "M/s", round(d["ms_per_step"],2), "ms/step; solo acc", round(s.get("avg_launch_ms",0),3), "ms")'
