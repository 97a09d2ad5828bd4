# NTT change check: NTT + prover parity tests, standalone NTT bench lines at 2^20 / 2^23,
# then the default bench line
set -o pipefail
export TMPDIR=/tmp
d=gpurun_out/ntt; rm -rf $d; mkdir -p $d
timeout -k 10 600 python -u -m pytest tests/test_ntt_gpu.py tests/test_prover_gpu.py tests/test_prover_oracle.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $d/tests.log 2>&1 || { echo TESTS_FAILED; tail -40 $d/tests.log; exit 1; }
tail -1 $d/tests.log
for k in 20 23; do
  timeout -k 10 300 python bench.py --mode ntt --log-n $k --steps 20 --warmup 3 --no-cpu-baseline > $d/ntt$k.log 2>&1 || { echo NTT_BENCH_FAILED; tail -20 $d/ntt$k.log; exit 1; }
  grep '"metric"' $d/ntt$k.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("ntt 2^'$k'", d["value"]/1e9, "G points/s", d["ms_per_step"], "ms/step", d.get("bit_exact_vs_oracle"))'
done
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 6 --warmup 2 > $d/bench20.log 2>&1 || { echo BENCH_FAILED; tail -20 $d/bench20.log; exit 1; }
grep '"metric"' $d/bench20.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,3), "M/s", round(d["ms_per_step"],2), "ms/step")'
