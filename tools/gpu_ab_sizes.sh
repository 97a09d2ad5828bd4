# A/B at both metric sizes: GPU MSM + prover parity tests on the default build, then the
# bench line (2^20 and 2^16, default lanes) and the single-lane kernel breakdown for each
# library (default build first; others as dusk-plonk_amd/libplk-<variant>.so), interleaved
# so that box-to-box clock differences cancel.
# usage: bash tools/gpu_ab_sizes.sh [variant ...]
set -o pipefail
export TMPDIR=/tmp
d=gpurun_out/abs; rm -rf $d; mkdir -p $d
timeout -k 10 400 python -u -m pytest tests/test_msm_gpu.py tests/test_prover_gpu.py -x -q -p no:cacheprovider --timeout 200 > $d/tests.log 2>&1 || { echo TESTS_FAILED; tail -40 $d/tests.log; exit 1; }
tail -1 $d/tests.log
summ='import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,3), "M/s", round(d["ms_per_step"],2), "ms/step")'
for k in 20 16; do
  for v in default "$@"; do
    if [ "$v" = default ]; then lib=""; else lib="$PWD/dusk-plonk_amd/libplk-$v.so"; fi
    PLK_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --log-n $k $( [ $k = 16 ] && echo "--steps 20 --warmup 3" ) > $d/bench_${v}_$k.log 2>&1 || { echo BENCH_FAILED $v; tail -20 $d/bench_${v}_$k.log; exit 1; }
    echo -n "2^$k $v: "; grep '"metric"' $d/bench_${v}_$k.log | python3 -c "$summ"
  done
done
for k in 20 16; do
  for v in default "$@"; do
    if [ "$v" = default ]; then export PLK_LIB=""; else export PLK_LIB="$PWD/dusk-plonk_amd/libplk-$v.so"; fi
    o=$d/bd_${v}_$k; mkdir -p $o
    timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $o -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --lanes 1 --log-n $k > $o/bench.log 2>&1 || { echo PROF_FAILED; tail -20 $o/bench.log; exit 1; }
    echo "== 2^$k $v"; python3 tools/trace_breakdown.py $o/run_kernel_trace.csv | tee $o/breakdown.txt | head -9
  done
done
