# Quick A/B of library variants (dusk-plonk_amd/libplk-<v>.so) against the default build:
# MSM + prover parity tests on every variant, then the bench line at 2^20 and 2^16 for each
# library, interleaved twice so that box clock drift cancels. Prints value and the solo
# k_accumulate launch time of each run.
# usage: bash tools/gpu_ab_quick.sh [variant ...]   (SIZES="20 16" by default)
set -o pipefail
export TMPDIR=/tmp
d=gpurun_out/abq; rm -rf $d; mkdir -p $d
for v in "$@"; do
  PLK_LIB="$PWD/dusk-plonk_amd/libplk-$v.so" timeout -k 10 400 python -u -m pytest tests/test_msm_gpu.py tests/test_prover_gpu.py -x -q -p no:cacheprovider --timeout 200 > $d/tests_$v.log 2>&1 || { echo TESTS_FAILED $v; tail -40 $d/tests_$v.log; exit 1; }
  echo -n "tests $v: "; tail -1 $d/tests_$v.log
done
summ='import json,sys; d=json.loads(sys.stdin.read()); s=d["roofline"].get("solo",{}); print(round(d["value"]/1e6,3), "M/s", round(d["ms_per_step"],2), "ms/step; solo acc", round(s.get("avg_launch_ms",0),3), "ms")'
for rep in 1 2; do
  for k in ${SIZES:-20 16}; do
    for v in default "$@"; do
      if [ "$v" = default ]; then lib=""; else lib="$PWD/dusk-plonk_amd/libplk-$v.so"; fi
      PLK_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --log-n $k $( [ $k = 16 ] && echo "--steps 20 --warmup 3" || echo "--steps 6 --warmup 2" ) > $d/bench_${v}_${k}_$rep.log 2>&1 || { echo BENCH_FAILED $v; tail -20 $d/bench_${v}_${k}_$rep.log; exit 1; }
      echo -n "2^$k $v #$rep: "; grep '"metric"' $d/bench_${v}_${k}_$rep.log | python3 -c "$summ"
    done
  done
done
