# A/B: GPU parity tests on the default build, then the default bench line for each
# library given (default build first; others as dusk-plonk_amd/libplk-<variant>.so).
# usage: bash tools/gpu_ab.sh [variant ...]   (extra bench args in $BENCH_ARGS)
set -o pipefail
mkdir -p gpurun_out/ab
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 > gpurun_out/ab/tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/ab/tests.log; exit 1; }
tail -1 gpurun_out/ab/tests.log
summ='import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(round(d["value"]/1e6,3), "M/s", round(d["ms_per_step"],2), "ms/step acc", round(r["avg_launch_ms"],3), "solo", round(r["solo"]["avg_launch_ms"],3), round(r["solo"]["point_adds_per_s"]/1e9,3), "Gadd/s")'
for v in default "$@"; do
  if [ "$v" = default ]; then lib=""; else lib="$PWD/dusk-plonk_amd/libplk-$v.so"; fi
  PLK_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline $BENCH_ARGS > gpurun_out/ab/bench_$v.log 2>&1 || { echo BENCH_FAILED $v; tail -20 gpurun_out/ab/bench_$v.log; exit 1; }
  echo -n "$v: "; grep '"metric"' gpurun_out/ab/bench_$v.log | python3 -c "$summ"
done
