# one iteration: MSM + prover GPU parity tests, A/B bench of the given variants, and the
# single-lane kernel breakdown of the default build
# usage: bash tools/gpu_iter.sh [variant ...]
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/it
timeout -k 10 400 python -u -m pytest tests/test_msm_gpu.py tests/test_prover_gpu.py -x -q -p no:cacheprovider --timeout 200 > gpurun_out/it/tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/it/tests.log; exit 1; }
tail -1 gpurun_out/it/tests.log
summ='import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(round(d["value"]/1e6,3), "M/s", round(d["ms_per_step"],2), "ms/step acc", round(r["avg_launch_ms"],3), "solo", round(r["solo"]["avg_launch_ms"],3), round(r["solo"]["point_adds_per_s"]/1e9,3), "Gadd/s")'
for v in default "$@"; do
  if [ "$v" = default ]; then lib=""; else lib="$PWD/dusk-plonk_amd/libplk-$v.so"; fi
  PLK_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline $BENCH_ARGS > gpurun_out/it/bench_$v.log 2>&1 || { echo BENCH_FAILED $v; tail -20 gpurun_out/it/bench_$v.log; exit 1; }
  echo -n "$v: "; grep '"metric"' gpurun_out/it/bench_$v.log | python3 -c "$summ"
done
for v in default "$@"; do
  timeout -k 10 400 bash tools/gpu_breakdown.sh $v > gpurun_out/it/bd_$v.txt 2>&1 || { echo BD_FAILED; tail -20 gpurun_out/it/bd_$v.txt; exit 1; }
  echo "== $v"; head -12 gpurun_out/it/bd_$v.txt
done
