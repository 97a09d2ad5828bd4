# A/B at n = 2^16 only: default bench line for each library, twice, interleaved
# usage: bash tools/gpu_ab16.sh [variant ...]
set -o pipefail
export TMPDIR=/tmp
d=gpurun_out/ab16; rm -rf $d; mkdir -p $d
summ='import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,3), "M/s", round(d["ms_per_step"],2), "ms/step")'
for rep in 1 2; do
  for v in default "$@"; do
    if [ "$v" = default ]; then lib=""; else lib="$PWD/dusk-plonk_amd/libplk-$v.so"; fi
    PLK_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --log-n 16 --steps 10 --warmup 3 > $d/bench_${v}_$rep.log 2>&1 || { echo BENCH_FAILED $v; tail -20 $d/bench_${v}_$rep.log; exit 1; }
    echo -n "2^16 $v #$rep: "; grep '"metric"' $d/bench_${v}_$rep.log | python3 -c "$summ"
  done
done
