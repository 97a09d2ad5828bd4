# A/B at n = 2^20: default bench line for each library variant (dusk-plonk_amd/libplk-<v>.so),
# twice, interleaved; then the default library at other lane counts
# usage: bash tools/gpu_ab20.sh [variant ...]
set -o pipefail
export TMPDIR=/tmp
d=gpurun_out/ab20; rm -rf $d; mkdir -p $d
summ='import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,3), "M/s", round(d["ms_per_step"],2), "ms/step")'
for rep in 1 2; do
  for v in default "$@"; do
    if [ "$v" = default ]; then lib=""; else lib="$PWD/dusk-plonk_amd/libplk-$v.so"; fi
    PLK_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --steps 8 --warmup 2 > $d/bench_${v}_$rep.log 2>&1 || { echo BENCH_FAILED $v; tail -20 $d/bench_${v}_$rep.log; exit 1; }
    echo -n "2^20 $v #$rep: "; grep '"metric"' $d/bench_${v}_$rep.log | python3 -c "$summ"
  done
done
for L in ${LANES:-}; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 8 --warmup 2 --lanes $L > $d/bench_l$L.log 2>&1 || { echo BENCH_FAILED l$L; exit 1; }
  echo -n "2^20 lanes $L: "; grep '"metric"' $d/bench_l$L.log | python3 -c "$summ"
done
