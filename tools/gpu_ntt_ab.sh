# NTT A/B: NTT + prover parity on the default library, then the standalone NTT lines at
# 2^20 / 2^23 for the default build and each variant (dusk-plonk_amd/libplk-<v>.so),
# interleaved twice so box drift cancels.   usage: bash tools/gpu_ntt_ab.sh [variant ...]
set -o pipefail
export TMPDIR=/tmp
d=gpurun_out/ntt_ab; rm -rf $d; mkdir -p $d
timeout -k 10 600 python -u -m pytest tests/test_ntt_gpu.py tests/test_prover_oracle.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $d/tests.log 2>&1 || { echo TESTS_FAILED; tail -40 $d/tests.log; exit 1; }
tail -1 $d/tests.log
summ='import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e9,3), "G points/s", round(d["ms_per_step"],4), "ms/step exact", d.get("bit_exact_vs_oracle"))'
for rep in 1 2; do
  for k in 20 23; do
    for v in default "$@"; do
      if [ "$v" = default ]; then lib=""; else lib="$PWD/dusk-plonk_amd/libplk-$v.so"; fi
      PLK_LIB=$lib timeout -k 10 300 python bench.py --mode ntt --log-n $k --steps 20 --warmup 3 --no-cpu-baseline > $d/ntt_${v}_${k}_$rep.log 2>&1 || { echo NTT_BENCH_FAILED $v; tail -20 $d/ntt_${v}_${k}_$rep.log; exit 1; }
      echo -n "2^$k $v #$rep: "; grep '"metric"' $d/ntt_${v}_${k}_$rep.log | python3 -c "$summ"
    done
  done
done
