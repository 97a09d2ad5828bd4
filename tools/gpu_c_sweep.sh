# window-size sweep through PLK_MSM_C (srs.hip choose_c override): default bench lines at
# 2^16 and 2^20, interleaved twice. usage: bash tools/gpu_c_sweep.sh "15 16 17" "19 20 21"
set -o pipefail
export TMPDIR=/tmp
d=gpurun_out/csweep; rm -rf $d; mkdir -p $d
summ='import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,3), "M/s", round(d["ms_per_step"],2), "ms/step; c", d["config"].get("msm_window_bits"))'
for rep in 1 2; do
  for c in ${1:-15 16 17}; do
    PLK_MSM_C=$c timeout -k 10 300 python bench.py --no-cpu-baseline --log-n ${LOGN:-16} --steps 20 --warmup 3 > $d/b16_${c}_$rep.log 2>&1 || { echo BENCH_FAILED 16 $c; tail -20 $d/b16_${c}_$rep.log; exit 1; }
    echo -n "2^${LOGN:-16} c=$c #$rep: "; grep '"metric"' $d/b16_${c}_$rep.log | python3 -c "$summ"
  done
  for c in ${2:-}; do
    PLK_MSM_C=$c timeout -k 10 300 python bench.py --no-cpu-baseline --log-n 20 --steps 6 --warmup 2 > $d/b20_${c}_$rep.log 2>&1 || { echo BENCH_FAILED 20 $c; tail -20 $d/b20_${c}_$rep.log; exit 1; }
    echo -n "2^20 c=$c #$rep: "; grep '"metric"' $d/b20_${c}_$rep.log | python3 -c "$summ"
  done
done
