# A/B of environment settings on the default library: MSM + prover parity tests (default
# env), then bench lines per size for "default" and each VAR=value variant, twice
# interleaved. usage: SIZES="12 16 20" bash tools/gpu_ab_env.sh PLK_MSM_GRAPHS=0 ...
set -o pipefail
export TMPDIR=/tmp
d=gpurun_out/abenv; rm -rf $d; mkdir -p $d
timeout -k 10 600 python -u -m pytest tests/test_msm_gpu.py tests/test_prover_gpu.py tests/test_prover_lanes.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $d/tests.log 2>&1 || { echo TESTS_FAILED; tail -40 $d/tests.log; exit 1; }
tail -1 $d/tests.log
summ='import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,3), "M/s", round(d["ms_per_step"],2), "ms/step")'
for rep in 1 2; do
  for k in ${SIZES:-12 16 20}; do
    for v in default "$@"; do
      st=$([ $k -le 16 ] && echo "--steps 20 --warmup 3" || echo "--steps 6 --warmup 2")
      if [ "$v" = default ]; then envs=""; else envs="$v"; fi
      env $envs timeout -k 10 300 python bench.py --no-cpu-baseline --log-n $k $st > $d/b_${k}_${v}_$rep.log 2>&1 || { echo BENCH_FAILED $k $v; tail -20 $d/b_${k}_${v}_$rep.log; exit 1; }
      echo -n "2^$k $v #$rep: "; grep '"metric"' $d/b_${k}_${v}_$rep.log | python3 -c "$summ"
    done
  done
done
