#!/bin/bash
# Round 4: (a) the quad k_bitsum1 of wide sets as two workgroups per group, (b) k_sort_one for
# batches up to 2^14 buckets (2^14 proofs' commits, one dispatch instead of five), (c)
# k_perm_numden without scratch. Parity, then interleaved: libplk (all) / libplk-sob0 (all but
# b) / libplk-prev (the previous commit + c).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_msm_gpu.py tests/test_prover_gpu.py tests/test_prover_oracle.py tests/test_prover_lanes.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r04z_tests.log 2>&1 || { tail -30 gpurun_out/r04z_tests.log; exit 1; }
echo "tests: $(tail -n 1 gpurun_out/r04z_tests.log)"
out=gpurun_out/r04z_ab.jsonl; : > $out
run() {  # lib args
  line=$(PLK_LIB=$PWD/dusk-plonk_amd/$1 timeout -k 10 300 python bench.py $2 --warmup 3 --no-cpu-baseline 2>>gpurun_out/r04z_ab.err) || return 1
  python -c "import json,sys;d=json.loads(sys.argv[1]);print(json.dumps({'lib':sys.argv[2],'args':sys.argv[3],'value':d['value'],'ms':d['ms_per_step'],'checked':d.get('proofs_checked', d.get('bit_exact_vs_oracle'))}))" "$line" $1 "$2" | tee -a $out
}
for r in 1 2; do
  for lib in libplk.so libplk-prev.so; do
    run $lib "--mode msm --log-n 16 --steps 50" || exit 1
    run $lib "--mode msm --log-n 20 --steps 30" || exit 1
  done
  for lib in libplk.so libplk-sob0.so libplk-prev.so; do
    run $lib "--log-n 14 --steps 20" || exit 1
    run $lib "--log-n 12 --steps 30" || exit 1
  done
done
for lib in libplk.so libplk-prev.so; do
  run $lib "--log-n 20 --steps 10" || exit 1
done
