#!/bin/bash
# Round 4: the wide sort's temporary as 4-byte codes + 2-byte in-bin buckets (6 instead of 8
# bytes per entry; k_fine's counting pass reads 2) — parity, then interleaved against the
# previous commit (libplk-prev): lone MSMs 2^16 / 2^20, 2^20 proofs.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_msm_gpu.py tests/test_prover_oracle.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r04ad_tests.log 2>&1 || { tail -30 gpurun_out/r04ad_tests.log; exit 1; }
echo "tests: $(tail -n 1 gpurun_out/r04ad_tests.log)"
out=gpurun_out/r04ad_ab.jsonl; : > $out
run() {  # lib args
  line=$(PLK_LIB=$PWD/dusk-plonk_amd/$1 timeout -k 10 300 python bench.py $2 --warmup 3 --no-cpu-baseline 2>>gpurun_out/r04ad_ab.err) || return 1
  python -c "import json,sys;d=json.loads(sys.argv[1]);print(json.dumps({'lib':sys.argv[2],'args':sys.argv[3],'value':d['value'],'ms':d['ms_per_step'],'checked':d.get('proofs_checked', d.get('bit_exact_vs_oracle'))}))" "$line" $1 "$2" | tee -a $out
}
for r in 1 2; do
  for lib in libplk.so libplk-prev.so; do
    run $lib "--mode msm --log-n 20 --steps 30" || exit 1
    run $lib "--mode msm --log-n 16 --steps 50" || exit 1
    run $lib "--log-n 20 --steps 10" || exit 1
  done
done
