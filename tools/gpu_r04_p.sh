#!/bin/bash
# Round 4: (1) prover lanes' tail form: PLK_TAIL_QUAD=1 / 0 interleaved at 2^14 / 2^16 / 2^20
# (twice); (2) madd grouping A/B, default against libplk-g2 (PLK_MADD_GROUPED=2): the
# accumulate micro-benchmark and 2^20 proofs / lone MSMs.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_msm_gpu.py tests/test_prover_gpu.py tests/test_prover_lanes.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r04p_tests0.log 2>&1 || { tail -30 gpurun_out/r04p_tests0.log; exit 1; }
echo "quad bucket-sum tests: $(tail -n 1 gpurun_out/r04p_tests0.log)"
out=gpurun_out/r04p_ab.jsonl; : > $out
run() {  # tag env lib args
  line=$(env $2 PLK_LIB=$PWD/dusk-plonk_amd/$3 timeout -k 10 300 python bench.py $4 --warmup 3 --no-cpu-baseline 2>>gpurun_out/r04p_ab.err) || return 1
  python -c "import json,sys;d=json.loads(sys.argv[1]);print(json.dumps({'tag':sys.argv[2],'args':sys.argv[3],'value':d['value'],'ms':d['ms_per_step'],'checked':d.get('proofs_checked', d.get('bit_exact_vs_oracle'))}))" "$line" "$1" "$4" | tee -a $out
}
for r in 1 2; do
  for q in 1 0; do
    run quad$q PLK_TAIL_QUAD=$q libplk.so "--log-n 12 --steps 30" || exit 1
    run quad$q PLK_TAIL_QUAD=$q libplk.so "--log-n 14 --steps 20" || exit 1
    run quad$q PLK_TAIL_QUAD=$q libplk.so "--log-n 16 --steps 20" || exit 1
    run quad$q PLK_TAIL_QUAD=$q libplk.so "--log-n 20 --steps 10" || exit 1
  done
done
for r in 1 2; do
  for v in grp grp2; do
    echo "== $v run $r"; timeout -k 10 120 ./tools/ubench_acc_$v | grep v4_lazy || exit 1
  done
done 2>&1 | tee gpurun_out/r04p_ubench.txt || exit 1
PLK_LIB=$PWD/dusk-plonk_amd/libplk-g2.so timeout -k 10 400 python -u -m pytest tests/test_msm_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r04p_tests.log 2>&1 || { tail -30 gpurun_out/r04p_tests.log; exit 1; }
echo "g2 msm tests: $(tail -n 1 gpurun_out/r04p_tests.log)"
for r in 1 2; do
  for lib in libplk.so libplk-g2.so; do
    run $lib X=1 $lib "--log-n 20 --steps 10" || exit 1
    run $lib X=1 $lib "--mode msm --log-n 20 --steps 30" || exit 1
  done
done
