#!/bin/bash
# Round 4: the top window's digits spread over the bucket range (plk_srs::top_shift; c = 20
# at 2^20, c = 10 at 2^12): MSM / prover parity, then PLK_TOP_SPREAD=1 / 0 interleaved.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_msm_gpu.py tests/test_prover_gpu.py tests/test_prover_oracle.py tests/test_parallel.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r04u_tests.log 2>&1 || { tail -30 gpurun_out/r04u_tests.log; exit 1; }
echo "tests: $(tail -n 1 gpurun_out/r04u_tests.log)"
out=gpurun_out/r04u_ab.jsonl; : > $out
run() {  # spread args
  line=$(PLK_TOP_SPREAD=$1 timeout -k 10 300 python bench.py $2 --warmup 3 --no-cpu-baseline 2>>gpurun_out/r04u_ab.err) || return 1
  python -c "import json,sys;d=json.loads(sys.argv[1]);print(json.dumps({'spread':sys.argv[2],'args':sys.argv[3],'value':d['value'],'ms':d['ms_per_step'],'checked':d.get('proofs_checked', d.get('bit_exact_vs_oracle'))}))" "$line" $1 "$2" | tee -a $out
}
for r in 1 2; do
  for sp in 1 0; do
    run $sp "--mode msm --log-n 20 --steps 30" || exit 1
    run $sp "--log-n 12 --steps 30" || exit 1
    run $sp "--log-n 20 --steps 10" || exit 1
  done
done
