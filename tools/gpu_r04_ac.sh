#!/bin/bash
# Round 4: tail forms for prover lanes at 2^16 / 2^20 — PLK_TAIL_QUAD=0 (single-lane trees,
# the lanes' default above 2^14) against 2 (quad k_bitsum2 only), three times interleaved;
# parity of mode 2 first.
set -o pipefail
mkdir -p gpurun_out
PLK_TAIL_QUAD=2 timeout -k 10 600 python -u -m pytest tests/test_msm_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r04ac_tests.log 2>&1 || { tail -30 gpurun_out/r04ac_tests.log; exit 1; }
echo "tests (mode 2): $(tail -n 1 gpurun_out/r04ac_tests.log)"
out=gpurun_out/r04ac_ab.jsonl; : > $out
for r in 1 2 3; do
  for q in 0 2; do
    for args in "--log-n 16 --steps 20" "--log-n 20 --steps 10"; do
      line=$(PLK_TAIL_QUAD=$q timeout -k 10 300 python bench.py $args --warmup 3 --no-cpu-baseline 2>>gpurun_out/r04ac.err) || exit 1
      python -c "import json,sys;d=json.loads(sys.argv[1]);print(json.dumps({'tail':sys.argv[2],'args':sys.argv[3],'value':d['value'],'ms':d['ms_per_step'],'checked':d.get('proofs_checked')}))" "$line" $q "$args" | tee -a $out
    done
  done
done
