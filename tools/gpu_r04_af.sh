#!/bin/bash
# Round 4: single-dispatch Ruffini with y_j parked in q (2 products per element in its second
# pass instead of 4) — prover / opening parity, then 2^12 / 2^14 proofs interleaved against
# the previous commit (libplk-prev), twice.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_prover_gpu.py tests/test_prover_oracle.py tests/test_opening_gpu.py tests/test_prover_lanes.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r04af_tests.log 2>&1 || { tail -30 gpurun_out/r04af_tests.log; exit 1; }
echo "tests: $(tail -n 1 gpurun_out/r04af_tests.log)"
out=gpurun_out/r04af_ab.jsonl; : > $out
for r in 1 2; do
  for lib in libplk.so libplk-prev.so; do
    for args in "--log-n 12 --steps 30" "--log-n 14 --steps 20"; do
      line=$(PLK_LIB=$PWD/dusk-plonk_amd/$lib timeout -k 10 300 python bench.py $args --warmup 3 --no-cpu-baseline 2>>gpurun_out/r04af.err) || exit 1
      python -c "import json,sys;d=json.loads(sys.argv[1]);print(json.dumps({'lib':sys.argv[2],'args':sys.argv[3],'value':d['value'],'ms':d['ms_per_step'],'checked':d.get('proofs_checked')}))" "$line" $lib "$args" | tee -a $out
    done
  done
done
