#!/bin/bash
# Round 4: the lanes' size policy for the tail forms, default settings: prover-lane parity,
# then 2^12 / 2^14 / 2^16 proofs (no PLK_TAIL_QUAD).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_prover_lanes.py tests/test_prover_gpu.py tests/test_msm_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r04ah_tests.log 2>&1 || { tail -30 gpurun_out/r04ah_tests.log; exit 1; }
echo "tests: $(tail -n 1 gpurun_out/r04ah_tests.log)"
for r in 1 2; do
  for args in "--log-n 12 --steps 30" "--log-n 14 --steps 20" "--log-n 16 --steps 20"; do
    line=$(timeout -k 10 300 python bench.py $args --warmup 3 --no-cpu-baseline 2>>gpurun_out/r04ah.err) || exit 1
    python -c "import json,sys;d=json.loads(sys.argv[1]);print(json.dumps({'args':sys.argv[2],'value':d['value'],'checked':d.get('proofs_checked')}))" "$line" "$args" | tee -a gpurun_out/r04ah.jsonl
  done
done
