#!/bin/bash
# Round 5 (v): choose_c takes c = 12 at 2^13 and c = 13 at 2^14 SRS points (balanced windows):
# the new narrow-window and small bench-proof parity tests, the MSM / prover suites, then
# interleaved proofs at 2^12 .. 2^16 against the previous build.
set -o pipefail
mkdir -p gpurun_out/r05v
timeout -k 10 600 python -u -m pytest tests/test_msm_gpu.py tests/test_prover_oracle.py tests/test_prover_gpu.py \
  -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05v/tests.log 2>&1 \
  || { tail -n 30 gpurun_out/r05v/tests.log; exit 1; }
tail -n 1 gpurun_out/r05v/tests.log
timeout -k 10 900 python -u tools/ab.py --out gpurun_out/r05v/ab.jsonl --reps 3 \
  --lib prev=libplk-prev.so --lib new=libplk.so \
  --args "--log-n 13 --steps 30" --args "--log-n 14 --steps 20" --args "--log-n 12 --steps 40" \
  --args "--log-n 15 --steps 15" || exit 1
