#!/bin/bash
# Round 5 (s): the prover-lane k_accumulate form with plain product chains at 2 waves per SIMD
# (d2g0, 173 VGPRs) against the grouped products at 2 (prev): MSM / prover parity, then
# interleaved proofs at 2^20 (x3), 2^18, 2^16.
set -o pipefail
mkdir -p gpurun_out/r05s
timeout -k 10 1100 python -u tools/ab.py --out gpurun_out/r05s/ab.jsonl --reps 3 \
  --lib prev=libplk-prev.so --lib d2g0=libplk-d2g0.so \
  --tests "tests/test_msm_gpu.py tests/test_prover_gpu.py" \
  --args "--log-n 20 --steps 6" --args "--log-n 18 --steps 8" --args "--log-n 16 --steps 10" || exit 1
