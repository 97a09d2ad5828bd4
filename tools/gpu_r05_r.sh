#!/bin/bash
# Round 5 (r): k_runsum2 at 2 waves per SIMD (256 VGPRs, 3 registers spilled around the loop,
# none inside it) against 1 (256 VGPRs + 3 AGPRs): MSM / prover parity, then interleaved lone
# MSMs, the 8-part split and proofs.
set -o pipefail
mkdir -p gpurun_out/r05r
timeout -k 10 1100 python -u tools/ab.py --out gpurun_out/r05r/ab.jsonl --reps 3 \
  --lib prev=libplk-prev.so --lib new=libplk.so \
  --tests "tests/test_msm_gpu.py tests/test_prover_gpu.py" \
  --args "--mode msm --log-n 20 --steps 30" --args "--mode msm --log-n 20 --steps 10 --bucket-parts 8" \
  --args "--log-n 16 --steps 10" --args "--log-n 20 --steps 5" || exit 1
