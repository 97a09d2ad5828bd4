#!/bin/bash
# Round 5 (e): sort kernels with the window layout as a compile-time constant (each_digit<C>:
# unrolled funnel-shift digits for c = 10 / 15 / 17 / 20) against the previous build: MSM and
# prover parity, then interleaved proofs at 2^12 / 2^14 / 2^16 / 2^20, the lone 2^20 MSM and
# the 8-part split.
set -o pipefail
mkdir -p gpurun_out/r05e
timeout -k 10 1100 python -u tools/ab.py --out gpurun_out/r05e/ab.jsonl --reps 3 \
  --lib prev=libplk-prev.so --lib new=libplk.so \
  --tests "tests/test_msm_gpu.py tests/test_prover_gpu.py" \
  --args "--log-n 12 --steps 40" --args "--log-n 14 --steps 20" --args "--log-n 16 --steps 10" \
  --args "--mode msm --log-n 20 --steps 30" --args "--mode msm --log-n 20 --steps 10 --bucket-parts 8" \
  --args "--log-n 20 --steps 5" || exit 1
