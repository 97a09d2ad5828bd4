#!/bin/bash
# Round 5 (x): (new) the one-dispatch sort for up to 32 K scalars per slot (the 2^14-size
# commits at c = 13: k_sort_one with both passes reading the scalars, 4 workgroups per slot)
# plus compile-time digit layouts for c = 12 / 13; (nobig) the digit layouts only; against
# the previous build. MSM / prover parity, then interleaved proofs at 2^14 (x3), 2^13, 2^12.
set -o pipefail
mkdir -p gpurun_out/r05x
timeout -k 10 1100 python -u tools/ab.py --out gpurun_out/r05x/ab.jsonl --reps 3 \
  --lib prev=libplk-prev.so --lib new=libplk.so --lib nobig=libplk-nobig.so \
  --tests "tests/test_msm_gpu.py tests/test_prover_gpu.py tests/test_prover_oracle.py" \
  --args "--log-n 14 --steps 20" --args "--log-n 13 --steps 30" --args "--log-n 12 --steps 40" || exit 1
