#!/bin/bash
# Round 5 (aa): workgroups per slot of the one-dispatch sort in its big mode (the 2^14-size
# commits at c = 13, scalars read twice): 4 (default) / 8 / 16; MSM parity on the variants,
# then interleaved 2^14 proofs (x3).
set -o pipefail
mkdir -p gpurun_out/r05aa
timeout -k 10 1100 python -u tools/ab.py --out gpurun_out/r05aa/ab.jsonl --reps 3 \
  --lib p4=libplk.so --lib p8=libplk-bp8.so --lib p16=libplk-bp16.so \
  --tests "tests/test_msm_gpu.py -k narrow_balanced" \
  --args "--log-n 14 --steps 20" || exit 1
