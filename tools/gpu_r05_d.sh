#!/bin/bash
# Round 5 (d): small proofs, balanced windows (libplk.so) against round 4's short top window
# (libplk-prev.so), four interleaved repetitions at 2^12 / 2^13; then the prover lanes' tail
# form at the sizes the round-4 policy had no measurement for (2^15, 2^17, 2^18: PLK_TAIL_QUAD
# 0 / 1 / 2 forced on every workspace).
set -o pipefail
mkdir -p gpurun_out/r05d
timeout -k 10 700 python -u tools/ab.py --out gpurun_out/r05d/small_ab.jsonl --reps 4 \
  --lib prev=libplk-prev.so --lib new=libplk.so \
  --args "--log-n 12 --steps 40" --args "--log-n 13 --steps 30" || exit 1
timeout -k 10 900 python -u tools/ab.py --out gpurun_out/r05d/tail_ab.jsonl --reps 2 \
  --venv q0=PLK_TAIL_QUAD=0 --venv q1=PLK_TAIL_QUAD=1 --venv q2=PLK_TAIL_QUAD=2 \
  --args "--log-n 15 --steps 15" --args "--log-n 17 --steps 8" --args "--log-n 18 --steps 6" || exit 1
