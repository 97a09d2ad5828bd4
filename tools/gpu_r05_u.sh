#!/bin/bash
# Round 5 (u): window sizes with balanced windows, confirmation — 2^14 and 2^15 proofs at
# c = 13 / 14 / 15 (default), 2^13 at c = 10 (default) / 12 / 13, 2^16 at c = 15 / 16 / 17
# (default); three interleaved runs each (PLK_MSM_C).
set -o pipefail
mkdir -p gpurun_out/r05u
timeout -k 10 700 python -u tools/ab.py --out gpurun_out/r05u/ab.jsonl --reps 3 \
  --venv c13=PLK_MSM_C=13 --venv c14=PLK_MSM_C=14 --venv c15=PLK_MSM_C=15 \
  --args "--log-n 14 --steps 20" --args "--log-n 15 --steps 15" || exit 1
timeout -k 10 400 python -u tools/ab.py --out gpurun_out/r05u/ab13.jsonl --reps 3 \
  --venv c10=PLK_MSM_C=10 --venv c12=PLK_MSM_C=12 --venv c13=PLK_MSM_C=13 \
  --args "--log-n 13 --steps 30" || exit 1
timeout -k 10 500 python -u tools/ab.py --out gpurun_out/r05u/ab16.jsonl --reps 2 \
  --venv c15=PLK_MSM_C=15 --venv c16=PLK_MSM_C=16 --venv c17=PLK_MSM_C=17 \
  --args "--log-n 16 --steps 10" || exit 1
