#!/bin/bash
# Round 5 (t): window sizes for small proofs now that the windows are balanced (round 4's
# c = 11 / 12 / 14 lost to a 1-3-bit top window holding hot buckets): 2^12 proofs at
# c = 10 (default) / 11 / 12 / 13, 2^14 at c = 13 / 14 / 15 (default), via PLK_MSM_C.
set -o pipefail
mkdir -p gpurun_out/r05t
timeout -k 10 1100 python -u tools/ab.py --out gpurun_out/r05t/ab.jsonl --reps 2 \
  --venv c10=PLK_MSM_C=10 --venv c11=PLK_MSM_C=11 --venv c12=PLK_MSM_C=12 --venv c13=PLK_MSM_C=13 \
  --args "--log-n 12 --steps 40" || exit 1
timeout -k 10 900 python -u tools/ab.py --out gpurun_out/r05t/ab14.jsonl --reps 2 \
  --venv c13=PLK_MSM_C=13 --venv c14=PLK_MSM_C=14 --venv c15=PLK_MSM_C=15 \
  --args "--log-n 14 --steps 20" || exit 1
