#!/bin/bash
# Round 5 (w): the lane tail form (PLK_TAIL_QUAD 0 / 1 / 2) at 2^13 and 2^14 now that those
# sizes take c = 12 / 13 (lane_tail_policy was measured with c = 10 / 15).
set -o pipefail
mkdir -p gpurun_out/r05w
timeout -k 10 1000 python -u tools/ab.py --out gpurun_out/r05w/ab.jsonl --reps 3 \
  --venv t0=PLK_TAIL_QUAD=0 --venv t1=PLK_TAIL_QUAD=1 --venv t2=PLK_TAIL_QUAD=2 \
  --args "--log-n 14 --steps 20" --args "--log-n 13 --steps 30" || exit 1
