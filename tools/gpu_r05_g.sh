#!/bin/bash
# Round 5 (g): small proofs (2^12 / 2^14) against the hardware-queue count and lane count:
# 16 lanes on 32 (default: 2 x lanes) / 16 / 8 queues, and 12 lanes on 24.
set -o pipefail
mkdir -p gpurun_out/r05g
timeout -k 10 1000 python -u tools/ab.py --out gpurun_out/r05g/ab.jsonl --reps 2 \
  --args "--log-n 12 --steps 40" --args "--log-n 12 --steps 40 --hw-queues 16" \
  --args "--log-n 12 --steps 40 --hw-queues 8" --args "--log-n 12 --steps 40 --lanes 12" \
  --args "--log-n 14 --steps 20" --args "--log-n 14 --steps 20 --hw-queues 16" \
  --args "--log-n 14 --steps 20 --hw-queues 8" --args "--log-n 14 --steps 20 --lanes 12" || exit 1
