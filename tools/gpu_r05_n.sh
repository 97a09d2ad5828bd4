#!/bin/bash
# Round 5 (n): hardware queues at the large sizes — 2^20 with 12 lanes on 24 (default) / 32
# queues and 14 / 16 lanes on 32; 2^16 with 14 lanes on 28 (default) / 32 and 16 lanes on 32.
set -o pipefail
mkdir -p gpurun_out/r05n
timeout -k 10 1100 python -u tools/ab.py --out gpurun_out/r05n/ab.jsonl --reps 2 \
  --args "--log-n 20 --steps 6" --args "--log-n 20 --steps 6 --hw-queues 32" \
  --args "--log-n 20 --steps 6 --lanes 14 --hw-queues 32" --args "--log-n 20 --steps 6 --lanes 16 --hw-queues 32" \
  --args "--log-n 16 --steps 10" --args "--log-n 16 --steps 10 --hw-queues 32" \
  --args "--log-n 16 --steps 10 --lanes 16 --hw-queues 32" || exit 1
