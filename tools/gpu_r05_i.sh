#!/bin/bash
# Round 5 (i): NTT tiles of 512 elements (PLK_NTT_MAX_LE=9: twice the workgroups, ~22 KiB of
# LDS each) against 1 024: NTT parity, then lone transforms and proofs, interleaved.
set -o pipefail
mkdir -p gpurun_out/r05i
timeout -k 10 1100 python -u tools/ab.py --out gpurun_out/r05i/ab.jsonl --reps 2 \
  --lib base=libplk.so --lib le9=libplk-le9.so --tests "tests/test_ntt_gpu.py" \
  --args "--mode ntt --log-n 20 --steps 50" --args "--mode ntt --log-n 23 --steps 10" \
  --args "--mode ntt --log-n 21 --steps 20" \
  --args "--log-n 12 --steps 40" --args "--log-n 16 --steps 10" --args "--log-n 20 --steps 5" || exit 1
