#!/bin/bash
# Round 5 (h): k_ntt_pass without its 76-B scratch object (r4_math templated on h == 1) and
# the scratch-free k_ruffini_single, against the previous build: NTT / prover / opening
# parity, then interleaved lone transforms (2^20, 2^23) and proofs (2^12, 2^14, 2^16, 2^20).
set -o pipefail
mkdir -p gpurun_out/r05h
timeout -k 10 1100 python -u tools/ab.py --out gpurun_out/r05h/ab.jsonl --reps 2 \
  --lib prev=libplk-prev.so --lib new=libplk.so \
  --tests "tests/test_ntt_gpu.py tests/test_prover_gpu.py tests/test_opening_gpu.py" \
  --args "--mode ntt --log-n 20 --steps 50" --args "--mode ntt --log-n 23 --steps 10" \
  --args "--log-n 12 --steps 40" --args "--log-n 14 --steps 20" --args "--log-n 16 --steps 10" \
  --args "--log-n 20 --steps 5" || exit 1
