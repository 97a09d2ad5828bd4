#!/bin/bash
# Round 5 (q): (new) k_scan_buckets stages the bucket counts in LDS before its two walks;
# (scan4k) the same plus the grand-product scans in the 3-phase multi-workgroup form from
# n > 4096 instead of n > 32768 (2^13-2^15 proofs). MSM / prover parity, then interleaved
# proofs at 2^14 (x3), 2^13, 2^15 against the previous build.
set -o pipefail
mkdir -p gpurun_out/r05q
timeout -k 10 1100 python -u tools/ab.py --out gpurun_out/r05q/ab.jsonl --reps 3 \
  --lib prev=libplk-prev.so --lib new=libplk.so --lib scan4k=libplk-scan4k.so \
  --tests "tests/test_msm_gpu.py tests/test_prover_gpu.py" \
  --args "--log-n 14 --steps 20" --args "--log-n 13 --steps 30" --args "--log-n 15 --steps 15" || exit 1
