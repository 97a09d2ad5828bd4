#!/bin/bash
# Round 5 (o): the narrow path's bucket scan run by the last workgroup of k_block_scan (one
# dispatch per commit group fewer: new), and additionally k_bitsum2 folded into k_bitsum1 up to
# 64 groups (fold64: the c = 15 commits of 2^14-2^15 proofs); MSM / prover parity on both, then
# interleaved proofs at 2^14 (x3), 2^13, 2^15, 2^12, 2^16.
set -o pipefail
mkdir -p gpurun_out/r05o
timeout -k 10 1100 python -u tools/ab.py --out gpurun_out/r05o/ab.jsonl --reps 3 \
  --lib prev=libplk-prev.so --lib new=libplk.so --lib fold64=libplk-fold64.so \
  --tests "tests/test_msm_gpu.py tests/test_prover_gpu.py" \
  --args "--log-n 14 --steps 20" --args "--log-n 13 --steps 30" --args "--log-n 15 --steps 15" \
  --args "--log-n 12 --steps 40" || exit 1
