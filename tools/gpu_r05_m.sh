#!/bin/bash
# Round 5 (m): a plain idft's n^-1 folded into the last pass' inter-pass twiddle table
# (pass_tw_inv_last) instead of a product per output: NTT / prover / opening parity, then
# interleaved lone transforms and proofs against the previous build.
set -o pipefail
mkdir -p gpurun_out/r05m
timeout -k 10 1100 python -u tools/ab.py --out gpurun_out/r05m/ab.jsonl --reps 3 \
  --lib prev=libplk-prev.so --lib new=libplk.so \
  --tests "tests/test_ntt_gpu.py tests/test_prover_gpu.py tests/test_opening_gpu.py tests/test_abi.py" \
  --args "--mode ntt --log-n 20 --steps 50" --args "--mode ntt --log-n 23 --steps 10" \
  --args "--log-n 14 --steps 20" --args "--log-n 20 --steps 5" || exit 1
