#!/bin/bash
# Round 5 (p): k_sort_one over several workgroups per slot by bucket range (each histograms all
# digits, then writes the task records and scatters only its own range): 4 (new) / 8 (so8)
# workgroups against one (prev). MSM / prover parity on both, then interleaved small proofs
# and the lone 2^12 MSM.
set -o pipefail
mkdir -p gpurun_out/r05p
timeout -k 10 1100 python -u tools/ab.py --out gpurun_out/r05p/ab.jsonl --reps 3 \
  --lib prev=libplk-prev.so --lib new=libplk.so --lib so8=libplk-so8.so \
  --tests "tests/test_msm_gpu.py tests/test_prover_gpu.py tests/test_prover_lanes.py" \
  --args "--log-n 12 --steps 40" --args "--log-n 13 --steps 30" \
  --args "--mode msm --log-n 12 --steps 100" || exit 1
