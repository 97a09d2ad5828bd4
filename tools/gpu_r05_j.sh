#!/bin/bash
# Round 5 (j): (new) sort passes with loads issued ahead — k_hist / k_scatter / k_chist /
# k_cscatter load 4 scalars per thread before processing the first — and the MSM readback
# record / round-4 evaluations written by the kernels into mapped host memory (no copy
# dispatch); (f8) the same with 8 entries in flight per k_fine thread instead of 4; against
# the previous build: full -m gpu suite on new, MSM / prover parity on f8, then interleaved
# lone MSMs, the 8-part split and proofs.
set -o pipefail
mkdir -p gpurun_out/r05j
PLK_LIB=$PWD/dusk-plonk_amd/libplk.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/r05j/tests_new_full.log 2>&1 \
  || { tail -n 30 gpurun_out/r05j/tests_new_full.log; exit 1; }
tail -n 1 gpurun_out/r05j/tests_new_full.log
timeout -k 10 1000 python -u tools/ab.py --out gpurun_out/r05j/ab.jsonl --reps 2 \
  --lib prev=libplk-prev.so --lib new=libplk.so --lib f8=libplk-f8.so \
  --args "--mode msm --log-n 20 --steps 30" --args "--mode msm --log-n 16 --steps 50" \
  --args "--mode msm --log-n 20 --steps 10 --bucket-parts 8" \
  --args "--log-n 12 --steps 40" --args "--log-n 20 --steps 5" || exit 1
