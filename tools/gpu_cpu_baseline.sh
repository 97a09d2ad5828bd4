#!/bin/bash
# The restated reference CPU prover timed directly at 2^20 on the GPU box's host cores
# (OMP_NUM_THREADS as the box sets it: the CPU share of one GPU), no extrapolation.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/cpu
timeout -k 10 1000 python3 -u tools/cpu_full_proof.py --log-n 20 > gpurun_out/cpu/cpu_full_n20.json 2> gpurun_out/cpu/cpu_full_n20.err || { tail -5 gpurun_out/cpu/cpu_full_n20.err; exit 1; }
cat gpurun_out/cpu/cpu_full_n20.json
