#!/bin/bash
# Round-4 final evidence, part B: BASELINE configs[1] / [2] lines with kernel traces and PMC
# passes (tools/gpu_configs.sh), then the size sweep 2^12..2^20 (tools/gpu_size_sweep.sh).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/final
bash tools/gpu_configs.sh > gpurun_out/final/configs.log 2>&1 || { echo CONFIGS_FAILED; tail -30 gpurun_out/final/configs.log; exit 1; }
grep -h '"metric"' gpurun_out/configs/bench_*.json | cut -c1-160
bash tools/gpu_size_sweep.sh 2>&1 | tee gpurun_out/final/sizes.txt
