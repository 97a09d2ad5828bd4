#!/bin/bash
# Round 4: lone-wave latency of the quad addition with 1 / 2 / 4 accumulator chains per product
# column (tools/ubench_quad.hip), twice.
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do for v in 0 2 4; do timeout -k 10 60 ./tools/ubench_quad$v || exit 1; done; done 2>&1 | tee gpurun_out/r04ab_ubench_quad.txt
