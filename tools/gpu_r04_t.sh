#!/bin/bash
# Round 4: lone-wave latency of the lazy full addition, grouped products (default) against
# the plain chains (PLK_MADD_GROUPED=0), tools/ubench_tail.hip.
set -o pipefail
mkdir -p gpurun_out
for v in g1 g0 g1 g0; do echo "== $v"; timeout -k 10 120 ./tools/ubench_tail_$v || exit 1; done 2>&1 | tee gpurun_out/r04t_ubench_tail.txt
