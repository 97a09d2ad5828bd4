#!/bin/bash
# Round 4: small-proof traces at 2^12 and 2^14 on the current code (quad tails, spread top
# window), tools/gpu_small_trace.sh twice.
set -o pipefail
mkdir -p gpurun_out
for k in 12 14; do
  LOGN=$k bash tools/gpu_small_trace.sh > /dev/null 2>&1 || { echo TRACE_FAILED $k; exit 1; }
  cp gpurun_out/small/summary.txt gpurun_out/r04v_small_$k.txt
  echo "== 2^$k"; head -60 gpurun_out/r04v_small_$k.txt
done
