#!/bin/bash
# Lone-MSM kernel breakdown (bench.py --mode msm, 2^20 and 2^16) from a kernel trace.
set -uo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/.."
O=gpurun_out/r03msm
rm -rf $O; mkdir -p $O
for k in 20 16; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/t$k -o run -- python3 bench.py --mode msm --log-n $k --steps 12 --warmup 3 --no-cpu-baseline > $O/b$k.log 2>&1 || { echo PROF_FAILED $k; tail -20 $O/b$k.log; exit 1; }
  echo "== 2^$k"; grep -o '"ms_per_step": [0-9.]*' $O/b$k.log
  python3 tools/msm_trace.py $O/t$k/run_kernel_trace.csv 8 | tee $O/summary$k.txt
done
echo done
