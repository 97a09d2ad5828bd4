#!/bin/bash
# Round 4: lone-MSM kernel breakdown with the quad tails (rocprofv3 kernel trace ->
# tools/msm_trace.py), then the run-lane sweep again (the bit sums got cheaper).
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r04r
rm -rf $O; mkdir -p $O
for k in 20 16; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/t$k -o run -- python3 bench.py --mode msm --log-n $k --steps 12 --warmup 3 --no-cpu-baseline > $O/m$k.log 2>&1 || { echo PROF_FAILED $k; tail -20 $O/m$k.log; exit 1; }
  echo "== lone MSM 2^$k"; grep -o '"ms_per_step": [0-9.]*' $O/m$k.log
  python3 tools/msm_trace.py $O/t$k/run_kernel_trace.csv 8 | tee $O/msm_summary$k.txt
done
for r in 1 2; do
  for L in 65536 131072 262144; do
    for k in 20 16; do
      line=$(PLK_RUN_LANES=$L timeout -k 10 200 python3 bench.py --mode msm --log-n $k --steps 30 --warmup 3 --no-cpu-baseline 2>>$O/sweep.err) || exit 1
      python3 -c "import json,sys;d=json.loads(sys.argv[1]);print('2^$k run_lanes=$L', round(d['ms_per_step'],4), 'ms')" "$line" | tee -a $O/runlanes.txt
    done
  done
done
