#!/bin/bash
# SQ issue/stall counters per kernel of lone MSMs (bench.py --mode msm, 2^20 and 2^16; one
# --pmc pass each, kernel trace only): what the latency-bound reduction tail waits on.
set -o pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/.."
d=gpurun_out/sqmsm
rm -rf $d; mkdir -p $d
for k in 20 16; do
  timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $d/m$k -o run -- python3 bench.py --mode msm --log-n $k --steps 3 --warmup 1 --no-cpu-baseline > $d/m$k.log 2>&1 || { echo PMC_FAILED $k; tail -20 $d/m$k.log; exit 1; }
  echo "== lone MSM 2^$k"
  python3 tools/sq_summary.py $d/m$k/run_counter_collection.csv | tee $d/summary$k.txt
done
