#!/bin/bash
# Round 5 (y): SQ issue / stall counters on the final code (one --pmc pass each, kernel trace
# only; 7 SQ + 1 GRBM counters): a single-lane 2^20 proof and the lone 2^20 MSM.
set -o pipefail
export TMPDIR=/tmp
C="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE"
d=gpurun_out/r05y
rm -rf $d; mkdir -p $d/proof $d/msm
timeout -s KILL 240 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $d/proof -o run -- \
  python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --lanes 1 > $d/proof/bench.log 2>&1 || { tail -20 $d/proof/bench.log; exit 1; }
python3 tools/sq_summary.py $d/proof/run_counter_collection.csv > $d/sq_proof.txt
timeout -s KILL 240 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $d/msm -o run -- \
  python3 bench.py --mode msm --log-n 20 --steps 5 --warmup 1 --no-cpu-baseline > $d/msm/bench.log 2>&1 || { tail -20 $d/msm/bench.log; exit 1; }
python3 tools/sq_summary.py $d/msm/run_counter_collection.csv > $d/sq_msm.txt
head -12 $d/sq_proof.txt
head -8 $d/sq_msm.txt
