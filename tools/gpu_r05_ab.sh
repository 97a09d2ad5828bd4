#!/bin/bash
# Round 5 (ab): SQ issue counters and the effective clock of the lone NTT (bench.py --mode ntt
# at 2^20 and 2^23), one --pmc pass each (7 SQ + 1 GRBM counters, kernel trace only).
set -o pipefail
export TMPDIR=/tmp
C="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE"
d=gpurun_out/r05ab
rm -rf $d; mkdir -p $d/n20 $d/n23
for k in 20 23; do
  timeout -s KILL 240 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $d/n$k -o run -- \
    python3 bench.py --mode ntt --log-n $k --steps 10 --warmup 2 --no-cpu-baseline > $d/n$k/bench.log 2>&1 || { tail -20 $d/n$k/bench.log; exit 1; }
  python3 tools/sq_summary.py $d/n$k/run_counter_collection.csv > $d/sq_ntt$k.txt
  python3 tools/effective_clock.py $d/n$k/run_counter_collection.csv --min-ms 0.05 > $d/clock_ntt$k.txt
  cat $d/clock_ntt$k.txt
done
