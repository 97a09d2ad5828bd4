#!/bin/bash
# Small-proof study: bench lines at 2^12 / 2^14, kernel traces at 2^12
# (one lane: per-proof dispatch list; default lanes: busy fraction, concurrency, kernel shares)
# and one SQ PMC pass (single lane, VALU instructions per proof).
set -uo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/.."
O=gpurun_out/r03small
rm -rf $O; mkdir -p $O
for k in 12 14; do
  timeout -k 10 200 python3 -u bench.py --log-n $k --steps 20 --warmup 3 --no-cpu-baseline > $O/bench$k.log 2>&1 || { echo BENCH_FAILED; tail -20 $O/bench$k.log; exit 1; }
  grep '"metric"' $O/bench$k.log | cut -c1-160
done
k=12
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/one -o run -- python3 bench.py --log-n $k --steps 3 --warmup 1 --no-cpu-baseline --lanes 1 > $O/one.log 2>&1 || { echo PROF1_FAILED; tail -20 $O/one.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/many -o run -- python3 bench.py --log-n $k --steps 20 --warmup 3 --no-cpu-baseline > $O/many.log 2>&1 || { echo PROF2_FAILED; tail -20 $O/many.log; exit 1; }
python3 tools/small_trace.py $O/one/run_kernel_trace.csv $O/many/run_kernel_trace.csv > $O/summary.txt 2>&1
cat $O/summary.txt
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/sq -o run -- python3 bench.py --log-n $k --steps 2 --warmup 1 --no-cpu-baseline --lanes 1 > $O/sq.log 2>&1 || { echo PMC_FAILED; tail -20 $O/sq.log; exit 1; }
python3 tools/sq_summary.py $O/sq/run_counter_collection.csv > $O/sq_summary.txt 2>&1
python3 - <<PY
import csv
tot = 0.0
rows = list(csv.DictReader(open("$O/sq/run_counter_collection.csv")))
ids = sorted({int(r["Dispatch_Id"]) for r in rows})
for r in rows:
    if r["Counter_Name"] == "SQ_INSTS_VALU":
        tot += float(r["Counter_Value"])
print(f"SQ_INSTS_VALU over the run: {tot:.4g} in {len(ids)} dispatches")
PY
echo done
