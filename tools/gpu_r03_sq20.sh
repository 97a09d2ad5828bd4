#!/bin/bash
# Per-kernel SQ counters of one single-lane 2^20 proof (VALU instructions and busy cycles),
# to price the proof's VALU work against the multi-lane step time.
set -uo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/.."
O=gpurun_out/r03sq20
rm -rf $O; mkdir -p $O
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --lanes 1 > $O/bench.log 2>&1 || { echo PMC_FAILED; tail -20 $O/bench.log; exit 1; }
python3 tools/sq_summary.py $O/run_counter_collection.csv > $O/sq_summary.txt 2>&1
python3 - <<PY
import csv, collections
rows = list(csv.DictReader(open("$O/run_counter_collection.csv")))
tot = collections.Counter(); n = collections.Counter()
for r in rows:
    if r["Counter_Name"] == "SQ_INSTS_VALU":
        k = r["Kernel_Name"].split("(")[0].split("::")[-1]
        tot[k] += float(r["Counter_Value"]); n[k] += 1
print("SQ_INSTS_VALU by kernel (whole run: key compile + 3 proofs):")
for k, v in tot.most_common(20):
    print(f"  {k[:40]:40s} {n[k]:5d} {v:.4g}")
print("total", sum(tot.values()))
PY
echo done
