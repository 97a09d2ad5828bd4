#!/bin/bash
# rocprofv3 evidence for the current code (one GPU call):
#  1. the default bench command (2^20, default lanes) under --kernel-trace --stats
#  2. one PMC pass per counter (FETCH_SIZE, WRITE_SIZE) of the same command, --kernel-trace
#     only (no sys/runtime trace domains with --pmc), summarised per kernel
#  3. single-lane proof breakdowns (last proof's kernel window) at 2^20 and 2^16
# usage: bash tools/gpu_profile.sh   -> gpurun_out/prof/ ; tools/save_profiles.sh <tag> copies
set -o pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/.."
O=gpurun_out/prof
rm -rf $O; mkdir -p $O/stats $O/pmc $O/bd20 $O/bd16
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python3 bench.py --no-cpu-baseline > $O/stats/bench.log 2>&1 || { echo PROF_FAILED; tail -30 $O/stats/bench.log; exit 1; }
grep '"metric"' $O/stats/bench.log > $O/bench_line.json
python3 -c "import json; d=json.load(open('$O/bench_line.json')); r=d['roofline']; print('bench', round(d['value']/1e6,3), 'M/s; k_accumulate solo', round(r['avg_launch_ms'],3), 'ms, binding', r['bound'], round(r['frac'],3))"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 600 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/pmc/$c -o run -- python3 bench.py --no-cpu-baseline > $O/pmc/$c.log 2>&1 || { echo PMC_FAILED $c; tail -20 $O/pmc/$c.log; exit 1; }
done
python3 tools/pmc_summary.py $O/pmc $O/pmc_traffic.json
for k in 20 16; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/bd$k -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --lanes 1 --log-n $k > $O/bd$k/bench.log 2>&1 || { echo BD_FAILED $k; tail -20 $O/bd$k/bench.log; exit 1; }
  python3 tools/trace_breakdown.py $O/bd$k/run_kernel_trace.csv > $O/bd$k/breakdown.txt
  echo "== 2^$k single lane"; head -14 $O/bd$k/breakdown.txt
done
echo done
