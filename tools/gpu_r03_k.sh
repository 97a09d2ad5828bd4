#!/bin/bash
# 2^20 study on the current code: single-lane proof breakdown and default 8-lane kernel shares
# (kernel trace), the rocprofv3 --stats summary of the default bench command, and the
# configs[1] / [2] standalone lines with their CPU baselines.
set -uo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/.."
O=gpurun_out/r03k
rm -rf $O; mkdir -p $O
k=20
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/one -o run -- python3 bench.py --log-n $k --steps 2 --warmup 1 --no-cpu-baseline --lanes 1 > $O/one.log 2>&1 || { echo PROF1_FAILED; tail -20 $O/one.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/many -o run -- python3 bench.py --log-n $k --steps 6 --warmup 2 --no-cpu-baseline > $O/many.log 2>&1 || { echo PROF2_FAILED; tail -20 $O/many.log; exit 1; }
python3 tools/small_trace.py $O/one/run_kernel_trace.csv $O/many/run_kernel_trace.csv > $O/summary.txt 2>&1
cat $O/summary.txt
grep '"metric"' $O/many.log | cut -c1-200
for m in ntt msm; do
  timeout -k 10 400 python3 -u bench.py --mode $m --steps 20 --warmup 3 > $O/$m.log 2>&1 || { echo MODE_FAILED $m; tail -20 $O/$m.log; exit 1; }
  grep '"metric"' $O/$m.log > $O/$m.json
  python3 -c "
import json; d=json.load(open('$O/$m.json')); r=d['roofline']
print('$m', round(d['value']/1e9,3), 'G points/s', round(d['ms_per_step'],4), 'ms/step', 'frac', round(r['frac'],4), 'exact', d.get('bit_exact_vs_oracle'), 'cpu', round(d['cpu_baseline']['value']/1e6,3), 'M/s')"
done
echo done
