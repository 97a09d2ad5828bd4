#!/bin/bash
# 2^16 multi-lane study: kernel trace of the default-lane bench (busy, concurrency, kernel
# shares) and a lane sweep at 32 hardware queues.
set -uo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/.."
O=gpurun_out/r03mid
rm -rf $O; mkdir -p $O
k=16
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/one -o run -- python3 bench.py --log-n $k --steps 3 --warmup 1 --no-cpu-baseline --lanes 1 > $O/one.log 2>&1 || { echo PROF1_FAILED; tail -20 $O/one.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/many -o run -- python3 bench.py --log-n $k --steps 12 --warmup 3 --no-cpu-baseline > $O/many.log 2>&1 || { echo PROF2_FAILED; tail -20 $O/many.log; exit 1; }
python3 tools/small_trace.py $O/one/run_kernel_trace.csv $O/many/run_kernel_trace.csv > $O/summary.txt 2>&1
cat $O/summary.txt
for L in 8 12 16 24 32; do
  timeout -k 10 200 python3 bench.py --log-n $k --steps 16 --warmup 3 --no-cpu-baseline --lanes $L --hw-queues 32 > $O/lanes$L.log 2>&1 || { echo LANES_FAILED $L; tail -20 $O/lanes$L.log; exit 1; }
  echo -n "lanes $L: "; grep '"metric"' $O/lanes$L.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,3), "M/s")'
done
echo done
