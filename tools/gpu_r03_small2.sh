#!/bin/bash
# The opt-in NTT plans' parity test, then a 2^12 single-lane dispatch list and the multi-lane
# summary (tools/small_trace.py) on the current code.
set -uo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/.."
O=gpurun_out/r03small2
rm -rf $O; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_ntt_gpu.py -k opt_in > $O/pytest.log 2>&1 || { echo PYTEST_FAILED; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
k=12
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/one -o run -- python3 bench.py --log-n $k --steps 3 --warmup 1 --no-cpu-baseline --lanes 1 > $O/one.log 2>&1 || { echo PROF1_FAILED; tail -20 $O/one.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/many -o run -- python3 bench.py --log-n $k --steps 20 --warmup 3 --no-cpu-baseline > $O/many.log 2>&1 || { echo PROF2_FAILED; tail -20 $O/many.log; exit 1; }
python3 tools/small_trace.py $O/one/run_kernel_trace.csv $O/many/run_kernel_trace.csv > $O/summary.txt 2>&1
cat $O/summary.txt
echo done
