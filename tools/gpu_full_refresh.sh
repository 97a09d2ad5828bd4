# all GPU tests, then the committed rocprof evidence refresh (tools/gpu_refresh_profiles.sh)
# and the single-lane 2^16 breakdown
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 > gpurun_out/tq.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/tq.log; exit 1; }
tail -1 gpurun_out/tq.log
bash tools/gpu_refresh_profiles.sh || exit 1
d=gpurun_out/prof16; rm -rf $d; mkdir -p $d
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $d -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --lanes 1 --log-n 16 > $d/bench.log 2>&1 || { echo PROF16_FAILED; tail -20 $d/bench.log; exit 1; }
python3 tools/trace_breakdown.py $d/run_kernel_trace.csv > $d/breakdown.txt; head -12 $d/breakdown.txt
timeout -k 10 300 python bench.py --log-n 16 > $d/bench16_line.log 2>&1 || { echo BENCH16_FAILED; tail -20 $d/bench16_line.log; exit 1; }
grep '"metric"' $d/bench16_line.log > $d/bench16_line.json; cat $d/bench16_line.json | cut -c1-300
