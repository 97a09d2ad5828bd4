# GPU cycle: all GPU tests, full-prover bench at 2^20, kernel-trace profile of the bench
set -o pipefail
mkdir -p gpurun_out/prof_full
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/tq.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/tq.log; exit 1; }
tail -1 gpurun_out/tq.log
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/full20.log 2>&1 || { echo FULL20_FAILED; tail -30 gpurun_out/full20.log; exit 1; }
grep metric gpurun_out/full20.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['breakdown_ms_per_step'], d['roofline']['avg_launch_ms'])"
rm -rf gpurun_out/prof_full/*
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_full -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --lanes 1 > gpurun_out/prof_full/bench.log 2>&1 || { echo PROF_FAILED; tail -20 gpurun_out/prof_full/bench.log; exit 1; }
python3 tools/trace_breakdown.py gpurun_out/prof_full/run_kernel_trace.csv
