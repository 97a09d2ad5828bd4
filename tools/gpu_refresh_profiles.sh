# Refresh the committed rocprof evidence for the current code: the default bench command
# under --kernel-trace --stats, one PMC pass per counter, and a single-lane proof breakdown.
set -o pipefail
bash tools/gpu_pmc.sh || exit 1
mkdir -p gpurun_out/prof_full
rm -rf gpurun_out/prof_full/*
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_full -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --lanes 1 > gpurun_out/prof_full/bench.log 2>&1 || { echo PROF_FAILED; tail -20 gpurun_out/prof_full/bench.log; exit 1; }
python3 tools/trace_breakdown.py gpurun_out/prof_full/run_kernel_trace.csv > gpurun_out/prof_full/breakdown.txt
cat gpurun_out/prof_full/breakdown.txt
grep -h '"metric"' gpurun_out/prof/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"
