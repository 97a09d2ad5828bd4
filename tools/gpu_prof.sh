set -o pipefail
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof/bench.log 2>&1 || { echo PROF_FAILED; tail -30 gpurun_out/prof/bench.log; exit 1; }
tail -1 gpurun_out/prof/bench.log
find gpurun_out/prof -name "*stats*" | head
