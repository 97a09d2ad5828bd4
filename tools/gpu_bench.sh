set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --log-n 16 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/full16.log 2>&1 || { echo FULL16_FAILED; tail -30 gpurun_out/full16.log; exit 1; }
grep metric gpurun_out/full16.log
timeout -k 10 600 python bench.py > gpurun_out/full20.log 2>&1 || { echo FULL20_FAILED; tail -30 gpurun_out/full20.log; exit 1; }
grep metric gpurun_out/full20.log
