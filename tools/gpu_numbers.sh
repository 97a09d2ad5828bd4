# headline numbers: default bench (2^20 full prover + CPU baseline), 2^16 full prover,
# 2^20 hot-path mode
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python bench.py > gpurun_out/b20.log 2>&1 || { echo B20_FAILED; tail -30 gpurun_out/b20.log; exit 1; }
grep metric gpurun_out/b20.log
timeout -k 10 600 python bench.py --log-n 16 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/b16.log 2>&1 || { echo B16_FAILED; tail -30 gpurun_out/b16.log; exit 1; }
grep metric gpurun_out/b16.log
timeout -k 10 600 python bench.py --mode hotpath --no-cpu-baseline > gpurun_out/bhot.log 2>&1 || { echo BHOT_FAILED; tail -30 gpurun_out/bhot.log; exit 1; }
grep metric gpurun_out/bhot.log
