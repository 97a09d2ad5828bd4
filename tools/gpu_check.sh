set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/t2.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/t2.log; exit 1; }
tail -3 gpurun_out/t2.log
timeout -k 10 120 ./tools/ubench > gpurun_out/ubench.log 2>&1 || { echo UBENCH_FAILED; cat gpurun_out/ubench.log; exit 1; }
cat gpurun_out/ubench.log
timeout -k 10 300 python bench.py --log-n 16 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench16.log 2>&1 || { echo BENCH16_FAILED; tail -30 gpurun_out/bench16.log; exit 1; }
tail -2 gpurun_out/bench16.log
timeout -k 10 400 python bench.py > gpurun_out/bench20.log 2>&1 || { echo BENCH20_FAILED; tail -30 gpurun_out/bench20.log; exit 1; }
tail -2 gpurun_out/bench20.log
