set -e
mkdir -p gpurun_out/r06a
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_bench.py tests/test_ntt_gpu.py -m gpu -k "extras or msm_curve or identity_rows or kernel_mode or msm_split or world2" > gpurun_out/r06a/tests.log 2>&1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r06a/bench.log 2>&1
