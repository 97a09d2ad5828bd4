set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_msm_gpu.py -x -v -p no:cacheprovider --timeout 300 > gpurun_out/msm_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/msm_tests.log; exit 1; }
grep -E "PASS|FAIL" gpurun_out/msm_tests.log | tail -30
