# k_accumulate timing: bench HIP events vs rocprofv3 kernel trace of the same default run
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_msm_gpu.py -x -q -p no:cacheprovider --timeout 200 > gpurun_out/m.log 2>&1 || { echo TESTS_FAILED; tail -20 gpurun_out/m.log; exit 1; }
tail -1 gpurun_out/m.log
rm -rf gpurun_out/pchk
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pchk -o run -- python3 bench.py --no-cpu-baseline > gpurun_out/pchk.log 2>&1 || { echo PROF_FAILED; tail -20 gpurun_out/pchk.log; exit 1; }
python3 tools/acc_timing_check.py gpurun_out/pchk/run_kernel_trace.csv gpurun_out/pchk.log
