set -o pipefail
mkdir -p gpurun_out/sweep
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests/test_prover_oracle.py tests/test_prover_gpu.py tests/test_msm_gpu.py -x -q -p no:cacheprovider > gpurun_out/sweep/tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/sweep/tests.log; exit 1; }
tail -1 gpurun_out/sweep/tests.log
# (the PLK_HIST_BLOCKS override this sweep used was removed after the measurement)
for hb in 256 128 64 32; do
  rm -rf gpurun_out/sweep/p$hb
  PLK_HIST_BLOCKS=$hb timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/sweep/p$hb -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/sweep/b$hb.log 2>&1 || { echo PROF_FAILED $hb; tail -20 gpurun_out/sweep/b$hb.log; exit 1; }
  echo "== hist_blocks $hb"; python3 tools/trace_breakdown.py gpurun_out/sweep/p$hb/run_kernel_trace.csv | grep -E "proof window|k_scatter|k_hist|k_accumulate|k_eval|k_scale"
done
