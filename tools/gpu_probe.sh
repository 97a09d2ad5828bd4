set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_msm_gpu.py tests/test_prover_gpu.py -x -q -p no:cacheprovider > gpurun_out/tq.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/tq.log; exit 1; }
tail -1 gpurun_out/tq.log
timeout -k 10 300 python tools/synth_probe.py > gpurun_out/probe.log 2>&1 || { echo PROBE_FAILED; tail -20 gpurun_out/probe.log; exit 1; }
cat gpurun_out/probe.log
