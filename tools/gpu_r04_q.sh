#!/bin/bash
# Round 4: the whole -m gpu suite on the quad-tail code, then lone-MSM bench lines (default
# settings) at 2^16 / 2^20.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r04q_tests.log 2>&1 || { tail -40 gpurun_out/r04q_tests.log; exit 1; }
tail -n 2 gpurun_out/r04q_tests.log
for k in 16 20; do
  timeout -k 10 300 python bench.py --mode msm --log-n $k --steps 50 --warmup 3 --no-cpu-baseline 2>>gpurun_out/r04q.err | tee -a gpurun_out/r04q_msm.jsonl || exit 1
done
