#!/bin/bash
# Round 5 (a): k_accumulate with the next point prefetched by LDS-DMA, at 2 and 3 waves per
# SIMD and four product groupings, against round 4's register prefetch (libplk-base): MSM
# parity of every variant, then interleaved lone-MSM and 2^20 proof lines (tools/ab.py).
# Last, once: the rebuilt libplk-g2 (round 4's aborting build: PLK_MADD_GROUPED=2, register
# prefetch, 1-wave bound) runs test_msm_golden under AMD_LOG_LEVEL=1.
set -o pipefail
mkdir -p gpurun_out
V="--lib base=libplk-base.so --lib d2g1=libplk.so --lib d3g1=libplk-d3g1.so --lib d3g0=libplk-d3g0.so --lib d3g2=libplk-d3g2.so"
timeout -k 10 1080 python -u tools/ab.py --out gpurun_out/r05a_ab.jsonl --reps 2 $V \
  --tests "tests/test_msm_gpu.py -k 'golden or wide_buckets or 2_20_vs_oracle'" \
  --args "--mode msm --log-n 20 --steps 30" --args "--log-n 20 --steps 6" || exit 1
timeout -k 10 300 python -u -m pytest tests/test_msm_gpu.py -k "bucket_parts" -x -v --timeout 200 --timeout-method thread \
  > gpurun_out/r05a_parts_tests.log 2>&1 || { tail -n 30 gpurun_out/r05a_parts_tests.log; exit 1; }
tail -n 2 gpurun_out/r05a_parts_tests.log
for p in 1 2 4 8; do
  timeout -k 10 200 python bench.py --mode msm --log-n 20 --steps 20 --warmup 3 --no-cpu-baseline --bucket-parts $p \
    >> gpurun_out/r05a_parts_bench.jsonl 2>> gpurun_out/r05a_parts_bench.err || exit 1
done
AMD_LOG_LEVEL=1 PLK_LIB=$PWD/dusk-plonk_amd/libplk-g2.so timeout -k 10 300 python -u -m pytest \
  "tests/test_msm_gpu.py::test_msm_golden" -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/r05a_g2.log 2>&1
echo "g2 test_msm_golden rc $?"; tail -n 5 gpurun_out/r05a_g2.log
