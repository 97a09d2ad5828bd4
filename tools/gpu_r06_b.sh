#!/bin/bash
# Round 6 (b): the new line fields and the bucket-split sharded prover on the GPU, then an
# interleaved A/B of k_accumulate's s_nop cost (PLK_EXTRA_NOPS: +1 s_nop per product-group
# step) and the per-mad inline-asm form (PLK_RX_ASM_MAD), then the default bench line.
set -eo pipefail
d=gpurun_out/r06b; rm -rf $d; mkdir -p $d
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu \
  tests/test_bench.py tests/test_ntt_gpu.py::test_idft_multipass_identity_rows \
  "tests/test_parallel.py::test_sharded_prover_bucket_split" \
  tests/test_parallel.py::test_sharded_prover_bucket_split_refused_small_srs \
  tests/test_parallel.py::test_sharded_prover_2_20_bucket_split_equals_fixture > $d/tests.log 2>&1
timeout -k 10 600 python tools/ab.py --out $d/ab.jsonl --reps 2 --lib base=libplk.so \
  --lib nops=libplk-nops.so --lib asm1=libplk-asm1.so --args "--log-n 20 --steps 10" > $d/ab.log 2>&1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $d/bench.log 2>&1
