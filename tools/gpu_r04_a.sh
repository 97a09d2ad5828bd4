#!/bin/bash
# Round 4, first GPU pass: the full -m gpu suite (incl. the 12-lane 2^20 byte check, the
# RCCL world-1 sharded prover, the aggregate-witness / ntt_stream entries) then the default
# bench line (proofs_checked) and a --shard-msm world-1 RCCL line at 2^20.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r04a_gputest.log 2>&1 || { tail -30 gpurun_out/r04a_gputest.log; exit 1; }
tail -3 gpurun_out/r04a_gputest.log
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 > gpurun_out/r04a_bench.json \
  2> gpurun_out/r04a_bench.err || { tail -20 gpurun_out/r04a_bench.err; exit 1; }
cat gpurun_out/r04a_bench.json
timeout -k 10 300 python -u bench.py --shard-msm --steps 5 --warmup 1 --no-cpu-baseline \
  > gpurun_out/r04a_shard1.json 2> gpurun_out/r04a_shard1.err || { tail -20 gpurun_out/r04a_shard1.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r04a_shard1.json'));print(d['value'],d['config']['parallelism'],d['proofs_checked'])"
