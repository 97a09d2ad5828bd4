#!/bin/bash
# Round 4: accumulation-loop codegen A/B (ubench_acc built three ways: default, per-mad
# pinned chains, interleaved product groups) twice interleaved, then the RCCL world-1 test.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
  for v in base pin grp; do
    echo "== $v run $r"; timeout -k 10 120 ./tools/ubench_acc_$v || exit 1
  done
done 2>&1 | tee gpurun_out/r04b_ubench_acc.txt
timeout -k 10 300 python -u -m pytest tests/test_parallel.py -k rccl -x -v -s --timeout 240 \
  --timeout-method thread > gpurun_out/r04b_rccl.log 2>&1; rc=$?
tail -25 gpurun_out/r04b_rccl.log
exit $rc
