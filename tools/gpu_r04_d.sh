#!/bin/bash
# Round 4: accumulation-loop A/B with use-only chain pins (ubench_acc four ways), twice.
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  for v in base pin grp grppin; do
    echo "== $v run $r"; timeout -k 10 120 ./tools/ubench_acc_$v | grep -E "v4|v0" || exit 1
  done
done 2>&1 | tee gpurun_out/r04d_ubench_acc.txt
