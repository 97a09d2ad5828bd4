#!/bin/bash
# Round 4: window size for small proofs again, now that a short top window is spread over the
# buckets (plk_srs::top_shift): PLK_MSM_C at 2^12 and 2^14, twice interleaved.
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/r04x_small_c.txt; : > $out
for r in 1 2; do
  for kc in "12 10" "12 11" "12 12" "12 13" "14 15" "14 13" "14 14" "14 16"; do
    set -- $kc
    line=$(PLK_MSM_C=$2 timeout -k 10 300 python bench.py --log-n $1 --steps 30 --warmup 3 --no-cpu-baseline 2>>gpurun_out/r04x.err) || exit 1
    python -c "import json,sys;d=json.loads(sys.argv[1]);print('2^$1 c=$2', round(d['value']/1e6,3), 'M constraints/s', d.get('proofs_checked'))" "$line" | tee -a $out
  done
done
