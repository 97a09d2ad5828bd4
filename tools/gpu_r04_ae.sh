#!/bin/bash
# Round 4: prover lanes at 2^20 on the final code, 12 / 14 / 16 (default queues), three times
# interleaved.
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/r04ae_lanes20.txt; : > $out
for r in 1 2 3; do
  for L in 12 14 16; do
    line=$(timeout -k 10 400 python bench.py --lanes $L --steps 8 --warmup 2 --no-cpu-baseline 2>>gpurun_out/r04ae.err) || exit 1
    python -c "import json,sys;d=json.loads(sys.argv[1]);print('2^20 lanes=$L', round(d['value']/1e6,3), 'M constraints/s', d.get('proofs_checked'))" "$line" | tee -a $out
  done
done
