#!/bin/bash
# Round 4: prover lanes for small proofs with 32 hardware queues (one per lane at 32 lanes),
# twice interleaved.
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/r04aa_small_lanes.txt; : > $out
for r in 1 2; do
  for kl in "12 16" "12 24" "12 32" "14 16" "14 24" "14 32"; do
    set -- $kl
    line=$(timeout -k 10 300 python bench.py --log-n $1 --lanes $2 --hw-queues 32 --steps 20 --warmup 3 --no-cpu-baseline 2>>gpurun_out/r04aa.err) || exit 1
    python -c "import json,sys;d=json.loads(sys.argv[1]);print('2^$1 lanes=$2', round(d['value']/1e6,3), 'M constraints/s', d.get('proofs_checked'), 'host_cores', json.dumps(d.get('host_cores'))[:160])" "$line" | tee -a $out
  done
done
