#!/bin/bash
# Round 4: (1) tools/gpu_r04_m.sh (madd grouping A/B), then (2) small-proof window sweep:
# PLK_MSM_C for 2^12 and 2^14 proofs, then (3) prover lanes at 2^12 / 2^14 (32 HW queues).
set -o pipefail
./tools/gpu_r04_m.sh || exit 1
out=gpurun_out/r04n_small_c.txt; : > $out
for r in 1; do
  for kc in "12 8" "12 9" "12 10" "12 11" "12 13" "14 10" "14 11" "14 13" "14 15" "14 16"; do
    set -- $kc
    line=$(PLK_MSM_C=$2 timeout -k 10 300 python bench.py --log-n $1 --steps 20 --warmup 3 --no-cpu-baseline 2>>gpurun_out/r04n.err) || exit 1
    python -c "import json,sys;d=json.loads(sys.argv[1]);print('2^$1 c=$2', round(d['value']/1e6,2), 'M constraints/s', d.get('proofs_checked'))" "$line" | tee -a $out
  done
done
out=gpurun_out/r04n_small_lanes.txt; : > $out
for kl in "12 16" "12 24" "12 32" "14 16" "14 24"; do
  set -- $kl
  line=$(timeout -k 10 300 python bench.py --log-n $1 --lanes $2 --hw-queues 32 --steps 12 --warmup 2 --no-cpu-baseline 2>>gpurun_out/r04n.err) || exit 1
  python -c "import json,sys;d=json.loads(sys.argv[1]);print('2^$1 lanes=$2', round(d['value']/1e6,2), 'M constraints/s', d.get('proofs_checked'))" "$line" | tee -a $out
done
