#!/bin/bash
# Round 4: lone-MSM run length sweep (PLK_RUN_LANES: run lanes a lone wide MSM aims at; K =
# the largest run length <= 16 giving that many lanes) at 2^20 and 2^16, twice.
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/r04l_runlanes.txt; : > $out
for r in 1 2; do
  for L in 32768 65536 131072 262144; do
    for k in 20 16; do
      line=$(PLK_RUN_LANES=$L timeout -k 10 200 python bench.py --mode msm --log-n $k --steps 30 --warmup 3 --no-cpu-baseline 2>>gpurun_out/r04l.err) || exit 1
      python -c "import json,sys;d=json.loads(sys.argv[1]);print('2^$k run_lanes=$L', round(d['ms_per_step'],4), 'ms', round(d['value']/1e6,1), 'M points/s')" "$line" | tee -a $out
    done
  done
done
