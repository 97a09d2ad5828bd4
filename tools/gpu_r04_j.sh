#!/bin/bash
# Round 4: small-proof sweep at 2^12 (and 2^14): MSM window c (PLK_MSM_C) and lanes / hardware
# queues, twice each.
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/r04j_small_sweep.txt; : > $out
run() {  # run <label> <env...> -- <args>
  local label=$1; shift
  line=$(env "$@" timeout -k 10 200 python bench.py --warmup 3 --no-cpu-baseline 2>>gpurun_out/r04j.err) || return 1
  python -c "import json,sys;d=json.loads(sys.argv[1]);print(sys.argv[2], round(d['value']/1e6,3), 'M', round(d['ms_per_step'],3), 'ms', d['config'].get('msm_window_bits'), d['config'].get('hip_hw_queues'))" "$line" "$label" | tee -a $out
}
for r in 1 2; do
  for c in 8 9 10 11 12; do
    line=$(PLK_MSM_C=$c timeout -k 10 200 python bench.py --log-n 12 --steps 30 --warmup 3 --no-cpu-baseline 2>>gpurun_out/r04j.err) || exit 1
    python -c "import json,sys;d=json.loads(sys.argv[1]);print('2^12 c=$c', round(d['value']/1e6,3), 'M', round(d['ms_per_step'],3), 'ms', d['config'].get('msm_window_bits'))" "$line" | tee -a $out
  done
  for L in 16 24 32; do
    line=$(timeout -k 10 200 python bench.py --log-n 12 --steps 30 --warmup 3 --no-cpu-baseline --lanes $L --hw-queues 32 2>>gpurun_out/r04j.err) || exit 1
    python -c "import json,sys;d=json.loads(sys.argv[1]);print('2^12 lanes=$L q=32', round(d['value']/1e6,3), 'M', round(d['ms_per_step'],3), 'ms')" "$line" | tee -a $out
  done
  for L in 14 20 28; do
    line=$(timeout -k 10 200 python bench.py --log-n 14 --steps 20 --warmup 3 --no-cpu-baseline --lanes $L --hw-queues 32 2>>gpurun_out/r04j.err) || exit 1
    python -c "import json,sys;d=json.loads(sys.argv[1]);print('2^14 lanes=$L q=32', round(d['value']/1e6,3), 'M', round(d['ms_per_step'],3), 'ms')" "$line" | tee -a $out
  done
done
