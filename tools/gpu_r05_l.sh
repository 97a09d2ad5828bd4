#!/bin/bash
# Round 5 final evidence, part 2 (final code): BASELINE configs[1] / [2] (tools/gpu_configs.sh:
# standalone NTT / MSM lines bit-exact vs the oracle with their kernel traces and FETCH / WRITE
# passes), a 2^12 .. 2^20 size sweep, the 8-part split MSM line.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05l
rm -rf $O; mkdir -p $O
timeout -k 10 900 bash tools/gpu_configs.sh > $O/configs.log 2>&1 || { tail -n 30 $O/configs.log; exit 1; }
tail -n 12 $O/configs.log
for k in 12 14 16 18 20; do
  timeout -k 10 400 python bench.py --log-n $k --steps 10 --warmup 3 --no-cpu-baseline >> $O/sizes.jsonl 2>> $O/sizes.err || exit 1
done
timeout -k 10 300 python bench.py --mode msm --log-n 20 --steps 20 --warmup 3 --no-cpu-baseline --bucket-parts 8 > $O/parts8.json || exit 1
python3 -c "
import json
for l in open('$O/sizes.jsonl'):
    d = json.loads(l); print(d['config']['log_n'], round(d['value'] / 1e6, 2), round(d['ms_per_step'], 2))
d = json.loads(open('$O/parts8.json').read().strip().splitlines()[-1]); print('parts8', round(d['ms_per_step'], 3))
"
