#!/bin/bash
# Round 5 (z): bench.py with the stored DVFS reading in its roofline: the bench GPU tests, then
# the default line exactly as the driver runs it.
set -o pipefail
mkdir -p gpurun_out/r05z
timeout -k 10 600 python -u -m pytest tests/test_bench.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r05z/tests.log 2>&1 || { tail -n 30 gpurun_out/r05z/tests.log; exit 1; }
tail -n 1 gpurun_out/r05z/tests.log
timeout -k 10 900 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r05z/bench_default.json 2> gpurun_out/r05z/bench_default.err || { tail -n 20 gpurun_out/r05z/bench_default.err; exit 1; }
python3 -c "
import json
d = json.loads(open('gpurun_out/r05z/bench_default.json').read().strip().splitlines()[-1]); r = d['roofline']
print('default', round(d['value'] / 1e6, 3), round(d['ms_per_step'], 2), round(r['frac'], 3), r.get('dvfs'))
"
