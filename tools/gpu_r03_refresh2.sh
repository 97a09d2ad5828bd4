#!/bin/bash
# Round-3 evidence, part 2: BASELINE configs[1] / [2] lines (tools/gpu_configs.sh) and the plain
# default bench lines with their CPU baselines (what the driver runs), 2^20 and 2^16.
set -o pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/refresh
bash tools/gpu_configs.sh > gpurun_out/refresh/configs.log 2>&1 || { echo CONFIGS_FAILED; tail -30 gpurun_out/refresh/configs.log; exit 1; }
grep -h '"metric"' gpurun_out/configs/bench_*.json | cut -c1-200
timeout -k 10 600 python3 bench.py > gpurun_out/refresh/bench_default.log 2>&1 || { echo BENCH_FAILED; tail -30 gpurun_out/refresh/bench_default.log; exit 1; }
grep '"metric"' gpurun_out/refresh/bench_default.log > gpurun_out/refresh/bench_default.json
timeout -k 10 600 python3 bench.py --log-n 16 > gpurun_out/refresh/bench16.log 2>&1 || { echo BENCH16_FAILED; tail -30 gpurun_out/refresh/bench16.log; exit 1; }
grep '"metric"' gpurun_out/refresh/bench16.log > gpurun_out/refresh/bench16.json
python3 -c "
import json
for f in ('gpurun_out/refresh/bench_default.json','gpurun_out/refresh/bench16.json'):
    d=json.load(open(f)); c=d.get('cpu_baseline',{}); print(f, round(d['value']/1e6,3), 'M/s', round(d['ms_per_step'],1), 'ms/step; cpu', c.get('value'), c.get('ratio'))"
echo done
