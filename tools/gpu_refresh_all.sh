# One GPU call for the round's evidence: every GPU test, the rocprofv3 evidence of
# tools/gpu_profile.sh (default bench under --kernel-trace --stats, FETCH/WRITE PMC passes,
# single-lane breakdowns at 2^20 / 2^16), BASELINE configs[1]/[2] lines (tools/gpu_configs.sh)
# and the plain default bench line with its CPU baseline (what the driver runs).
set -o pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/refresh
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/refresh/pytest.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/refresh/pytest.log; exit 1; }
tail -1 gpurun_out/refresh/pytest.log
bash tools/gpu_profile.sh || exit 1
bash tools/gpu_configs.sh > gpurun_out/refresh/configs.log 2>&1 || { echo CONFIGS_FAILED; tail -30 gpurun_out/refresh/configs.log; exit 1; }
grep -h '"metric"' gpurun_out/configs/bench_*.json | cut -c1-200
timeout -k 10 600 python bench.py > gpurun_out/refresh/bench_default.log 2>&1 || { echo BENCH_FAILED; tail -30 gpurun_out/refresh/bench_default.log; exit 1; }
grep '"metric"' gpurun_out/refresh/bench_default.log > gpurun_out/refresh/bench_default.json
timeout -k 10 600 python bench.py --log-n 16 > gpurun_out/refresh/bench16.log 2>&1 || { echo BENCH16_FAILED; tail -30 gpurun_out/refresh/bench16.log; exit 1; }
grep '"metric"' gpurun_out/refresh/bench16.log > gpurun_out/refresh/bench16.json
python3 -c "
import json
for f in ('gpurun_out/refresh/bench_default.json','gpurun_out/refresh/bench16.json'):
    d=json.load(open(f)); print(f, round(d['value']/1e6,3), 'M/s', round(d['ms_per_step'],1), 'ms/step; cpu', d.get('cpu_baseline',{}).get('value'))"
echo done
