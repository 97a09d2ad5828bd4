set -o pipefail
cd /root/repo
bash tools/gpu_configs.sh > gpurun_out/configs.log 2>&1 || { tail -20 gpurun_out/configs.log; exit 1; }
cat gpurun_out/configs/bench_*.json | grep '"metric"' | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['metric'][:60], round(d['value']/1e6,2), 'M', round(d['roofline']['avg_launch_ms'],4), d.get('bit_exact_vs_oracle'), d.get('cpu_baseline',{}).get('value'))"
