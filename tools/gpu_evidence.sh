set -o pipefail
cd /root/repo
bash tools/gpu_ranks_rehearsal.sh 2>&1 | cut -c1-300 || exit 1
bash tools/gpu_size_sweep.sh > gpurun_out/sweep.log 2>&1 || exit 1
bash tools/gpu_configs.sh > gpurun_out/configs.log 2>&1 || { tail -20 gpurun_out/configs.log; exit 1; }
grep -h '"metric"' gpurun_out/configs/bench_*.json | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['metric'][:60], round(d['value']/1e6,2), 'M', d['roofline']['avg_launch_ms'], d.get('bit_exact_vs_oracle'), d.get('cpu_baseline',{}).get('value'))"
