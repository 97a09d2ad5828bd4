set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/n16
for L in 3 6 8; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --log-n 16 --lanes $L --steps 10 --warmup 3 > gpurun_out/n16/bench_l$L.log 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/n16/bench_l$L.log; exit 1; }
  echo -n "lanes $L: "; grep '"metric"' gpurun_out/n16/bench_l$L.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,3), "M/s", round(d["ms_per_step"],2), "ms/step", d.get("breakdown_ms_per_step"))'
done
d=gpurun_out/n16/bd; rm -rf $d; mkdir -p $d
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $d -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --lanes 1 --log-n 16 > $d/bench.log 2>&1 || { echo PROF_FAILED; tail -20 $d/bench.log; exit 1; }
python3 tools/trace_breakdown.py $d/run_kernel_trace.csv | tee $d/breakdown.txt | head -30
