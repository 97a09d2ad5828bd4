#!/bin/bash
# Round 5 final evidence, part 1 (final code): whole -m gpu suite and smoke; the default bench
# line exactly as the driver runs it (--steps 20 --warmup 5, CPU baseline); the default bench
# under rocprofv3 --kernel-trace --stats; one --pmc pass per traffic counter (FETCH_SIZE,
# WRITE_SIZE: separate runs, kernel trace only); single-lane proof breakdowns at 2^20 / 2^16.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05k
rm -rf $O; mkdir -p $O/prof $O/pmc $O/bd20 $O/bd16
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/tests.log 2>&1 || { tail -n 40 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -n 20 $O/smoke.log; exit 1; }
timeout -k 10 900 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_default.json 2> $O/bench_default.err || { tail -n 20 $O/bench_default.err; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python3 bench.py --no-cpu-baseline > $O/prof_bench.json 2> $O/prof_bench.err || { tail -n 20 $O/prof_bench.err; exit 1; }
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 600 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/pmc/$c -o run -- \
    python3 bench.py --no-cpu-baseline > $O/pmc_$c.json 2> $O/pmc_$c.err || { tail -n 20 $O/pmc_$c.err; exit 1; }
done
python3 tools/pmc_summary.py $O/pmc $O/pmc_traffic.json
for k in 20 16; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/bd$k -o run -- python3 bench.py \
    --steps 2 --warmup 1 --no-cpu-baseline --lanes 1 --log-n $k > $O/bd$k/bench.log 2>&1 || { tail -20 $O/bd$k/bench.log; exit 1; }
  python3 tools/trace_breakdown.py $O/bd$k/run_kernel_trace.csv > $O/bd$k/breakdown.txt
  head -14 $O/bd$k/breakdown.txt
done
python3 -c "
import json
d = json.loads(open('$O/bench_default.json').read().strip().splitlines()[-1]); r = d['roofline']
print('default', round(d['value'] / 1e6, 3), round(d['ms_per_step'], 2), round(r['frac'], 3), r.get('traffic'))
"
