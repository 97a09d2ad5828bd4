#!/bin/bash
# Round 3: the whole -m gpu suite (verbose: one line per test), the default bench line with
# its CPU baseline (measured concurrent throughput), the 2^16 line, and the limb-form A/B
# microbenchmark (tools/ubench_limbs.hip: 14x28 vs 13x30 Fp multiply). Each step has its own
# time limit; the chain stops at the first failure.
set -uo pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r03b
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 \
  || { echo TESTS_FAILED; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 600 python3 -u bench.py > $O/bench20.log 2>&1 || { echo BENCH_FAILED; tail -30 $O/bench20.log; exit 1; }
grep '"metric"' $O/bench20.log > $O/bench20.json
timeout -k 10 300 python3 -u bench.py --log-n 16 --no-cpu-baseline > $O/bench16.log 2>&1 || { echo BENCH16_FAILED; tail -30 $O/bench16.log; exit 1; }
grep '"metric"' $O/bench16.log > $O/bench16.json
timeout -k 10 120 ./tools/ubench_limbs > $O/ubench_limbs.txt 2>&1 || { echo UBENCH_FAILED; cat $O/ubench_limbs.txt; exit 1; }
cat $O/ubench_limbs.txt
python3 -c "
import json
for f in ('$O/bench20.json','$O/bench16.json'):
    d=json.load(open(f)); r=d['roofline']
    print(f, round(d['value']/1e6,3), 'M/s', round(d['ms_per_step'],1), 'ms/step; roofline', r['bound'], round(r['frac'],3), 'cpu', json.dumps(d.get('cpu_baseline',{}).get('ratio')))"
echo done
