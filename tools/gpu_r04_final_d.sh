#!/bin/bash
# Round-4 last check on the final library: the whole -m gpu suite, smoke(), one default
# bench line (with its CPU baseline).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/finald
rm -rf $O; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -n 1 $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench_default.log 2>&1 || { tail -30 $O/bench_default.log; exit 1; }
grep '"metric"' $O/bench_default.log > $O/bench_default.json
python -c "
import json
d=json.load(open('$O/bench_default.json')); r=d['roofline']
print(round(d['value']/1e6,3), 'M/s', round(d['ms_per_step'],1), 'ms/step; checked', d.get('proofs_checked'), '; frac', round(r['frac'],3), '; cpu', round(d['cpu_baseline']['value']))"
