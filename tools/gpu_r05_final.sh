#!/bin/bash
# Round 5 final evidence on the final code: the whole -m gpu suite and smoke; the default bench
# line with its CPU baseline; the default bench command under rocprofv3 --kernel-trace --stats
# and one --pmc pass per traffic counter (FETCH_SIZE, WRITE_SIZE: separate runs, kernel trace
# only); BASELINE configs[1] / [2] lines (bit-exact vs the oracle, CPU baseline) with their
# own kernel traces; a 2^12 .. 2^20 size sweep; the 8-part split MSM line.
set -o pipefail
O=gpurun_out/r05f
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/tests.log 2>&1 || { tail -n 40 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -n 20 $O/smoke.log; exit 1; }
timeout -k 10 900 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -n 20 $O/bench_default.err; exit 1; }
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python3 bench.py --no-cpu-baseline > $O/prof_bench.json 2> $O/prof_bench.err || { tail -n 20 $O/prof_bench.err; exit 1; }
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/pmc/$c -o run -- \
    python3 bench.py --no-cpu-baseline > $O/pmc_$c.json 2> $O/pmc_$c.err || { tail -n 20 $O/pmc_$c.err; exit 1; }
done
python3 tools/pmc_summary.py $O/pmc $O/pmc_traffic.json
for m in ntt msm; do
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$m -o run -- \
    python3 bench.py --mode $m --log-n 20 --steps 30 --warmup 3 > $O/$m.json 2> $O/$m.err || { tail -n 20 $O/$m.err; exit 1; }
done
for k in 12 14 16 18 20; do
  timeout -k 10 400 python bench.py --log-n $k --steps 10 --warmup 3 --no-cpu-baseline >> $O/sizes.jsonl 2>> $O/sizes.err || exit 1
done
timeout -k 10 300 python bench.py --mode msm --log-n 20 --steps 20 --warmup 3 --no-cpu-baseline --bucket-parts 8 > $O/parts8.json || exit 1
for L in 10 14 16; do
  timeout -k 10 300 python bench.py --lanes $L --steps 8 --warmup 3 --no-cpu-baseline >> $O/lanes20.jsonl 2>> $O/lanes20.err || exit 1
done
python3 -c "
import json
for f in ['bench_default', 'ntt', 'msm', 'parts8']:
    d = json.loads(open('$O/' + f + '.json').read().strip().splitlines()[-1]); r = d['roofline']
    print(f, round(d['value'] / 1e6, 2), round(d['ms_per_step'], 3), round(r['frac'], 3))
for l in open('$O/sizes.jsonl'):
    d = json.loads(l); print(d['config']['log_n'], round(d['value'] / 1e6, 2))
for l in open('$O/lanes20.jsonl'):
    d = json.loads(l); print('lanes', d['host_cores']['lanes_run'], round(d['value'] / 1e6, 2))
"
