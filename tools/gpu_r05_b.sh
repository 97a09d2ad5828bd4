#!/bin/bash
# Round 5 (b): the pruned library (NTT / MSM switches removed, LDS-DMA accumulation with the
# lone / lane forms, tail policy read once): the whole -m gpu suite and smoke, then kernel traces
# of the lone 2^20 MSM whole and as 8 bucket-range parts, and the default / lone-MSM lines.
set -o pipefail
mkdir -p gpurun_out/r05b
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r05b/tests.log 2>&1 || { tail -n 40 gpurun_out/r05b/tests.log; exit 1; }
tail -n 2 gpurun_out/r05b/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05b/smoke.log 2>&1 || { tail -n 20 gpurun_out/r05b/smoke.log; exit 1; }
tail -n 1 gpurun_out/r05b/smoke.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for p in 1 8; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05b/prof_parts$p -o run -- \
    python bench.py --mode msm --log-n 20 --steps 10 --warmup 2 --no-cpu-baseline --bucket-parts $p \
    > gpurun_out/r05b/parts$p.json 2> gpurun_out/r05b/parts$p.err || { tail -n 20 gpurun_out/r05b/parts$p.err; exit 1; }
done
timeout -k 10 300 python bench.py --mode msm --log-n 20 --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/r05b/msm20.json || exit 1
timeout -k 10 400 python bench.py --steps 8 --warmup 3 --no-cpu-baseline > gpurun_out/r05b/prove20.json || exit 1
cat gpurun_out/r05b/msm20.json gpurun_out/r05b/prove20.json | python -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); r=d['roofline']; print(d['metric'][:40], round(d['value']/1e6,2), round(d['ms_per_step'],3), r.get('point_adds_per_s'), round(r['frac'],3))"
