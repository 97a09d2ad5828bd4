#!/bin/bash
# BASELINE.json configs[1] / configs[2]: standalone NTT (dft + idft) and G1 MSM bench lines
# (bit-exact against the oracle, CPU baseline on the box's host cores) at 2^20, plus 2^23 /
# 2^16; a kernel-trace summary and FETCH/WRITE passes of each 2^20 line (units = the
# transforms / MSMs of that run: (steps + warmup) x 2 / x 1).
set -euo pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/configs
mkdir -p $O
B="--steps 10 --warmup 2"
for m in ntt msm; do
  u=$([ $m = ntt ] && echo 24 || echo 12)
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$m -o run -- \
    python3 -u bench.py --mode $m --log-n 20 $B --no-cpu-baseline > $O/prof_$m.log 2>&1
  cp $O/prof_$m/run_kernel_stats.csv $O/${m}20_kernel_stats.csv
  mkdir -p $O/pmc_$m
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/pmc_$m/$c -o run -- \
      python3 -u bench.py --mode $m --log-n 20 $B --no-cpu-baseline > $O/pmc_$m/$c.log 2>&1
  done
  python3 tools/pmc_summary.py $O/pmc_$m $O/pmc_traffic_${m}20.json
  python3 -c "import json,sys; f=sys.argv[1]; d=json.load(open(f)); d['units']=int(sys.argv[2]); json.dump(d,open(f,'w'),indent=1)" $O/pmc_traffic_${m}20.json $u
  cp $O/pmc_traffic_${m}20.json profiles/  # box-local copy: the bench lines below read it
done
for a in "ntt 20" "msm 20" "ntt 23" "msm 16"; do
  set -- $a
  echo "== $1 2^$2"
  timeout -k 10 300 python3 -u bench.py --mode $1 --log-n $2 $B > $O/bench_$1_$2.json 2> $O/bench_$1_$2.err
  cat $O/bench_$1_$2.json
done
echo done
