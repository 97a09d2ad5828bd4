#!/bin/bash
# Round 4: tail forms at 2^14 / 2^12 proofs (PLK_TAIL_QUAD 0 / 1 / 2), three times interleaved.
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/r04ag_ab.jsonl; : > $out
for r in 1 2 3; do
  for q in 1 0 2; do
    for args in "--log-n 14 --steps 20" "--log-n 12 --steps 30"; do
      line=$(PLK_TAIL_QUAD=$q timeout -k 10 300 python bench.py $args --warmup 3 --no-cpu-baseline 2>>gpurun_out/r04ag.err) || exit 1
      python -c "import json,sys;d=json.loads(sys.argv[1]);print(json.dumps({'tail':sys.argv[2],'args':sys.argv[3],'value':d['value'],'checked':d.get('proofs_checked')}))" "$line" $q "$args" | tee -a $out
    done
  done
done
