#!/bin/bash
# Round 4: parity of the grouped-product build (default libplk.so) on the whole -m gpu suite,
# then an interleaved A/B against the ungrouped build (libplk-ungrp.so): 2^20 and 2^16 proofs,
# lone 2^20 / 2^16 MSMs.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r04c_gputest.log 2>&1 || { tail -40 gpurun_out/r04c_gputest.log; exit 1; }
tail -n 2 gpurun_out/r04c_gputest.log
out=gpurun_out/r04c_ab.jsonl; : > $out
for r in 1 2; do
  for lib in libplk.so libplk-ungrp.so; do
    for args in "--log-n 20 --steps 8" "--log-n 16 --steps 20" "--mode msm --log-n 20 --steps 20" "--mode msm --log-n 16 --steps 50"; do
      line=$(PLK_LIB=$PWD/dusk-plonk_amd/$lib timeout -k 10 300 python bench.py $args --warmup 2 --no-cpu-baseline 2>>gpurun_out/r04c_ab.err) || exit 1
      python -c "import json,sys;d=json.loads(sys.argv[1]);r=d['roofline'];print(json.dumps({'lib':sys.argv[2],'args':sys.argv[3],'value':d['value'],'ms':d['ms_per_step'],'adds_per_s':r.get('point_adds_per_s'),'frac':r['frac'],'insn':r.get('instructions_per_point_add'),'checked':d.get('proofs_checked')}))" "$line" $lib "$args" | tee -a $out
    done
  done
done
