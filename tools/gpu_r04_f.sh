#!/bin/bash
# Round 4: NTT last-two-steps quad exchange variants (PLK_NTT_QUADX 0 default / 1 wave-local
# LDS exchange without barrier / 2 DPP register transpose): NTT parity for each build, then
# interleaved A/B of standalone transforms and the 2^20 proof.
set -o pipefail
mkdir -p gpurun_out
for lib in libplk-qx1.so libplk-qx2.so; do
  PLK_LIB=$PWD/dusk-plonk_amd/$lib timeout -k 10 300 python -u -m pytest tests/test_ntt_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread \
    > gpurun_out/r04f_tests_$lib.log 2>&1 || { tail -30 gpurun_out/r04f_tests_$lib.log; exit 1; }
  echo "$lib: $(tail -n 1 gpurun_out/r04f_tests_$lib.log)"
done
out=gpurun_out/r04f_ab.jsonl; : > $out
for r in 1 2; do
  for lib in libplk.so libplk-qx1.so libplk-qx2.so; do
    for args in "--mode ntt --log-n 20 --steps 50" "--mode ntt --log-n 23 --steps 20" "--mode ntt --log-n 17 --steps 100" "--log-n 20 --steps 6"; do
      line=$(PLK_LIB=$PWD/dusk-plonk_amd/$lib timeout -k 10 300 python bench.py $args --warmup 2 --no-cpu-baseline 2>>gpurun_out/r04f_ab.err) || exit 1
      python -c "import json,sys;d=json.loads(sys.argv[1]);r=d['roofline'];print(json.dumps({'lib':sys.argv[2],'args':sys.argv[3],'value':d['value'],'ms':d['ms_per_step'],'frac':r['frac'],'checked':d.get('proofs_checked')}))" "$line" $lib "$args" | tee -a $out
    done
  done
done
