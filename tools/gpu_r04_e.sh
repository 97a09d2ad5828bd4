#!/bin/bash
# Round 4: NTT radix-4 products grouped (default: triple + single; ntt2: two pairs; ntt0: one
# by one). NTT + prover parity on the default build, then interleaved A/B of the standalone
# transforms (2^20, 2^23) and proofs (2^20, 2^16).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_ntt_gpu.py tests/test_prover_oracle.py tests/test_opening_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r04e_tests.log 2>&1 || { tail -30 gpurun_out/r04e_tests.log; exit 1; }
tail -n 1 gpurun_out/r04e_tests.log
out=gpurun_out/r04e_ab.jsonl; : > $out
for r in 1 2; do
  for lib in libplk.so libplk-ntt2.so libplk-ntt0.so; do
    for args in "--mode ntt --log-n 20 --steps 50" "--mode ntt --log-n 23 --steps 20" "--log-n 20 --steps 6" "--log-n 16 --steps 20"; do
      line=$(PLK_LIB=$PWD/dusk-plonk_amd/$lib timeout -k 10 300 python bench.py $args --warmup 2 --no-cpu-baseline 2>>gpurun_out/r04e_ab.err) || exit 1
      python -c "import json,sys;d=json.loads(sys.argv[1]);r=d['roofline'];print(json.dumps({'lib':sys.argv[2],'args':sys.argv[3],'value':d['value'],'ms':d['ms_per_step'],'frac':r['frac'],'checked':d.get('proofs_checked')}))" "$line" $lib "$args" | tee -a $out
    done
  done
done
