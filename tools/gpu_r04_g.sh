#!/bin/bash
# Round 4: constant-twiddle Shoup product. Microbenchmark (device check against the
# Montgomery product + throughput), NTT / prover parity with the Shoup build, then an
# interleaved A/B against the default build; also the run-sum step 2 at two waves per SIMD
# (libplk-rs2.so, PLK_RUNSUM_WAVES=2: 256 VGPRs + 3 spills instead of 259 registers at one wave).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 ./tools/ubench_shoup | tee gpurun_out/r04g_ubench_shoup.txt || exit 1
PLK_LIB=$PWD/dusk-plonk_amd/libplk-shoup.so timeout -k 10 400 python -u -m pytest tests/test_ntt_gpu.py tests/test_prover_oracle.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r04g_tests.log 2>&1 || { tail -30 gpurun_out/r04g_tests.log; exit 1; }
echo "shoup build: $(tail -n 1 gpurun_out/r04g_tests.log)"
out=gpurun_out/r04g_ab.jsonl; : > $out
for r in 1 2; do
  for lib in libplk.so libplk-shoup.so libplk-rs2.so; do
    for args in "--mode ntt --log-n 20 --steps 50" "--mode ntt --log-n 23 --steps 20" "--log-n 20 --steps 6" "--log-n 16 --steps 20" "--mode msm --log-n 20 --steps 20"; do
      line=$(PLK_LIB=$PWD/dusk-plonk_amd/$lib timeout -k 10 300 python bench.py $args --warmup 2 --no-cpu-baseline 2>>gpurun_out/r04g_ab.err) || exit 1
      python -c "import json,sys;d=json.loads(sys.argv[1]);r=d['roofline'];print(json.dumps({'lib':sys.argv[2],'args':sys.argv[3],'value':d['value'],'ms':d['ms_per_step'],'frac':r['frac'],'checked':d.get('proofs_checked')}))" "$line" $lib "$args" | tee -a $out
    done
  done
done
