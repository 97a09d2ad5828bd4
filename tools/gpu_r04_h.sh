#!/bin/bash
# Round 4: full -m gpu suite on the default build (grouped products, DPP quad NTT exchange,
# one-dispatch small sort), the Shoup microbenchmark and NTT parity of the Shoup build, then
# interleaved A/Bs: Shoup NTT (libplk-shoup), run-sum step 2 at 2 waves (libplk-rs2), the
# one-dispatch small sort off (libplk-so0).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r04h_gputest.log 2>&1 || { tail -40 gpurun_out/r04h_gputest.log; exit 1; }
tail -n 1 gpurun_out/r04h_gputest.log
timeout -k 10 120 ./tools/ubench_shoup > gpurun_out/r04h_ubench_shoup.txt || exit 1
cat gpurun_out/r04h_ubench_shoup.txt
PLK_LIB=$PWD/dusk-plonk_amd/libplk-shoup.so timeout -k 10 400 python -u -m pytest tests/test_ntt_gpu.py tests/test_prover_oracle.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r04h_shoup_tests.log 2>&1 || { tail -30 gpurun_out/r04h_shoup_tests.log; exit 1; }
echo "shoup build: $(tail -n 1 gpurun_out/r04h_shoup_tests.log)"
out=gpurun_out/r04h_ab.jsonl; : > $out
ab() {  # ab <variant lib> <args...>
  local v=$1; shift
  for r in 1 2; do
    for lib in libplk.so $v; do
      for args in "$@"; do
        line=$(PLK_LIB=$PWD/dusk-plonk_amd/$lib timeout -k 10 300 python bench.py $args --warmup 2 --no-cpu-baseline 2>>gpurun_out/r04h_ab.err) || exit 1
        python -c "import json,sys;d=json.loads(sys.argv[1]);r=d['roofline'];print(json.dumps({'lib':sys.argv[2],'args':sys.argv[3],'value':d['value'],'ms':d['ms_per_step'],'frac':r['frac'],'checked':d.get('proofs_checked')}))" "$line" $lib "$args" | tee -a $out
      done
    done
  done
}
ab libplk-so0.so "--log-n 12 --steps 30" "--log-n 14 --steps 20" || exit 1
ab libplk-rs2.so "--log-n 20 --steps 6" "--log-n 16 --steps 20" "--mode msm --log-n 20 --steps 20" || exit 1
ab libplk-shoup.so "--mode ntt --log-n 20 --steps 50" "--mode ntt --log-n 23 --steps 20" || exit 1
