#!/bin/bash
# Round 4: k_sort_one with the scalars kept in registers (default build) — MSM / prover parity,
# then an interleaved A/B against PLK_CHUNK_SMALL=16 (libplk-cs16: the round-3 task floor for
# small batches) at 2^12 / 2^14 / 2^16.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_msm_gpu.py tests/test_prover_gpu.py tests/test_prover_oracle.py tests/test_prover_lanes.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r04k_tests.log 2>&1 || { tail -30 gpurun_out/r04k_tests.log; exit 1; }
tail -n 1 gpurun_out/r04k_tests.log
PLK_LIB=$PWD/dusk-plonk_amd/libplk-cs16.so timeout -k 10 600 python -u -m pytest tests/test_msm_gpu.py tests/test_prover_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r04k_tests_cs16.log 2>&1 || { tail -30 gpurun_out/r04k_tests_cs16.log; exit 1; }
echo "cs16: $(tail -n 1 gpurun_out/r04k_tests_cs16.log)"
out=gpurun_out/r04k_ab.jsonl; : > $out
for r in 1 2; do
  for lib in libplk.so libplk-cs16.so; do
    for args in "--log-n 12 --steps 30" "--log-n 14 --steps 20" "--log-n 16 --steps 20" "--mode msm --log-n 16 --steps 50"; do
      line=$(PLK_LIB=$PWD/dusk-plonk_amd/$lib timeout -k 10 300 python bench.py $args --warmup 3 --no-cpu-baseline 2>>gpurun_out/r04k_ab.err) || exit 1
      python -c "import json,sys;d=json.loads(sys.argv[1]);print(json.dumps({'lib':sys.argv[2],'args':sys.argv[3],'value':d['value'],'ms':d['ms_per_step'],'checked':d.get('proofs_checked')}))" "$line" $lib "$args" | tee -a $out
    done
  done
done
