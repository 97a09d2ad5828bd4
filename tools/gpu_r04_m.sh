#!/bin/bash
# Round 4: madd product grouping A/B — (PPP, Q) + (Y3, ZZ3, ZZZ3) [default] against
# (PPP, Q, ZZ3) + (Y3, ZZZ3) [PLK_MADD_GROUPED=2, libplk-g2]: accumulate micro-benchmark,
# MSM parity of the variant, then interleaved bench lines.
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  for v in grp grp2; do
    echo "== $v run $r"; timeout -k 10 120 ./tools/ubench_acc_$v | grep v4_lazy || exit 1
  done
done 2>&1 | tee gpurun_out/r04m_ubench.txt || exit 1
PLK_LIB=$PWD/dusk-plonk_amd/libplk-g2.so timeout -k 10 400 python -u -m pytest tests/test_msm_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r04m_tests.log 2>&1 || { tail -30 gpurun_out/r04m_tests.log; exit 1; }
echo "g2 msm tests: $(tail -n 1 gpurun_out/r04m_tests.log)"
out=gpurun_out/r04m_ab.jsonl; : > $out
for r in 1 2; do
  for lib in libplk.so libplk-g2.so; do
    for args in "--log-n 20 --steps 12" "--mode msm --log-n 20 --steps 30"; do
      line=$(PLK_LIB=$PWD/dusk-plonk_amd/$lib timeout -k 10 300 python bench.py $args --warmup 3 --no-cpu-baseline 2>>gpurun_out/r04m_ab.err) || exit 1
      python -c "import json,sys;d=json.loads(sys.argv[1]);print(json.dumps({'lib':sys.argv[2],'args':sys.argv[3],'value':d['value'],'ms':d['ms_per_step']}))" "$line" $lib "$args" | tee -a $out
    done
  done
done
