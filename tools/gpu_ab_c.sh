set -o pipefail
cd /root/repo
PLK_LIB=$PWD/dusk-plonk_amd/libplk-c16.so timeout -k 10 300 python3 -m pytest tests/test_msm_gpu.py -k "vs_oracle and (14 or 16)" -x -q --timeout 200 > gpurun_out/ab_c16_tests.log 2>&1 || { tail -20 gpurun_out/ab_c16_tests.log; exit 1; }
tail -1 gpurun_out/ab_c16_tests.log
bash tools/gpu_ab16.sh c15 c16
for L in 16; do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --log-n 16 --steps 10 --warmup 3 --lanes $L > gpurun_out/ab16_l$L.log 2>&1 || exit 1
  echo -n "lanes $L: "; grep '"metric"' gpurun_out/ab16_l$L.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,3))'
  PLK_LIB=$PWD/dusk-plonk_amd/libplk-c16.so timeout -k 10 300 python3 bench.py --no-cpu-baseline --log-n 16 --steps 10 --warmup 3 --lanes $L > gpurun_out/ab16_c16_l$L.log 2>&1 || exit 1
  echo -n "c16 lanes $L: "; grep '"metric"' gpurun_out/ab16_c16_l$L.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,3))'
done
