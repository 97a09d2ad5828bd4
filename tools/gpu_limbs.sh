set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 ./tools/ubench_limbs > gpurun_out/ubench_limbs.log 2>&1 || { echo UBL_FAILED; cat gpurun_out/ubench_limbs.log; exit 1; }
cat gpurun_out/ubench_limbs.log
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/full20.log 2>&1 || { echo FULL20_FAILED; tail -30 gpurun_out/full20.log; exit 1; }
grep metric gpurun_out/full20.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['breakdown_ms_per_step'])"
