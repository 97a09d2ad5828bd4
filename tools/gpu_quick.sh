# quick GPU cycle: MSM + prover parity tests, then the full-prover bench at 2^20
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/tq.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/tq.log; exit 1; }
tail -2 gpurun_out/tq.log
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/full20.log 2>&1 || { echo FULL20_FAILED; tail -30 gpurun_out/full20.log; exit 1; }
grep metric gpurun_out/full20.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['breakdown_ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['point_adds_per_s'])"
