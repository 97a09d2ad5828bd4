# rocprofv3 evidence for the default bench command (2^20 full prover, default steps /
# warmup / lanes; the bench's JSON line saved beside its kernel-trace stats),
# then one PMC pass per counter (FETCH_SIZE, WRITE_SIZE) in separate runs with
# --kernel-trace only (no sys/runtime trace domains with --pmc)
set -o pipefail
mkdir -p gpurun_out/pmc gpurun_out/prof
export TMPDIR=/tmp
rm -rf gpurun_out/pmc/* gpurun_out/prof/*
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --no-cpu-baseline > gpurun_out/prof/bench.log 2>&1 || { echo PROF_FAILED; tail -30 gpurun_out/prof/bench.log; exit 1; }
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/pmc/$c -o run -- python3 bench.py --no-cpu-baseline > gpurun_out/pmc/$c.log 2>&1 || { echo PMC_FAILED $c; tail -20 gpurun_out/pmc/$c.log; exit 1; }
done
python3 tools/pmc_summary.py gpurun_out/pmc gpurun_out/pmc/pmc_traffic.json
grep '"metric"' gpurun_out/prof/bench.log > gpurun_out/prof/bench_line.json
