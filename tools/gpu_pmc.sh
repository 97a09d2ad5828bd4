set -o pipefail
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/pmc/$c -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/pmc/$c.log 2>&1 || { echo PMC_FAILED $c; tail -20 gpurun_out/pmc/$c.log; exit 1; }
done
ls -R gpurun_out/pmc | head -30
