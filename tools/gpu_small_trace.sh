# small-proof dispatch study at 2^LOGN (default 12): kernel trace of a single-lane bench (per-proof
# dispatch list) and of the default-lane bench (GPU busy fraction over the timed steps)
set -o pipefail
export TMPDIR=/tmp
k=${LOGN:-12}
d=gpurun_out/small; rm -rf $d; mkdir -p $d
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $d/one -o run -- python3 bench.py --log-n $k --steps 3 --warmup 1 --no-cpu-baseline --no-extras --lanes 1 > $d/one.log 2>&1 || { echo PROF1_FAILED; tail -20 $d/one.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $d/many -o run -- python3 bench.py --log-n $k --steps 20 --warmup 3 --no-cpu-baseline --no-extras > $d/many.log 2>&1 || { echo PROF2_FAILED; tail -20 $d/many.log; exit 1; }
python3 tools/small_trace.py $d/one/run_kernel_trace.csv $d/many/run_kernel_trace.csv | tee $d/summary.txt
