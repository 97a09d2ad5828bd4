set -o pipefail
export TMPDIR=/tmp
v=$1; k=$2
export PLK_LIB="$PWD/dusk-plonk_amd/libplk-$v.so"
o=gpurun_out/bdv_${v}_$k; rm -rf $o; mkdir -p $o
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $o -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --lanes 1 --log-n $k > $o/bench.log 2>&1 || { echo PROF_FAILED; tail -20 $o/bench.log; exit 1; }
python3 tools/trace_breakdown.py $o/run_kernel_trace.csv | head -14
