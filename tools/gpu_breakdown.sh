# single-lane 2^20 proof kernel breakdown (rocprofv3 kernel trace, last proof's window)
# usage: bash tools/gpu_breakdown.sh [variant]   (PLK_LIB from dusk-plonk_amd/libplk-<variant>.so)
set -o pipefail
export TMPDIR=/tmp
v=${1:-default}
if [ "$v" = default ]; then export PLK_LIB=""; else export PLK_LIB="$PWD/dusk-plonk_amd/libplk-$v.so"; fi
d=gpurun_out/bd_$v
rm -rf $d; mkdir -p $d
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $d -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --lanes 1 > $d/bench.log 2>&1 || { echo PROF_FAILED; tail -20 $d/bench.log; exit 1; }
python3 tools/trace_breakdown.py $d/run_kernel_trace.csv | tee $d/breakdown.txt
