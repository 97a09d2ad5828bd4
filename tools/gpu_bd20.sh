# single-lane 2^20 proof breakdowns (kernel trace) for the default build and variants
# usage: bash tools/gpu_bd20.sh [variant ...]   (LOGN=16 for 2^16)
set -o pipefail
export TMPDIR=/tmp
k=${LOGN:-20}
for v in default "$@"; do
  if [ "$v" = default ]; then export PLK_LIB=""; else export PLK_LIB="$PWD/dusk-plonk_amd/libplk-$v.so"; fi
  o=gpurun_out/bd20_${v}_$k; rm -rf $o; mkdir -p $o
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $o -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --lanes 1 --log-n $k > $o/bench.log 2>&1 || { echo PROF_FAILED $v; tail -20 $o/bench.log; exit 1; }
  echo "== 2^$k $v"; python3 tools/trace_breakdown.py $o/run_kernel_trace.csv | tee $o/breakdown.txt
done
