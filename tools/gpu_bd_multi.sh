# single-lane proof breakdowns (window + MSM kernels) for several libraries at 2^16 and 2^20
# usage: bash tools/gpu_bd_multi.sh [variant ...]   (default build first)
set -o pipefail
export TMPDIR=/tmp
for k in 16 20; do
  for v in default "$@"; do
    if [ "$v" = default ]; then export PLK_LIB=""; else export PLK_LIB="$PWD/dusk-plonk_amd/libplk-$v.so"; fi
    o=gpurun_out/bdm_${v}_$k; rm -rf $o; mkdir -p $o
    timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $o -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --lanes 1 --log-n $k > $o/bench.log 2>&1 || { echo PROF_FAILED; tail -20 $o/bench.log; exit 1; }
    python3 tools/trace_breakdown.py $o/run_kernel_trace.csv > $o/breakdown.txt
    echo "== 2^$k $v: $(head -1 $o/breakdown.txt) | $(grep -E 'k_accumulate|k_bucket_sum|k_bitsum1' $o/breakdown.txt | awk '{print $1, $NF=="ms" ? $(NF-1) : $NF}' | tr '\n' ' ')"
  done
done
