# per-pass NTT kernel durations: kernel trace of the standalone NTT bench (2^LOGN, default 20)
set -o pipefail
export TMPDIR=/tmp
d=gpurun_out/nttrace; rm -rf $d; mkdir -p $d
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $d/p -o run -- python3 bench.py --mode ntt --log-n ${LOGN:-20} --steps 10 --warmup 2 --no-cpu-baseline > $d/b.log 2>&1 || { echo FAILED; tail -20 $d/b.log; exit 1; }
f=$(find $d/p -name '*kernel_trace.csv' | head -1); cp $f $d/kernel_trace.csv; echo ok
