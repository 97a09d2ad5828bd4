# SQ issue / LDS counters of the NTT pass kernel: standalone NTT bench at 2^LOGN (default 20),
# two --pmc passes (kernel trace only)
set -o pipefail
export TMPDIR=/tmp
d=gpurun_out/sqntt; rm -rf $d; mkdir -p $d
run() {  # $1 = pass name, rest = counters
  local n=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d $d/$n -o run -- python3 bench.py --mode ntt --log-n ${LOGN:-20} --steps 4 --warmup 1 --no-cpu-baseline > $d/$n.log 2>&1 || { echo PMC_FAILED $n; tail -20 $d/$n.log; return 1; }
  python3 tools/sq_summary.py $d/$n/run_counter_collection.csv | grep -E "k_ntt_pass"
}
run a SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE &&
run b SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_WAVES SQ_BUSY_CYCLES
