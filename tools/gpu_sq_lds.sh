# LDS counters for the prover kernels (one --pmc pass)
set -o pipefail
export TMPDIR=/tmp
d=gpurun_out/sqlds
rm -rf $d; mkdir -p $d
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_INSTS_VALU SQ_BUSY_CYCLES --kernel-trace --output-format csv -d $d -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --lanes 1 > $d/bench.log 2>&1 || { echo PMC_FAILED; tail -20 $d/bench.log; exit 1; }
python3 tools/sq_summary.py $d/run_counter_collection.csv | grep -E "k_hist|k_scatter|k_ntt_pass<0, 0>|k_bitsum|k_accum"
