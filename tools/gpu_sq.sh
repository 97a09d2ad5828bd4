# SQ issue/stall counters for the prover kernels (one --pmc pass, kernel trace only)
set -o pipefail
export TMPDIR=/tmp
d=gpurun_out/sq
rm -rf $d; mkdir -p $d
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $d -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --lanes 1 > $d/bench.log 2>&1 || { echo PMC_FAILED; tail -20 $d/bench.log; exit 1; }
python3 tools/sq_summary.py $d/run_counter_collection.csv
