#!/bin/bash
# Copy the rocprof evidence of tools/gpu_profile.sh from gpurun_out/prof into the tracked
# profiles/ directory under a round tag: bash tools/save_profiles.sh r02
set -e
t=${1:?round tag, e.g. r02}
P=gpurun_out/prof
cp $P/stats/run_kernel_stats.csv profiles/${t}_full_n20_kernel_stats.csv
cp $P/bench_line.json profiles/${t}_full_n20_bench_line.json
cp $P/bd20/breakdown.txt profiles/${t}_full_n20_proof_breakdown.txt
cp $P/bd16/breakdown.txt profiles/${t}_full_n16_proof_breakdown.txt
mkdir -p profiles/${t}_pmc
cp $P/pmc/FETCH_SIZE/run_counter_collection.csv profiles/${t}_pmc/FETCH_SIZE_counter_collection.csv
cp $P/pmc/WRITE_SIZE/run_counter_collection.csv profiles/${t}_pmc/WRITE_SIZE_counter_collection.csv
sed "s#\"source\": \"$P/pmc\"#\"source\": \"profiles/${t}_pmc\"#" $P/pmc_traffic.json > profiles/pmc_traffic.json
echo saved
