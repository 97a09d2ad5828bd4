# Copy the rocprof evidence of tools/gpu_refresh_profiles.sh from gpurun_out/ into the
# tracked profiles/ directory (round-1 names).
set -e
cp gpurun_out/prof/run_kernel_stats.csv profiles/r01_full_n20_kernel_stats.csv
cp gpurun_out/prof/bench_line.json profiles/r01_full_n20_bench_line.json
cp gpurun_out/prof_full/breakdown.txt profiles/r01_full_n20_proof_breakdown.txt
cp gpurun_out/pmc/FETCH_SIZE/run_counter_collection.csv profiles/r01_pmc/FETCH_SIZE_counter_collection.csv
cp gpurun_out/pmc/WRITE_SIZE/run_counter_collection.csv profiles/r01_pmc/WRITE_SIZE_counter_collection.csv
sed 's#"source": "gpurun_out/pmc"#"source": "profiles/r01_pmc"#' gpurun_out/pmc/pmc_traffic.json > profiles/pmc_traffic.json
