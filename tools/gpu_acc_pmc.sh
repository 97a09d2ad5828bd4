# accumulate-variant instruction mix: dynamic VALU/SALU instruction counts and VALU busy
# cycles per kernel (one --pmc pass per counter group, kernel-trace only)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/acc_pmc
rm -rf gpurun_out/acc_pmc/*
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES --output-format csv -d gpurun_out/acc_pmc/a -o run -- ./tools/ubench_acc > gpurun_out/acc_pmc/a.log 2>&1 || { echo PMC_A_FAILED; tail gpurun_out/acc_pmc/a.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d gpurun_out/acc_pmc/b -o run -- ./tools/ubench_acc > gpurun_out/acc_pmc/b.log 2>&1 || { echo PMC_B_FAILED; tail gpurun_out/acc_pmc/b.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob('gpurun_out/acc_pmc/*/run_counter_collection.csv'):
    for r in csv.DictReader(open(f)):
        agg[r['Kernel_Name'][:40]][r['Counter_Name']].append(float(r['Counter_Value']))
for k, d in agg.items():
    print(k, {c: '%.4g' % (sum(v) / len(v)) for c, v in d.items()})
PY
