set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 ./tools/ubench_acc > gpurun_out/ubench_acc.log 2>&1 || { echo UBA_FAILED; cat gpurun_out/ubench_acc.log; exit 1; }
cat gpurun_out/ubench_acc.log
cat > /tmp/synth_probe.py <<'PY'
import sys, time
sys.path.insert(0, '.')
from dusk_plonk_amd.prover import Plonk
cs = Plonk(); del cs
for rep in range(4):
    t = time.perf_counter(); cs = Plonk(); cs.synthetic_chain((1 << 20) - 14, 5 + rep); t1 = time.perf_counter(); del cs
    print(f"synth alone {1e3 * (t1 - t):.1f} ms")
PY
timeout -k 10 120 python /tmp/synth_probe.py
nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null || true
