"""bench.py's output contract (the driver parses one JSON line from rank 0): the CLI on the
CPU, and on the GPU the three single-rank modes at small sizes — prove (default), and the
standalone NTT / MSM lines of BASELINE configs[1] / [2], which check their own result
bit-exact against the oracle before printing."""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
CONTRACT = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
            "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config", "roofline")
ROOFLINE = ("bound", "achieved", "peak", "unit", "frac", "traffic")


def run_bench(*args, timeout=100):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, "bench.py", *args], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    return json.loads(lines[0])


def check_contract(d, steps, warmup):
    for k in CONTRACT:
        assert k in d, k
    for k in ROOFLINE:
        assert k in d["roofline"], k
    assert d["value"] > 0 and d["ms_per_step"] > 0
    assert d["n_gpus"] == 1 and d["steps"] == steps and d["warmup"] == warmup
    assert d["higher_is_better"] is True and d["vs_baseline"] is None
    assert "workload" in d["config"]
    assert d["roofline"]["frac"] == pytest.approx(d["roofline"]["achieved"] / d["roofline"]["peak"])


def test_cli_lists_modes():
    p = subprocess.run([sys.executable, "bench.py", "--help"], cwd=ROOT, capture_output=True,
                       text=True, timeout=60)
    assert p.returncode == 0
    for flag in ("--gpus", "--steps", "--warmup", "--mode", "--lanes", "--dist-backend"):
        assert flag in p.stdout
    for mode in ("prove", "hotpath", "ntt", "msm"):
        assert mode in p.stdout


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["ntt", "msm"])
def test_kernel_mode_line_is_bit_exact(mode):
    d = run_bench("--mode", mode, "--log-n", "12", "--steps", "3", "--warmup", "1",
                  "--cpu-threads", "4")
    check_contract(d, 3, 1)
    assert d["unit"] == "points/s" and d["config"]["log_n"] == 12
    assert d["bit_exact_vs_oracle"] is True
    cb = d["cpu_baseline"]
    assert cb["kind"] == "port" and cb["cores"] == 4 and cb["value"] > 0


@pytest.mark.gpu
def test_prove_mode_line():
    d = run_bench("--log-n", "12", "--steps", "2", "--warmup", "1", "--lanes", "2",
                  "--no-cpu-baseline")
    check_contract(d, 2, 1)
    assert d["unit"] == "constraints/s" and d["scaling"] == "weak"
    # value counts every lane's proof: n * steps * lanes / time
    assert d["value"] == pytest.approx(4096 * 2 * 2 / (d["ms_per_step"] * 2e-3), rel=1e-6)
