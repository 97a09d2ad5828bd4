#!/usr/bin/env python3
"""Interleaved A/B of library variants and bench settings on one GPU box (round 5: replaces
the per-experiment tools/gpu_r0*.sh scripts).

  python tools/ab.py --out gpurun_out/ab.jsonl --reps 2 \\
      --lib base=libplk-base.so --lib new=libplk.so \\
      --args "--log-n 20 --steps 10" --args "--mode msm --log-n 20 --steps 30" \\
      [--env KEY=VALUE ...] [--tests tests/test_msm_gpu.py]

For every repetition, every args set and every variant (in that nesting, so the variants of
one setting run back to back) it runs `python bench.py <args> --warmup W --no-cpu-baseline`
with PLK_LIB pointing at dusk-plonk_amd/<lib>, under its own timeout, and appends one JSON
line: tag, args, value, ms_per_step, the roofline's point_adds_per_s / frac, proofs checked.
--tests first runs the given -m gpu test files once per variant (parity before timing).
Stops at the first failure (non-zero exit, time limit): nothing more runs on the GPU after it.
"""
from __future__ import annotations

import argparse
import json
import os
import shlex
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--lib", action="append", default=[], help="tag=libfile (dusk-plonk_amd/)")
    ap.add_argument("--args", action="append", default=[])
    ap.add_argument("--env", action="append", default=[], help="KEY=VALUE for every run")
    ap.add_argument("--venv", action="append", default=[],
                    help="tag=KEY=VALUE: an environment-only variant on the default library")
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--timeout", type=int, default=300)
    ap.add_argument("--tests", action="append", default=[])
    a = ap.parse_args()
    variants = []
    for spec in a.lib:
        tag, lib = spec.split("=", 1)
        variants.append((tag, {"PLK_LIB": str(ROOT / "dusk-plonk_amd" / lib)}))
    for spec in a.venv:
        tag, kv = spec.split("=", 1)
        k, v = kv.split("=", 1)
        variants.append((tag, {k: v}))
    if not variants:
        variants = [("default", {})]
    base_env = dict(os.environ)
    for kv in a.env:
        k, v = kv.split("=", 1)
        base_env[k] = v
    out = Path(a.out)
    out.parent.mkdir(parents=True, exist_ok=True)
    for tag, ve in variants:
        for t in a.tests:
            log = out.with_name(f"{out.stem}_tests_{tag}.log")
            cmd = [sys.executable, "-u", "-m", "pytest", *shlex.split(t), "-m", "gpu", "-x", "-q",
                   "--timeout", "300", "--timeout-method", "thread"]
            with open(log, "a") as f:
                r = subprocess.run(["timeout", "-k", "10", str(a.timeout * 2), *cmd], cwd=ROOT,
                                   env={**base_env, **ve}, stdout=f, stderr=subprocess.STDOUT)
            last = log.read_text().strip().splitlines()[-1:] or [""]
            print(f"[ab] tests {tag} {t}: rc {r.returncode} {last[0]}", flush=True)
            if r.returncode != 0:
                return 1
    for rep in range(a.reps):
        for args in a.args:
            for tag, ve in variants:
                cmd = [sys.executable, "bench.py", *args.split(), "--warmup", str(a.warmup),
                       "--no-cpu-baseline", "--no-extras"]
                r = subprocess.run(["timeout", "-k", "10", str(a.timeout), *cmd], cwd=ROOT,
                                   env={**base_env, **ve}, capture_output=True, text=True)
                if r.returncode != 0:
                    print(f"[ab] {tag} {args}: rc {r.returncode}\n{r.stderr[-3000:]}", flush=True)
                    return 1
                d = json.loads(r.stdout.strip().splitlines()[-1])
                roof = d.get("roofline", {})
                rec = {"tag": tag, "rep": rep, "args": args, "value": d["value"],
                       "ms": d["ms_per_step"], "adds_per_s": roof.get("point_adds_per_s"),
                       "frac": roof.get("frac"), "acc_ms": roof.get("avg_launch_ms"),
                       "checked": d.get("proofs_checked", d.get("bit_exact_vs_oracle"))}
                if "dft_ms" in roof:
                    rec.update(dft_ms=roof["dft_ms"], idft_ms=roof["idft_ms"])
                print(json.dumps(rec), flush=True)
                with open(out, "a") as f:
                    f.write(json.dumps(rec) + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
