#!/usr/bin/env python3
"""Named GPU measurement recipes (round 6: replaces the per-call tools/gpu_r05_*.sh scripts,
which were one-off wrappers around tools/ab.py, pytest, bench.py and rocprofv3).

  /usr/local/graft/bin/gpurun --timeout 1200 -- python tools/recipes.py <recipe> [options]
  python tools/recipes.py --list

Every step runs under its own time limit (`timeout -k 10`), writes under gpurun_out/<recipe>/
(or --out), and the first failure (non-zero exit, time limit) ends the recipe: nothing more
runs on the GPU after it. rocprofv3 steps put the program itself after `--` (python3
bench.py ...), with TMPDIR=/tmp, and collect counters only with --kernel-trace (one --pmc
pass per counter). Options:
  --lib tag=file / --venv tag=KEY=VALUE / --args "..." / --reps N / --tests "..."
      for recipe "ab" (passed to tools/ab.py; the round-5 A/B scripts were all of this form)
  --sizes "12 14 16 18 20"  for recipe "sizes"
  --parts "1 2 4 8"         for recipe "parts"
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
PY = sys.executable


class Fail(RuntimeError):
    pass


def run(cmd: list, limit: int, out: Path | None = None, append: bool = False, kill: bool = False):
    """One GPU step under its own time limit; stdout to `out` (stderr beside it)."""
    env = dict(os.environ, TMPDIR="/tmp")
    pre = ["timeout", "-s", "KILL", str(limit)] if kill else ["timeout", "-k", "10", str(limit)]
    print(f"[recipe] {' '.join(shlex.quote(c) for c in cmd)}", flush=True)
    if out is None:
        r = subprocess.run(pre + cmd, cwd=ROOT, env=env)
    else:
        out.parent.mkdir(parents=True, exist_ok=True)
        with open(out, "a" if append else "w") as f, open(out.with_suffix(".err"), "a") as e:
            r = subprocess.run(pre + cmd, cwd=ROOT, env=env, stdout=f, stderr=e)
    if r.returncode != 0:
        if out is not None:
            err = out.with_suffix(".err").read_text().splitlines()[-20:]
            print("\n".join(err), flush=True)
        raise Fail(f"step failed (rc {r.returncode}): {cmd}")


def tests(o: Path, args: str = "tests", limit: int = 900):
    run([PY, "-u", "-m", "pytest", *shlex.split(args), "-m", "gpu", "-x", "-v", "--timeout", "300",
         "--timeout-method", "thread"], limit, o / "tests.log")


def smoke(o: Path):
    run([PY, "-c", "import __graft_entry__ as g; g.smoke()"], 300, o / "smoke.log")


def bench(o: Path, name: str, args: str, limit: int = 400, append: bool = False):
    run([PY, "bench.py", *shlex.split(args)], limit, o / f"{name}.jsonl", append=append)


def trace(o: Path, name: str, args: str, limit: int = 600):
    """rocprofv3 --kernel-trace --stats of one bench command (per-kernel average durations)."""
    run(["rocprofv3", "--kernel-trace", "--stats", "--output-format", "csv", "-d", str(o / name),
         "-o", "run", "--", "python3", "bench.py", *shlex.split(args)], limit, o / f"{name}.json")


def pmc(o: Path, name: str, counters: str, args: str, limit: int = 600):
    """One --pmc pass (kernel trace only) per entry of `counters` (';'-separated groups)."""
    for group in counters.split(";"):
        tag = group.split()[0]
        run(["rocprofv3", "--pmc", *group.split(), "--kernel-trace", "--output-format", "csv",
             "-d", str(o / name / tag), "-o", "run", "--", "python3", "bench.py", *shlex.split(args)],
            limit, o / f"{name}_{tag}.json", kill=True)


def tool(o: Path, out: str, *args):
    run([PY, *args], 120, o / out)


SQ = ("SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY "
      "SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE")


def r_refresh(o, a):
    """Round-end evidence (round 5's gpu_r05_final / gpu_r05_k / gpu_r05_b): every -m gpu test,
    smoke, the default line as the driver runs it, the default command under --kernel-trace
    --stats and one FETCH_SIZE / WRITE_SIZE pass each (-> pmc_traffic.json), the single-lane
    2^20 and 2^16 proof traces for the per-kernel breakdown."""
    tests(o, "tests", 1100)
    smoke(o)
    bench(o, "bench_default", "--steps 20 --warmup 5", 600)
    trace(o, "prof", "--no-cpu-baseline --no-extras")
    pmc(o, "pmc", "FETCH_SIZE;WRITE_SIZE", "--no-cpu-baseline --no-extras")
    tool(o, "pmc_summary.txt", "tools/pmc_summary.py", str(o / "pmc"), str(o / "pmc_traffic.json"))
    for k in (20, 16):
        trace(o, f"bd{k}", f"--log-n {k} --lanes 1 --steps 2 --warmup 1 --no-cpu-baseline --no-extras")
        tool(o, f"bd{k}.txt", "tools/trace_breakdown.py", str(o / f"bd{k}" / "run_kernel_trace.csv"))


def r_configs(o, a):
    """BASELINE configs[1] / [2] (round 5's gpu_configs.sh / gpu_r05_l): standalone NTT and MSM
    lines at 2^20 (bit-exact vs the oracle, CPU baseline) with kernel traces and FETCH / WRITE
    passes, plus NTT 2^23 and MSM 2^16, and the 8-part bucket split of the 2^20 MSM."""
    for m in ("ntt", "msm"):
        trace(o, f"prof_{m}", f"--mode {m} --log-n 20 --steps 10 --warmup 2 --no-cpu-baseline", 300)
        pmc(o, f"pmc_{m}", "FETCH_SIZE;WRITE_SIZE",
            f"--mode {m} --log-n 20 --steps 10 --warmup 2 --no-cpu-baseline", 120)
        out = o / f"pmc_traffic_{m}20.json"
        tool(o, f"pmc_{m}_summary.txt", "tools/pmc_summary.py", str(o / f"pmc_{m}"), str(out))
        # bytes per unit = all launches / the transforms (dft + idft per step) or MSMs of the run
        d = json.loads(out.read_text())
        d["units"] = (10 + 2) * (2 if m == "ntt" else 1)
        out.write_text(json.dumps(d, indent=1, sort_keys=True))
    for m, k in (("ntt", 20), ("msm", 20), ("ntt", 23), ("msm", 16)):
        bench(o, "lines", f"--mode {m} --log-n {k} --steps 10 --warmup 2", 300, append=True)
    bench(o, "lines", "--mode msm --log-n 20 --steps 20 --warmup 3 --no-cpu-baseline --bucket-parts 8",
          300, append=True)


def r_sizes(o, a):
    """Constraints/s at 2^12 .. 2^20 (round 5's gpu_r05_l / gpu_size_sweep.sh), default lanes,
    every lane's last proof re-proved and byte-compared."""
    for k in a.sizes.split():
        bench(o, "sizes", f"--log-n {k} --steps 10 --warmup 3 --no-cpu-baseline --no-extras", 400,
              append=True)


def r_parts(o, a):
    """The 2^20 MSM as G bucket-range parts on one GPU, each timed (round 5's gpu_r05_a /
    gpu_r05_b), with a kernel trace of G = 1 and the largest G."""
    for p in a.parts.split():
        bench(o, "parts", f"--mode msm --log-n 20 --steps 20 --warmup 3 --no-cpu-baseline "
                          f"--bucket-parts {p}", 300, append=True)
    for p in (a.parts.split()[0], a.parts.split()[-1]):
        trace(o, f"prof_parts{p}", f"--mode msm --log-n 20 --steps 10 --warmup 2 --no-cpu-baseline "
                                   f"--bucket-parts {p}", 300)


def r_counters(o, a):
    """SQ issue / stall counters and the effective clock (round 5's gpu_r05_y / gpu_r05_ab /
    gpu_sq*.sh): a single-lane 2^20 proof, the lone 2^20 MSM and the 2^20 / 2^23 NTT, one --pmc
    pass each (7 SQ + 1 GRBM counters)."""
    runs = {"proof": "--steps 1 --warmup 1 --no-cpu-baseline --no-extras --lanes 1",
            "msm": "--mode msm --log-n 20 --steps 5 --warmup 1 --no-cpu-baseline",
            "ntt20": "--mode ntt --log-n 20 --steps 10 --warmup 2 --no-cpu-baseline",
            "ntt23": "--mode ntt --log-n 23 --steps 10 --warmup 2 --no-cpu-baseline"}
    for name, args in runs.items():
        pmc(o, f"sq_{name}", SQ, args, 240)
        csv = o / f"sq_{name}" / "SQ_WAVE_CYCLES" / "run_counter_collection.csv"
        tool(o, f"sq_{name}.txt", "tools/sq_summary.py", str(csv))
        tool(o, f"clock_{name}.txt", "tools/effective_clock.py", str(csv), "--min-ms", "0.05")


def r_ab(o, a):
    """Interleaved A/B of library variants (--lib, built with build_ext.py <v>[:tu] -D...) and/or
    environment variants (--venv) over bench settings (--args), parity tests first (--tests):
    tools/ab.py. Every round-5 gpu_r05_<x>.sh A/B was one or two of these (tools/README.md maps
    them)."""
    cmd = [PY, "-u", "tools/ab.py", "--out", str(o / "ab.jsonl"), "--reps", str(a.reps)]
    for flag, vals in (("--lib", a.lib), ("--venv", a.venv), ("--args", a.args), ("--tests", a.tests),
                       ("--env", a.env)):
        for v in vals:
            cmd += [flag, v]
    run(cmd, a.limit)


def r_check(o, a):
    """Round 6 (tools/gpu_r06_b.sh): the line's new fields (msm_shard, n_2_16, build_id), the
    bucket-split sharded prover, then the default line."""
    tests(o, "tests/test_bench.py tests/test_ntt_gpu.py::test_idft_multipass_identity_rows "
             "tests/test_parallel.py::test_sharded_prover_bucket_split "
             "tests/test_parallel.py::test_sharded_prover_bucket_split_refused_small_srs "
             "tests/test_parallel.py::test_sharded_prover_2_20_bucket_split_equals_fixture", 900)
    bench(o, "bench_default", "--steps 20 --warmup 5", 600)


def r_shardprobe(o, a):
    """One rank's share of a bucket-split sharded 2^20 proof on ONE GPU (tools/shard_rank_probe.py:
    the all-gather emulated, every kernel of the rank as on a node) at G = 2, 4, 8 (ranks 0 and
    G - 1), beside an unsharded lane; a kernel trace of rank 0 of 8 for the per-kernel breakdown."""
    for g in (2, 4, 8):
        for r in sorted({0, g - 1}):
            run([PY, "tools/shard_rank_probe.py", "--world", str(g), "--rank", str(r), "--proofs", "4"],
                400, o / "probe.jsonl", append=True)
    run(["rocprofv3", "--kernel-trace", "--stats", "--output-format", "csv", "-d", str(o / "trace8"),
         "-o", "run", "--", "python3", "tools/shard_rank_probe.py", "--world", "8", "--rank", "0",
         "--proofs", "2"], 400, o / "trace8.json")
    tool(o, "trace8.txt", "tools/trace_breakdown.py", str(o / "trace8" / "run_kernel_trace.csv"))


RECIPES = {"refresh": r_refresh, "configs": r_configs, "sizes": r_sizes, "parts": r_parts,
           "counters": r_counters, "ab": r_ab, "check": r_check, "shardprobe": r_shardprobe}


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("recipe", nargs="?", choices=sorted(RECIPES))
    ap.add_argument("--list", action="store_true")
    ap.add_argument("--out", default=None)
    ap.add_argument("--lib", action="append", default=[])
    ap.add_argument("--venv", action="append", default=[])
    ap.add_argument("--args", action="append", default=[])
    ap.add_argument("--tests", action="append", default=[])
    ap.add_argument("--env", action="append", default=[],
                    help="KEY=VALUE for every run of recipe ab (e.g. PLK_LIB_ANY_SRC=1 for a library "
                         "built from another tree)")
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--limit", type=int, default=1100)
    ap.add_argument("--sizes", default="12 14 16 18 20")
    ap.add_argument("--parts", default="1 2 4 8")
    a = ap.parse_args()
    if a.list or not a.recipe:
        for k, f in sorted(RECIPES.items()):
            print(f"{k:9s} {' '.join(f.__doc__.split())}")
        return 0
    o = Path(a.out) if a.out else ROOT / "gpurun_out" / a.recipe
    o.mkdir(parents=True, exist_ok=True)
    try:
        RECIPES[a.recipe](o, a)
    except Fail as e:
        print(f"[recipe] {a.recipe}: {e}", flush=True)
        return 1
    (o / "done.json").write_text(json.dumps({"recipe": a.recipe, "ok": True}) + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
