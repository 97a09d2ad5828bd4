#!/usr/bin/env python3
"""Per-kernel summary of a rocprofv3 kernel trace in its default rocpd (SQLite) output, the
form ROCm 7's rocprofv3 writes (`<dir>/run_results.db`): calls, total / average / min / max
duration (us) per kernel (the --stats summary), optionally only the dispatches after the
first `--skip` ms of kernel activity (warmup and setup), plus the last `--window` dispatches
in time order (one step's kernels).

  python tools/rocpd_summary.py gpurun_out/r05b/prof_parts8/run_results.db [--skip-kernel k_srs]
"""
from __future__ import annotations

import argparse
import re
import sqlite3
from collections import defaultdict


def short(name: str) -> str:
    name = name.replace("plk::(anonymous namespace)::", "")
    name = re.sub(r"^void ", "", name)
    name = re.sub(r"\(.*$", "", name)            # argument list
    return name


def load(db: str):
    c = sqlite3.connect(db)
    rows = c.execute("select name, start, end from kernels order by start").fetchall()
    return [(short(n), s, e) for n, s, e in rows]


def summarize(rows):
    agg = defaultdict(list)
    for n, s, e in rows:
        agg[n].append((e - s) / 1e3)
    out = []
    for n, d in agg.items():
        out.append((n, len(d), sum(d), sum(d) / len(d), min(d), max(d)))
    out.sort(key=lambda r: -r[2])
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--after", default="", help="only dispatches after the LAST dispatch of "
                    "this kernel (substring), e.g. the setup kernels")
    ap.add_argument("--window", type=int, default=0, help="print the last N dispatches")
    a = ap.parse_args()
    rows = load(a.db)
    if a.after:
        idx = max((i for i, r in enumerate(rows) if a.after in r[0]), default=-1)
        rows = rows[idx + 1:]
    tot = sum(e - s for _, s, e in rows) / 1e3
    print(f"{len(rows)} dispatches, {tot:.1f} us of kernel time")
    print(f"{'kernel':60s} {'calls':>6s} {'total us':>10s} {'avg us':>9s} {'min':>8s} {'max':>8s}")
    for n, k, t, avg, mn, mx in summarize(rows):
        print(f"{n[:60]:60s} {k:6d} {t:10.1f} {avg:9.1f} {mn:8.1f} {mx:8.1f}")
    if a.window:
        w = rows[-a.window:]
        t0 = w[0][1]
        print(f"\nlast {len(w)} dispatches (start offset us, duration us):")
        for n, s, e in w:
            print(f"  {(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  {n[:70]}")


if __name__ == "__main__":
    main()
