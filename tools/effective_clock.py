#!/usr/bin/env python3
"""Effective shader clock per kernel from a rocprofv3 --pmc run that collected GRBM_GUI_ACTIVE
(MI355X_MICROARCH.md, "DVFS give-back": clock ≈ GRBM_GUI_ACTIVE / 8 XCDs / dispatch wall time;
reliable on dispatches >= ~0.3 ms), plus the VALU activity SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES
(both in quad-cycles) when present.

  python tools/effective_clock.py gpurun_out/r05y/msm/run_counter_collection.csv [--min-ms 0.3]
"""
from __future__ import annotations

import argparse
import collections
import csv
import re


def short(name: str) -> str:
    name = name.replace("plk::(anonymous namespace)::", "")
    name = re.sub(r"^void ", "", name)
    return re.sub(r"\(.*$", "", name)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--min-ms", type=float, default=0.3)
    ap.add_argument("--json", help="also write {kernel: {effective_ghz, valu_per_wave, ...}}")
    a = ap.parse_args()
    disp = collections.defaultdict(dict)  # dispatch id -> counter values, name, duration
    for r in csv.DictReader(open(a.csv)):
        d = disp[r["Dispatch_Id"]]
        d["name"] = short(r["Kernel_Name"])
        d["ms"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        d[r["Counter_Name"]] = float(r["Counter_Value"])
    per = collections.defaultdict(list)
    for d in disp.values():
        if "GRBM_GUI_ACTIVE" in d and d["ms"] >= a.min_ms:
            per[d["name"]].append(d)
    print(f"{'kernel':34s} {'n':>4s} {'avg ms':>8s} {'GHz':>6s} {'valu/wave':>9s}")
    out = {}
    for name, ds in sorted(per.items(), key=lambda kv: -sum(x["ms"] for x in kv[1])):
        ms = sum(x["ms"] for x in ds) / len(ds)
        ghz = sum(x["GRBM_GUI_ACTIVE"] / 8 / (x["ms"] * 1e6) for x in ds) / len(ds)
        v = [x["SQ_ACTIVE_INST_VALU"] / x["SQ_WAVE_CYCLES"] for x in ds if x.get("SQ_WAVE_CYCLES")]
        vs = f"{sum(v) / len(v):9.2f}" if v else f"{'-':>9s}"
        print(f"{name[:34]:34s} {len(ds):4d} {ms:8.3f} {ghz:6.2f} {vs}")
        out[name] = {"dispatches": len(ds), "avg_ms": ms, "effective_ghz": ghz,
                     "valu_per_wave": (sum(v) / len(v)) if v else None}
    if a.json:
        import json
        json.dump({"source": a.csv, "kernels": out}, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
