"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE runs into profiles/pmc_traffic.json.

Usage: python tools/pmc_summary.py <dir with FETCH_SIZE/ and WRITE_SIZE/ subdirs> <out.json>
Counters are per dispatch in KB (TCC EA requests); we report their per-launch average.
Per MI355X_MICROARCH.md §HBM, FETCH_SIZE reads 1/2 of a wide coalesced 16-B/lane stream on
gfx950; our dominant kernel is a random 96-B gather, a pattern the guide calls
uncalibrated, so `hbm_bytes_per_launch` is the raw (FETCH + WRITE) * 1024 and
`hbm_bytes_per_launch_stream_corrected` doubles FETCH for comparison.
"""
import collections
import csv
import json
import sys
from pathlib import Path

src, out = Path(sys.argv[1]), Path(sys.argv[2])
per = collections.defaultdict(dict)
for counter in ("FETCH_SIZE", "WRITE_SIZE"):
    f = src / counter / "run_counter_collection.csv"
    vals = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        vals[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    for k, v in vals.items():
        per[k][counter] = sum(v) / len(v)
        per[k][counter + "_last"] = v[-1]
        per[k]["launches"] = len(v)
kernels = {}
for k, d in per.items():
    fe, wr = d.get("FETCH_SIZE", 0.0), d.get("WRITE_SIZE", 0.0)
    kernels[k] = {
        "launches": d["launches"], "fetch_kb": fe, "write_kb": wr,
        "hbm_bytes_per_launch": (fe + wr) * 1024,
        "hbm_bytes_per_launch_stream_corrected": (2 * fe + wr) * 1024,
        # the last dispatch of the run (bench.py: the proof's opening-commit batch, the
        # launch its roofline `achieved` is computed for)
        "hbm_bytes_last_launch": (d.get("FETCH_SIZE_last", 0.0) + d.get("WRITE_SIZE_last", 0.0)) * 1024,
    }
json.dump({"source": str(src), "kernels": kernels}, open(out, "w"), indent=1, sort_keys=True)
print(f"wrote {out} ({len(kernels)} kernels)")
