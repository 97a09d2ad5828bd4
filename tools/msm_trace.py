"""Per-kernel breakdown of a lone-MSM bench run (bench.py --mode msm under rocprofv3
--kernel-trace): the dispatches of the last K MSMs (one MSM = the kernels from one
k_chist / k_hist to the next), averaged per MSM, with the gaps between them.

Usage: python tools/msm_trace.py run_kernel_trace.csv [K]
"""
import collections
import csv
import re
import sys


def name(r):
    m = re.search(r"(k_\w+(<[^>]*>)?)", r["Kernel_Name"])
    return m.group(1) if m else r["Kernel_Name"][:40]


rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
K = int(sys.argv[2]) if len(sys.argv) > 2 else 8
first = [i for i, r in enumerate(rows) if name(r) in ("k_chist", "k_hist", "k_any_nonzero")
         and (i == 0 or name(rows[i - 1]) not in ("k_any_nonzero",))]
starts = first[-K - 1:-1] if len(first) > K else first[:-1]
dur = collections.defaultdict(float)
cnt = collections.Counter()
wall = 0.0
for a, b in zip(starts, starts[1:] + [first[-1]]):
    seg = rows[a:b]
    t0 = int(seg[0]["Start_Timestamp"])
    t1 = max(int(r["End_Timestamp"]) for r in seg)
    wall += (t1 - t0) / 1e3
    for r in seg:
        cnt[name(r)] += 1
        dur[name(r)] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
n = len(starts)
busy = sum(dur.values()) / n
print(f"{n} MSMs: first-to-last dispatch {wall / n:.1f} us per MSM, kernels busy {busy:.1f} us")
for k, c in sorted(cnt.items(), key=lambda kv: -dur[kv[0]]):
    print(f"  {k:28s} {c / n:4.1f}/MSM {dur[k] / n:8.1f} us")
