"""Per-proof kernel breakdown of a rocprofv3 kernel trace of bench.py (full-prover mode):
the last proof's window starts at its k_gather_wires launch."""
import collections
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "k_gather_wires" in r["Kernel_Name"]]
seg = rows[idx[-1]:]
t0 = int(seg[0]["Start_Timestamp"])
t1 = max(int(r["End_Timestamp"]) for r in seg)
agg, cnt = collections.defaultdict(float), collections.Counter()
for r in seg:
    m = re.search(r"(k_\w+(<[^>]*>)?)", r["Kernel_Name"])
    n = m.group(1) if m else r["Kernel_Name"][:40]
    agg[n] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    cnt[n] += 1
busy = sum(agg.values())
print(f"proof window {(t1 - t0) / 1e6:.2f} ms, kernels busy {busy:.2f} ms")
for k, v in sorted(agg.items(), key=lambda x: -x[1]):
    if v > 0.05:
        print(f"  {k:42s} {cnt[k]:4d} {v:8.2f} ms")
