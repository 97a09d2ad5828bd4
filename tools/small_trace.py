"""Summary for tools/gpu_small_trace.sh: the last single-lane proof's dispatches (count per
kernel, window, busy time) and, for the multi-lane run, the fraction of its last 60 % of wall
time in which at least one kernel was executing."""
import collections
import csv
import re
import sys


def load(p):
    rows = list(csv.DictReader(open(p)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    return rows


def name(r):
    m = re.search(r"(k_\w+(<[^>]*>)?)", r["Kernel_Name"])
    return m.group(1) if m else r["Kernel_Name"][:40]


one = load(sys.argv[1])
idx = [i for i, r in enumerate(one) if "k_gather_wires" in r["Kernel_Name"]]
seg = one[idx[-1]:]
t0 = int(seg[0]["Start_Timestamp"])
t1 = max(int(r["End_Timestamp"]) for r in seg)
cnt, dur = collections.Counter(), collections.defaultdict(float)
for r in seg:
    cnt[name(r)] += 1
    dur[name(r)] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
print(f"single lane: {len(seg)} dispatches in the proof window {(t1 - t0) / 1e3:.0f} us, "
      f"kernels busy {sum(dur.values()):.0f} us")
for k, c in cnt.most_common():
    print(f"  {k:44s} {c:4d} {dur[k]:8.1f} us")
many = load(sys.argv[2])
T0 = int(many[0]["Start_Timestamp"])
T1 = max(int(r["End_Timestamp"]) for r in many)
lo = T0 + 0.4 * (T1 - T0)
iv = sorted((max(int(r["Start_Timestamp"]), lo), int(r["End_Timestamp"])) for r in many
            if int(r["End_Timestamp"]) > lo)
busy, cur_s, cur_e = 0, None, None
for s, e in iv:
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            busy += cur_e - cur_s
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
n = sum(1 for r in many if int(r["Start_Timestamp"]) >= lo)
print(f"multi-lane: last 60 % of the run {(T1 - lo) / 1e3:.0f} us, GPU busy (any kernel) "
      f"{100 * busy / (T1 - lo):.1f} %, {n} dispatches = {n / ((T1 - lo) / 1e9):.0f} /s")
# average number of kernels executing at once over the busy time, and each kernel's share
# of the summed kernel time in the multi-lane window
tot = sum(e - s for s, e in iv)
print(f"multi-lane: mean concurrency over busy time {tot / busy:.2f} kernels")
kt = collections.defaultdict(float)
kc = collections.Counter()
for r in many:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if e > lo:
        kt[name(r)] += (e - max(s, lo))
        kc[name(r)] += 1
for k, v in sorted(kt.items(), key=lambda kv: -kv[1])[:16]:
    print(f"  {k:44s} {kc[k]:6d} {100 * v / tot:5.1f} % of kernel time, avg {v / kc[k] / 1e3:7.1f} us")
