"""k_accumulate: the bench's HIP-event average vs the rocprofv3 kernel-trace durations of
the same run (all launches, and the 160 timed ones: lanes x steps x 4 batches)."""
import csv
import json
import sys

trace, log = sys.argv[1], sys.argv[2]
d = json.loads([l for l in open(log) if '"metric"' in l][-1])
r = d["roofline"]
rows = [x for x in csv.DictReader(open(trace)) if "k_accumulate" in x["Kernel_Name"]]
rows.sort(key=lambda x: int(x["Start_Timestamp"]))
dur = [(int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) / 1e6 for x in rows]
n = r["launches"]
timed = dur[-(n + 4):-4]  # the solo proof (4 launches) follows the timed region
print(f"bench {d['value'] / 1e6:.2f} M/s  events avg {r['avg_launch_ms']:.3f} ms over {n}; "
      f"rocprof all {sum(dur) / len(dur):.3f} ms over {len(dur)}, timed {sum(timed) / len(timed):.3f} ms; "
      f"solo {r['solo']['avg_launch_ms']:.3f}")
