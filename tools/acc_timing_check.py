"""k_accumulate: the bench's dispatch-stamped HIP-event averages against the rocprofv3
kernel-trace durations of the same run — the solo proof's launches (the roofline's
`avg_launch_ms`, the last 4 launches of the run) and the timed in-workload ones (before them).
Usage: python tools/acc_timing_check.py run_kernel_trace.csv bench.log"""
import csv
import json
import sys

trace, log = sys.argv[1], sys.argv[2]
d = json.loads([l for l in open(log) if '"metric"' in l][-1])
r = d["roofline"]
rows = [x for x in csv.DictReader(open(trace)) if "k_accumulate" in x["Kernel_Name"]]
rows.sort(key=lambda x: int(x["Start_Timestamp"]))
dur = [(int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) / 1e6 for x in rows]
ns = r["solo"]["launches"]
nw = r["in_workload"]["launches"]
solo = dur[-ns:]
timed = dur[-(nw + ns):-ns]
print(f"bench {d['value'] / 1e6:.2f} M/s")
print(f"solo (roofline avg_launch_ms): events {r['solo']['avg_launch_ms']:.3f} ms over {ns}; "
      f"rocprof {sum(solo) / len(solo):.3f} ms over the run's last {len(solo)}")
print(f"in workload: events {r['in_workload']['avg_launch_ms']:.3f} ms over {nw}; rocprof "
      f"{sum(timed) / len(timed):.3f} ms over the {len(timed)} before them; all launches "
      f"{sum(dur) / len(dur):.3f} ms over {len(dur)} (the --stats average)")
