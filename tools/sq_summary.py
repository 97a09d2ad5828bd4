"""Per-kernel averages of the SQ counters of a rocprofv3 --pmc run (tools/recipes.py counters)."""
import collections
import csv
import sys

vals = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(sys.argv[1])):
    name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].split("::")[-1]
    vals[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
for name, cs in sorted(vals.items(), key=lambda kv: -sum(kv[1].get("SQ_WAVE_CYCLES", [0]))):
    avg = {k: sum(v) / len(v) for k, v in cs.items()}
    wc = avg.get("SQ_WAVE_CYCLES", 0) or 1
    print(f"{name[:34]:34s} n={len(cs.get('SQ_WAVE_CYCLES', []))} " + " ".join(
        f"{k.replace('SQ_', '')}={v:.3g}" for k, v in sorted(avg.items())) +
        f"  waitany={avg.get('SQ_WAIT_ANY', 0) / wc:.2f} waitinst={avg.get('SQ_WAIT_INST_ANY', 0) / wc:.2f}"
        f" active={avg.get('SQ_ACTIVE_INST_ANY', 0) / wc:.2f} valu={avg.get('SQ_ACTIVE_INST_VALU', 0) / wc:.2f}")
