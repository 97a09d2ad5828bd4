"""Per-kernel VGPRs / spills / occupancy from a `-Rpass-analysis=kernel-resource-usage` log."""
import re
import sys


def parse(path):
    out, cur = {}, None
    for line in open(path):
        m = re.search(r"remark: ([^:]+): (.*?) \[-Rpass", line)
        if not m:
            continue
        k, v = m.group(1).strip(), m.group(2).strip()
        if k == "Function Name":
            cur = v
            out[cur] = {}
        elif cur:
            out[cur][k] = v
    return out


if __name__ == "__main__":
    pat = sys.argv[2] if len(sys.argv) > 2 else ""
    for fn, d in parse(sys.argv[1]).items():
        if pat in fn:
            print(f"{fn[:60]:60s} vgpr {d.get('VGPRs')} agpr {d.get('AGPRs')} spill {d.get('VGPRs Spill')} "
                  f"occ {d.get('Occupancy [waves/SIMD]')}")
