"""Instruction mix of the big basic blocks of one kernel in a hipcc -S listing.

Usage: python tools/isa_stats.py <file.s> <symbol substring> [min_block_len]
"""
import collections
import re
import sys

src, pat = sys.argv[1], sys.argv[2]
minlen = int(sys.argv[3]) if len(sys.argv) > 3 else 300
lines = open(src).read().split("\n")
start = next(i for i, l in enumerate(lines) if l.startswith("_Z") and pat in l and l.split(";")[0].rstrip().endswith(":"))
end = next(i for i in range(start, len(lines)) if "s_endpgm" in lines[i])
block, name = [], "entry"
def flush():
    if len(block) >= minlen:
        c = collections.Counter(block)
        mad = sum(v for k, v in c.items() if k.startswith("v_mad_u64_u32"))
        print(f"{name}: {len(block)} instr, {mad} mad")
        print("   ", ", ".join(f"{k} {v}" for k, v in c.most_common(22)))
for l in lines[start + 1:end + 1]:
    t = l.strip()
    if re.match(r"^\.LBB\S*:", t):
        flush()
        block, name = [], t
        continue
    if not t or t.startswith((".", ";")):
        continue
    block.append(t.split()[0])
flush()
