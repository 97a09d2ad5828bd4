"""Instruction counts of a kernel's largest straight-line block, read from the COMPILED
library (the gfx950 code object inside libplk.so), not from a formula.

bench.py reports k_accumulate's loop body this way (`mads_per_point_add`: the
v_mad_u64_u32 count of the mixed addition as compiled). The loop body of a kernel whose hot
loop is one long basic block is its largest block between branches / branch targets.

Usage: python tools/isa_count.py [libplk.so] [kernel substring]
"""
from __future__ import annotations

import collections
import re
import shutil
import subprocess
import sys
import tempfile
from pathlib import Path

LLVM = Path("/opt/rocm/lib/llvm/bin")
ROOT = Path(__file__).resolve().parent.parent


def _code_objects(lib: Path, tmp: Path) -> list[Path]:
    # llvm-objdump --offloading writes the bundles next to its input: work on a copy
    cp = tmp / lib.name
    shutil.copy(lib, cp)
    subprocess.run([str(LLVM / "llvm-objdump"), "--offloading", str(cp)], check=True,
                   capture_output=True, cwd=tmp)
    return sorted(p for p in tmp.iterdir() if "amdgcn" in p.name)


def _disasm(co: Path) -> list[str]:
    r = subprocess.run([str(LLVM / "llvm-objdump"), "-d", "--no-show-raw-insn", "--mcpu=gfx950",
                        str(co)], check=True, capture_output=True, text=True)
    return r.stdout.split("\n")


_FUNC = re.compile(r"^([0-9a-f]+) <(.+)>:$")
_INST = re.compile(r"^\s+([a-z_0-9]+)\b(.*?)(?://\s*([0-9A-F]+):)?")
_TARGET = re.compile(r"<(.+?)\+0x([0-9a-f]+)>")


def kernel_blocks(lines: list[str], pat: str):
    """[(start offset, Counter of opcodes)] of the straight-line blocks of the first function
    whose symbol contains `pat` (split after every branch and at every branch target)."""
    start = None
    for i, l in enumerate(lines):
        m = _FUNC.match(l.strip()) if l and not l.startswith(" ") else None
        if m and pat in m.group(2) and not m.group(2).endswith(".kd"):
            start = i
            break
    if start is None:
        return []
    body = []
    for l in lines[start + 1:]:
        if _FUNC.match(l.strip() or "-") and not l.startswith(" "):
            break
        m = re.match(r"^\s+(\S+)(.*?)\s*//\s*([0-9A-F]+):", l)
        if m:
            body.append((int(m.group(3), 16), m.group(1), m.group(2)))
    if not body:
        return []
    base = body[0][0]
    targets = set()
    for off, op, rest in body:
        if op.startswith("s_cbranch") or op == "s_branch":
            t = _TARGET.search(rest)
            if t:
                targets.add(base + int(t.group(2), 16))
    blocks, cur, cur_start = [], collections.Counter(), body[0][0]
    for off, op, rest in body:
        if off in targets and cur:
            blocks.append((cur_start, cur))
            cur, cur_start = collections.Counter(), off
        cur[op] += 1
        if op.startswith("s_cbranch") or op in ("s_branch", "s_setpc_b64", "s_endpgm"):
            blocks.append((cur_start, cur))
            cur, cur_start = collections.Counter(), off + 4
    if cur:
        blocks.append((cur_start, cur))
    return blocks


def largest_block(lib: Path, pat: str) -> dict | None:
    """{'instructions', 'v_mad_u64_u32', 'kernel'} of the largest block of kernel `pat`."""
    with tempfile.TemporaryDirectory() as d:
        for co in _code_objects(Path(lib), Path(d)):
            lines = _disasm(co)
            blocks = kernel_blocks(lines, pat)
            if blocks:
                _, c = max(blocks, key=lambda b: sum(b[1].values()))
                return {"kernel": pat, "instructions": sum(c.values()),
                        "v_mad_u64_u32": sum(v for k, v in c.items() if k.startswith("v_mad_u64_u32")),
                        "top": c.most_common(8), "mix": dict(c)}
    return None


if __name__ == "__main__":
    lib = Path(sys.argv[1]) if len(sys.argv) > 1 else ROOT / "dusk-plonk_amd" / "libplk.so"
    pat = sys.argv[2] if len(sys.argv) > 2 else "k_accumulateILb0E"
    print(largest_block(lib, pat))


# Issue cost of a VALU wave-instruction on one SIMD, in cycles, measured chip-wide at 4 waves
# per SIMD (tools/ubench_issue.hip, profiles/r03_ubench_issue.txt): 64-bit and 32-bit
# multiply forms issue at about half the rate of 32-bit integer ALU instructions.
ISSUE_CYCLES = {"v_mad_u64_u32": 4.53, "v_lshrrev_b64": 4.24, "v_lshlrev_b64": 4.24,
                "v_ashrrev_i64": 4.24, "v_lshl_add_u64": 4.36, "v_mul_lo_u32": 4.26,
                "v_mul_hi_u32": 4.26}
ISSUE_CYCLES_VALU32 = 2.30  # v_and / v_add / v_ashrrev measured 2.29-2.32


def valu_cycles(mix: dict) -> float:
    """SIMD issue cycles of one pass of a block with opcode counts `mix`: VALU instructions at
    their measured costs (prefix match on the mnemonic, e.g. v_add_u32_e32), scalar, memory and
    LDS instructions excluded (they issue on other units)."""
    cyc = 0.0
    for op, n in mix.items():
        if not op.startswith("v_"):
            continue
        base = next((c for k, c in ISSUE_CYCLES.items() if op.startswith(k)), ISSUE_CYCLES_VALU32)
        cyc += n * base
    return cyc
