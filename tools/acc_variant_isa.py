"""Compile ONE csrc TU (device code only, gfx950) with extra -D flags and print the
instruction mix and the VALU issue cycles of a kernel's largest block — the quick A/B of a
code-generation change before any GPU run (e.g. python tools/acc_variant_isa.py msm.hip
k_accumulateILb0E -DPLK_RX_CHAIN=1).
"""
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "tools"))
import isa_count  # noqa: E402


def mix_of(src: str, kernel: str, flags) -> dict:
    with tempfile.TemporaryDirectory() as d:
        co = Path(d) / "k.co"
        path = Path(src) if "/" in src else ROOT / "dusk-plonk_amd" / "csrc" / src
        cmd = ["/opt/rocm/bin/hipcc", "-std=c++17", "-O3", "--offload-arch=gfx950",
               "--cuda-device-only", "--no-gpu-bundle-output", "-c", str(path),
               f"-I{ROOT / 'include'}", "-o", str(co), *flags]
        subprocess.run(cmd, check=True)
        lines = isa_count._disasm(co)
        blocks = isa_count.kernel_blocks(lines, kernel)
        _, c = max(blocks, key=lambda b: sum(b[1].values()))
        return dict(c)


if __name__ == "__main__":
    src, kernel, *flags = sys.argv[1:]
    m = mix_of(src, kernel, flags)
    tot = sum(m.values())
    print(f"instructions {tot}  v_mad_u64_u32 {m.get('v_mad_u64_u32', 0)}  "
          f"valu_cycles {isa_count.valu_cycles(m):.0f}")
    for op, n in sorted(m.items(), key=lambda x: -x[1])[:16]:
        print(f"  {op:26s}{n}")
