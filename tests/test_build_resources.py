"""Kernel resource usage of the built library (no GPU needed): every kernel of every TU must
keep its values in registers — no scratch-memory object — except the ones listed here.

Round 5 found an 80-byte stack object in every `k_ntt_pass` instantiation (a run-time branch
assigning `r4_math`'s outputs on both sides: 18 scratch stores and loads per radix-4 step,
≈ 4 % of a transform) and one in `k_ruffini_single`; both were invisible to the parity tests.
The reports are written by `dusk-plonk_amd/build_ext.py` (hipcc
`-Rpass-analysis=kernel-resource-usage`, `build/<tu>.res.txt`); the test is skipped when the
library was built without them.
"""
from __future__ import annotations

import re
from pathlib import Path

import pytest

BUILD = Path(__file__).resolve().parent.parent / "dusk-plonk_amd" / "build"

# k_accumulate<HAS_INF = true, LONE = true>: the lone form for an SRS holding the point at
# infinity spills 2 VGPRs at its 3-wave budget (rare path; the prover never takes it)
ALLOWED = ("k_accumulateILb1ELb1E",)


def _reports():
    return sorted(BUILD.glob("*.res.txt"))


def _parse(path: Path):
    out, cur = {}, None
    for line in path.read_text().splitlines():
        m = re.search(r"remark: +([^:]+): (.*?) \[-Rpass", line)
        if not m:
            continue
        k, v = m.group(1).strip(), m.group(2).strip()
        if k == "Function Name":
            cur = v
            out[cur] = {}
        elif cur is not None:
            out[cur][k] = v
    return out


def test_resource_reports_parse():
    reps = _reports()
    if not reps:
        pytest.skip("library built without resource reports")
    kernels = {}
    for r in reps:
        kernels.update(_parse(r))
    assert any("k_ntt_pass" in k for k in kernels)
    assert any("k_accumulate" in k for k in kernels)
    for name, d in kernels.items():
        assert "ScratchSize [bytes/lane]" in d, name


def test_no_scratch_objects():
    reps = _reports()
    if not reps:
        pytest.skip("library built without resource reports")
    bad = []
    for r in reps:
        for name, d in _parse(r).items():
            scratch = int(d.get("ScratchSize [bytes/lane]", "0"))
            if scratch and not any(a in name for a in ALLOWED):
                bad.append(f"{r.stem}: {name} {scratch} B/lane")
    assert not bad, "kernels with scratch memory:\n" + "\n".join(bad)
