"""Generates tests/golden/proof_scale.npz: one proof of the restated CPU prover
(oracle/plk_prover_oracle.c) on the `public_sum` circuit of tests/test_prover_oracle.py,
its 11 commitments / 16 evaluations, and its SCALE bytes written by an independent
struct-level restatement of the assumed Proof encoding (include/plk.h plk_proof_encode:
per commitment x[6], y[6] as LE u64 Montgomery limbs + an is_infinity byte; per evaluation
4 LE u64 Montgomery limbs; proof.rs field order). Run from the repo root:
    python3 tests/golden/make_proof_scale.py
"""
import struct
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "tests"), str(ROOT / "oracle")]


def scale_bytes(comms: np.ndarray, evals: np.ndarray) -> bytes:
    out = b""
    for c in comms:
        out += struct.pack("<12Q", *[int(v) for v in c[:12]]) + bytes([int(c[12])])
    for e in evals:
        out += struct.pack("<4Q", *[int(v) for v in e])
    return out


def make():
    import oracle_lib
    from test_prover_oracle import build, n_trim, public_sum, tau_for
    orc = oracle_lib.load()
    tau_limbs, _ = tau_for(105)
    cs = build(public_sum(10, 20, 30))
    gates, wit = cs.export()
    res = orc.prove(gates, wit, orc.srs(tau_limbs, n_trim(gates.shape[0])), b"scale", 5)
    return res["comms"], res["evals"], scale_bytes(res["comms"], res["evals"])


if __name__ == "__main__":
    comms, evals, data = make()
    np.savez(Path(__file__).with_name("proof_scale.npz"), comms=comms, evals=evals,
             scale=np.frombuffer(data, dtype=np.uint8))
    print(f"wrote proof_scale.npz ({len(data)} SCALE bytes)")
