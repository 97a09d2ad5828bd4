"""Generates tests/golden/proof_2_20.npz: the headline workload's proof pinned by the
restated CPU prover (oracle/plk_prover_oracle.c, which follows PlonkKey::compile and
Prover::create_proof, /root/reference/src/key.rs:63-327 and src/prover.rs:67-474).

The circuit is bench.py's bench_circuit at n = 2^20 (Plonk::initialize + a chain of
2^20 - 15 gates x' = x*y + x from SplitMix64 seed 77 + one public input: m = n - 8 gates),
the SRS the oracle's [tau^i]G1 for tau = tests/test_prover_oracle.tau_for(0x5EED) over the
trimmed length n + 8, label b"bench", blinding seed 7 — the inputs of
test_prover_oracle.test_gpu_proof_equals_oracle_bench_2_16 at the bench's own size. Stored:
the 15 verifier-key commitments, the 11 proof commitments, the 16 evaluations, the public
input and the proof's SCALE bytes (make_proof_scale.scale_bytes, an independent restatement
of the assumed encoding). About 2 KB; the CPU proof takes minutes, so it is generated once
here and committed. Run from the repo root:
    python3 tests/golden/make_proof_2_20.py [threads]
"""
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "tests"), str(ROOT / "tests" / "golden"), str(ROOT / "oracle")]

LOG_N = 20
CHAIN_SEED, BLIND_SEED, TAU_SEED, LABEL = 77, 7, 0x5EED, b"bench"
OUT = Path(__file__).with_name("proof_2_20.npz")


def circuit():
    from test_prover_oracle import bench_chain, build
    return build(bench_chain((1 << LOG_N) - 15, CHAIN_SEED))


def make(threads: int = 0):
    import oracle_lib
    from make_proof_scale import scale_bytes
    from test_prover_oracle import n_trim, tau_for
    orc = oracle_lib.load()
    tau_limbs, _ = tau_for(TAU_SEED)
    cs = circuit()
    gates, wit = cs.export()
    assert gates.shape[0] == (1 << LOG_N) - 8
    t0 = time.time()
    srs = orc.srs(tau_limbs, n_trim(gates.shape[0]), threads)
    t1 = time.time()
    res = orc.prove(gates, wit, srs, LABEL, BLIND_SEED, threads)
    t2 = time.time()
    print(f"srs {t1 - t0:.1f} s, prove {t2 - t1:.1f} s", flush=True)
    return res, scale_bytes(res["comms"], res["evals"])


if __name__ == "__main__":
    threads = int(sys.argv[1]) if len(sys.argv) > 1 else int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    res, data = make(threads)
    np.savez(OUT, vk=res["vk"], comms=res["comms"], evals=res["evals"], pis=res["pis"],
             scale=np.frombuffer(data, dtype=np.uint8),
             meta=np.array([LOG_N, CHAIN_SEED, BLIND_SEED, TAU_SEED], dtype=np.uint64))
    print(f"wrote {OUT.name} ({len(data)} SCALE bytes)")
