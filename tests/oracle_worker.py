"""One restated-reference CPU proof in its own process (test infrastructure / bench.py's
cpu_baseline leg only): `python tests/oracle_worker.py <inputs.npz> <threads> <seed>` runs
oracle/plk_prover_oracle.c's create_proof on the circuit, witness, SRS and verifier key
stored in <inputs.npz> and prints one JSON line with its phase timings (seconds).

bench.py starts several of these at once to measure the CPU's concurrent proof throughput
(independent proofs, one per core, the way a CPU proof server would use the node). The key's
commitments come in precomputed (vk_in), so each process spends its time in create_proof
rather than in key compilation; the rest of the compile (selector / sigma transforms) still
runs first in every process and is excluded from the timed create_proof phase.
"""
import json
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent))

if __name__ == "__main__":
    import oracle_lib
    path, threads, seed = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    d = np.load(path, allow_pickle=False)
    orc = oracle_lib.load()
    t0 = time.time()
    res = orc.prove(d["gates"], d["witness"], d["srs"], b"cpu-node", seed, threads, vk_in=d["vk"])
    t1 = time.time()
    tm = res["timing_ns"].astype(np.float64) / 1e9
    print(json.dumps({"create_proof_s": float(tm[6]), "compile_s": float(tm[0]),
                      "wall_s": t1 - t0, "start": t0, "end": t1,
                      "prove_start": t1 - float(tm[6])}), flush=True)
