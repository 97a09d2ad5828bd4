"""Directly measured concurrent CPU proof throughput at n = 2^20: P
independent restated-reference proofs (tests/oracle_worker.py: oracle/plk_prover_oracle.c,
one process and one thread each) of bench.py's 2^20 circuit, started together on the
GPU box's CPU share, timed per process. Prints a heartbeat every 30 s (the runs take minutes)
and writes the JSON summary to the path given.

Usage (GPU box, after the library is built): python3 tools/cpu_node_n20.py out.json [P]
"""
import json
import os
import subprocess
import sys
import tempfile
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "tests")]


def main():
    out = Path(sys.argv[1])
    import bench
    import oracle_lib
    from dusk_plonk_amd.prover import Plonk
    from test_prover_oracle import n_trim, tau_for
    share = bench.cpu_share()
    procs = int(sys.argv[2]) if len(sys.argv) > 2 else share["available"]
    k = 20
    n = 1 << k
    orc = oracle_lib.load()
    cs = bench.bench_circuit(Plonk, n - 15, 77)
    gates, wit = cs.export()
    tau, _ = tau_for(0x5EED)
    t0 = time.time()
    srs = orc.srs(tau, n_trim(gates.shape[0]), share["available"])
    print(f"srs {time.time() - t0:.1f} s", flush=True)
    # the verifier key's commitments: one full compile + proof on the whole share first
    # (its timing is the single-proof latency on `available` threads)
    t0 = time.time()
    res = orc.prove(gates, wit, srs, b"cpu-node", 5, share["available"])
    lat = time.time() - t0
    tm = res["timing_ns"].astype(np.float64) / 1e9
    print(f"latency proof on {share['available']} threads: create_proof {tm[6]:.1f} s", flush=True)
    with tempfile.TemporaryDirectory() as d:
        f = Path(d) / "inputs.npz"
        np.savez(f, gates=gates, witness=wit, srs=srs, vk=res["vk"])
        env = dict(os.environ, OMP_NUM_THREADS="1")
        start = time.time()
        ps = [subprocess.Popen([sys.executable, str(ROOT / "tests" / "oracle_worker.py"), str(f), "1",
                                str(100 + i)], stdout=subprocess.PIPE, text=True, env=env)
              for i in range(procs)]
        while any(p.poll() is None for p in ps):
            time.sleep(30)
            print(f"  {time.time() - start:.0f} s, {sum(p.poll() is not None for p in ps)}/{procs} done",
                  flush=True)
        outs = []
        for p in ps:
            o, _ = p.communicate()
            if p.returncode != 0:
                raise SystemExit(f"worker failed ({p.returncode})")
            outs.append(json.loads(o.strip().splitlines()[-1]))
    cp = [o["create_proof_s"] for o in outs]
    window = max(o["end"] for o in outs) - min(o["prove_start"] for o in outs)
    summary = {
        "what": "MEASURED concurrent throughput of the restated reference CPU prover "
                "(oracle/plk_prover_oracle.c) at n = 2^20 on bench.py's circuit: independent "
                "single-thread proofs, one per core of the GPU box's CPU share, started together",
        "n": n, "procs": procs, "host": share,
        "create_proof_s": cp,
        "rate_sum_constraints_per_s": sum(n / t for t in cp),
        "window_s": window, "window_constraints_per_s": procs * n / window,
        "per_core_constraints_per_s": sum(n / t for t in cp) / procs,
        "node_projection_constraints_per_s": sum(n / t for t in cp) / procs * share["machine_cores"],
        "latency_threads": share["available"], "latency_create_proof_s": float(tm[6]),
        "latency_phases_s": {"msm": float(tm[1]), "ntt": float(tm[2]),
                             "quotient_loop": float(tm[3]), "grand_product": float(tm[4]),
                             "openings": float(tm[5])},
        "latency_wall_incl_compile_s": lat,
    }
    out.write_text(json.dumps(summary, indent=1))
    print(json.dumps(summary), flush=True)


if __name__ == "__main__":
    main()
