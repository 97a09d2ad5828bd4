"""Directly timed restated reference CPU prover (oracle/plk_prover_oracle.c) on the bench
circuit at n = 2^k — no extrapolation: key compile + one full create_proof, timed by phase,
on this host's cores (OMP threads = --threads or OMP_NUM_THREADS). Test/measurement
infrastructure only (the checker, never the product path). Prints one JSON line.

usage: python3 tools/cpu_full_proof.py [--log-n 20] [--threads N]
"""
import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "tests")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--log-n", type=int, default=20)
    ap.add_argument("--threads", type=int, default=0)
    a = ap.parse_args()
    import oracle_lib
    import bench
    from dusk_plonk_amd.prover import Plonk
    k, n = a.log_n, 1 << a.log_n
    threads = a.threads or int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or os.cpu_count()
    orc = oracle_lib.load()
    import threading
    t_start = time.perf_counter()

    def heartbeat():  # the C calls run minutes without output
        while True:
            time.sleep(30)
            print(f"[cpu_full_proof] running {time.perf_counter() - t_start:.0f} s",
                  file=sys.stderr, flush=True)
    threading.Thread(target=heartbeat, daemon=True).start()
    cs = bench.bench_circuit(Plonk, n - 15, 77)
    gates, wit = cs.export()
    trim = (1 << (gates.shape[0] + 6 - 1).bit_length()) + 8
    t0 = time.perf_counter()
    srs = orc.srs(bench.bench_tau(), trim, threads)
    t_srs = time.perf_counter() - t0
    t0 = time.perf_counter()
    res = orc.prove(gates, wit, srs, b"cpu-full", 5, threads)
    wall = time.perf_counter() - t0
    tm = res["timing_ns"].astype(np.float64) / 1e9
    names = ["key_compile", "msm", "ntt", "quotient_loop", "grand_product",
             "linearisation_openings", "create_proof", "transcript"]
    print(json.dumps({
        "what": "restated reference CPU prover (oracle/plk_prover_oracle.c), one full "
                "create_proof at n = 2^%d on the bench circuit (1 public input), timed directly" % k,
        "n": n, "m": int(gates.shape[0]), "threads": threads, "host": bench.host_info(),
        "create_proof_s": float(tm[6]), "constraints_per_s": n / float(tm[6]),
        "phases_s": {nm: float(v) for nm, v in zip(names, tm)},
        "wall_incl_compile_s": wall, "srs_setup_s": t_srs}), flush=True)


if __name__ == "__main__":
    main()
