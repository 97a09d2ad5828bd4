#!/usr/bin/env python3
"""One rank's share of a bucket-split sharded proof (BASELINE configs[4], plk_prover_shard_buckets)
measured on ONE GPU: kernel evidence for the per-GPU work of a proof whose commits are split
over G GPUs, which this pool cannot run (one GPU per box).

A prover lane is split as rank r of G, and its all-gather is emulated by repeating this rank's
payload G times. The folded commitments are then wrong (G x this rank's share), so the proof is
not a valid one, but every kernel this rank runs — its 1/G bucket range of every commit (sort,
accumulation, run sums, bit sums) and the full NTT / elementwise rounds it replicates — runs
exactly as on a node. Reported beside an unsharded lane on the same key: per-proof wall time
and the lane's k_accumulate time, launches and additions per proof. Run under
`rocprofv3 --kernel-trace --stats` for the per-kernel breakdown.

  python tools/shard_rank_probe.py --log-n 20 --world 8 --rank 0 --proofs 4
"""
from __future__ import annotations

import argparse
import json
import statistics
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--log-n", type=int, default=20)
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--proofs", type=int, default=4)
    a = ap.parse_args()
    import torch
    torch.cuda.set_device(0)
    import dusk_plonk_amd as plk
    import bench
    plk.check_build()
    ctx = plk.Context.default(0)
    base = bench.ProverBase(plk, a.log_n, ctx)

    def run(lane, tag):
        cs = bench.bench_circuit(base.Plonk, base.chain, 5)
        lane.prove_composer(cs, 5)  # warmup (workspace allocation)
        lane.msm_stats(reset=True)
        ts = []
        for i in range(a.proofs):
            cs = bench.bench_circuit(base.Plonk, base.chain, 10 + i)
            t0 = time.perf_counter()
            lane.prove_composer(cs, 10 + i)
            ts.append(time.perf_counter() - t0)
        ms, launches, adds, points = lane.msm_stats(reset=True)
        return {"tag": tag, "proof_ms_median": 1e3 * statistics.median(ts),
                "proof_ms": [round(1e3 * t, 3) for t in ts],
                "accumulate_ms_per_proof": ms / a.proofs, "launches_per_proof": launches / a.proofs,
                "point_adds_per_proof": adds / a.proofs, "msm_points_per_proof": points / a.proofs}

    whole = run(base.prover.lane(), "unsharded lane")
    lane = base.prover.lane()
    world = a.world
    lane.shard(None, 0, a.rank, world, lambda send: send * world, buckets=True)
    part = run(lane, f"rank {a.rank} of {world} (bucket range; all-gather emulated)")
    print(json.dumps({"log_n": a.log_n, "world": world, "rank": a.rank, "proofs": a.proofs,
                      "unsharded": whole, "rank_share": part,
                      "note": "one GPU: the rank's kernels exactly as on a node, its commitments "
                              "wrong (the emulated all-gather repeats its own shares)"}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
