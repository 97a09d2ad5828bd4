"""Multi-GPU: the sharded single MSM over torch.distributed (RCCL on GPUs).

For G ranks the SRS index range [0, N) is split into G contiguous shards; shard r lives on
GPU r (``PlonkParams.setup_range``). A commit runs the full Pippenger on each rank's slice
of the (replicated) coefficient vector, producing one canonical affine partial point
(104 B) per rank; one ``all_gather`` over xGMI moves G x 112 B (13 words + status) and
every rank folds the partials on the host (``plk_g1_sum``): EC addition is not an RCCL
reduction op, so the "all-reduce of partial sums" is an all-gather plus a local fold.
Batches of independent commits (the prover's commit groups) share one all-gather.
Proof batches need no collective at all (bench.py default mode).

The full prover uses the same split inside ``plk_prover_prove`` (BASELINE configs[4]):
``shard_prover_lane`` gives a prover lane its SRS slice and a torch.distributed all-gather
as the C ABI's ``plk_allgather_fn``; every rank then proves the same circuit with the same
seed, runs the NTT / elementwise rounds as replicas and splits each of the proof's 4 commit
groups (wires, z, quotient chunks, openings: prover.rs:133-136,194,262-265,440,452) by SRS
index — one all-gather of 14 words per commit per group, host fold on every rank.
"""
from __future__ import annotations

import numpy as np

from .plonk import PLK_E_DEGREE, PLK_OK, Commitment, PlonkError, PlonkParams, g1_sum


def shard_range(n: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous balanced shard [lo, hi) of range(n) for `rank`."""
    base, rem = divmod(n, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def gather_fold(partials: np.ndarray, statuses, group=None, device=None) -> list:
    """All-gather per-rank partial points uint64[slots, 13] (+ a status per slot) and fold.

    Returns one Commitment per slot, or a PlonkError for a slot any rank failed."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    slots = partials.shape[0]
    buf = np.zeros((slots, 14), dtype=np.uint64)
    buf[:, :13] = partials
    buf[:, 13] = np.asarray(statuses, dtype=np.uint64)
    t = torch.from_numpy(buf.view(np.int64).reshape(-1)).to(device or "cpu")
    out = torch.empty(world * slots * 14, dtype=torch.int64, device=t.device)
    dist.all_gather_into_tensor(out, t, group=group)
    allp = out.cpu().numpy().view(np.uint64).reshape(world, slots, 14)
    res = []
    for k in range(slots):
        st = int(allp[:, k, 13].max())
        res.append(g1_sum(allp[:, k, :13]) if st == PLK_OK else PlonkError(st, "sharded commit"))
    return res


def torch_allgather(group=None, device=None):
    """`allgather(send: bytes) -> bytes` over a torch.distributed group: every rank's
    bytes concatenated in rank order (all_gather_into_tensor; on `device` for RCCL, on the
    host under gloo). The byte-level collective behind plk_allgather_fn."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)

    def allgather(data: bytes) -> bytes:
        t = torch.frombuffer(bytearray(data), dtype=torch.uint8).to(device or "cpu")
        out = torch.empty(world * len(data), dtype=torch.uint8, device=t.device)
        dist.all_gather_into_tensor(out, t, group=group)
        return out.cpu().numpy().tobytes()

    return allgather


def srs_slice(tau, n_points: int, world: int, rank: int, ctx=None):
    """(slice start, PlonkParams) of rank `rank`'s share of the first `n_points` SRS
    powers of `tau` (plk_srs_setup_range on its GPU, window table included)."""
    lo, hi = shard_range(n_points, world, rank)
    return lo, PlonkParams.setup_range(tau, lo, hi - lo, ctx)


def shard_prover_lane(lane, tau, n_points: int, group=None, device=None, ctx=None,
                      slice_=None):
    """Split every commit of `lane` (a prover.ProverLane) over the ranks of `group`: this
    rank's slice of the first `n_points` SRS powers of `tau` and the group's all-gather.
    `slice_` = (start, PlonkParams) from srs_slice lets several lanes share one slice (the
    SRS is read-only; each lane brings its own MSM workspace). Returns the slice."""
    import torch.distributed as dist

    world, rank = dist.get_world_size(group), dist.get_rank(group)
    lo, sl = slice_ if slice_ is not None else srs_slice(tau, n_points, world, rank, ctx)
    lane.shard(sl, lo, rank, world, torch_allgather(group, device))
    return lo, sl


class ShardedPlonkParams:
    """PlonkParams whose G1 powers are spread over the ranks of a process group."""

    def __init__(self, k: int, tau, n_points: int | None = None, ctx=None, group=None):
        import torch.distributed as dist

        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.n = n_points if n_points is not None else (1 << k) + PlonkParams.SLACK
        self.lo, self.hi = shard_range(self.n, self.world, self.rank)
        self.local = PlonkParams.setup_range(tau, self.lo, self.hi - self.lo, ctx)

    def _local_spans(self, length: int) -> tuple[int, int]:
        """(offset, length) of this rank's part of a length-`length` polynomial; the last
        rank also covers [n, length) so the degree check sees the whole tail."""
        if self.rank == self.world - 1:
            return self.lo, max(0, length - self.lo)
        return self.lo, max(0, min(self.hi, length) - self.lo)

    def commit_batch_dev(self, ptrs_lens, stream: int = 0, device=None):
        """Independent commits of device polynomials [(ptr, len)] (coefficients replicated
        on every rank) -> list of Commitment / PlonkError, identical on every rank."""
        spans = []
        for ptr, length in ptrs_lens:
            off, m = self._local_spans(length)
            spans.append((ptr + 32 * off, m))
        part = self.local.commit_batch_dev(spans, stream, raise_on_error=False)
        words = np.zeros((len(part), 13), dtype=np.uint64)
        sts = []
        for i, p in enumerate(part):
            if isinstance(p, Commitment):
                words[i] = p.words
                sts.append(PLK_OK)
            else:
                words[i, 12] = 1
                sts.append(p.status)
        return gather_fold(words, sts, self.group, device)

    def commit_dev(self, ptr: int, length: int, stream: int = 0, device=None) -> Commitment:
        r = self.commit_batch_dev([(ptr, length)], stream, device)[0]
        if isinstance(r, PlonkError):
            raise r
        return r


__all__ = ["ShardedPlonkParams", "gather_fold", "shard_range", "shard_prover_lane",
           "srs_slice", "torch_allgather", "PLK_E_DEGREE"]
