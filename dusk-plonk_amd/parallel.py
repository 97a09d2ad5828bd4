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
index — one all-gather of 14 words per commit per group, host fold on every rank. With
several lanes per rank, ``ExchangeService`` runs every lane's all-gathers on one
communicator from one thread, in an order rank 0 sequences (deadlock-free by construction).
"""
from __future__ import annotations

import threading
import time
from collections import deque

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


class _Request:
    __slots__ = ("data", "done", "result", "error")

    def __init__(self, data: bytes):
        self.data = data
        self.done = threading.Event()
        self.result = None
        self.error = None


class ExchangeService:
    """The all-gathers of every prover lane of this rank on ONE communicator, issued by ONE
    thread, in an order every rank agrees on — deadlock-free by construction.

    With one communicator per lane, lanes reach their exchanges in timing-dependent order, so
    ranks could launch RCCL collectives on different communicators in different orders while
    other lanes' kernels hold the CUs — the pattern that can deadlock. Here:
      * every lane's `allgather` only queues its request and waits for the result;
      * rank 0's exchange thread picks the lanes whose requests are pending on rank 0 (arrival
        order) and broadcasts that list (lane id + byte count per entry) to every rank;
      * every rank's exchange thread then waits until those lanes' requests are pending
        locally and runs ONE all-gather of their payloads concatenated in list order.
    Collectives are thus issued by one thread per rank on one group — a group of the service's
    own, so no other thread's collective can interleave with them — in the same sequence on
    every rank. A rank only ever waits for a lane's NEXT request, and the lanes' request
    sequences are identical on every rank (every rank proves the same proofs with the same
    seeds; a commit's status travels in the exchange, so every rank takes the same error
    path), so each awaited request arrives: lanes never wait on anything but their own
    exchange. `close()` (every rank, after its lanes stopped) ends the thread: rank 0
    broadcasts a stop entry once nothing is pending.

    Failure: a lane whose proof fails BEFORE an exchange (a host error on one rank only) must
    still reach that exchange with an error status — the C++ prover sends its status in the
    exchanged words — or the peers wait for it (REQUEST_TIMEOUT_S). If the exchange thread
    itself fails, it wakes this rank's lanes with the error and destroys the service group, so
    the peers' pending collectives fail rather than block (the group is created with a
    GROUP_TIMEOUT_S timeout for backends that only time out).
    """

    MAX_BATCH = 64  # lanes served by one all-gather
    REQUEST_TIMEOUT_S = 600.0  # a lane rank 0 scheduled must reach its exchange by then
    # the service group's collective timeout: a peer whose exchange thread failed (and tore
    # its group down) makes this rank's pending collective fail instead of waiting forever
    GROUP_TIMEOUT_S = 900.0

    def __init__(self, group=None, device=None):
        """Collective: every rank of `group` (default: the world) constructs it at the same
        point. The service runs on a process group of its own over the same ranks, so the
        caller's collectives on `group` (barriers, timing reductions) never interleave with
        the exchange thread's on another thread."""
        import torch
        import torch.distributed as dist

        self.torch, self.dist = torch, dist
        ranks = dist.get_process_group_ranks(group) if group is not None else None
        import datetime
        self.group = dist.new_group(ranks=ranks, backend=dist.get_backend(group),
                                    timeout=datetime.timedelta(seconds=self.GROUP_TIMEOUT_S))
        self.device = device
        self.world = dist.get_world_size(self.group)
        self.rank = dist.get_rank(self.group)
        self.src = dist.get_global_rank(self.group, 0)
        self.cv = threading.Condition()
        self.pending = {}        # lane -> deque of _Request (a lane has at most one)
        self.arrivals = deque()  # rank 0: lane ids in arrival order
        self.closing = False
        self.error = None
        self.exchanges = 0       # all-gathers run (statistics)
        self.requests = 0        # lane requests served
        self.thread = threading.Thread(target=self._run, name="plk-exchange", daemon=True)
        self.thread.start()

    def allgather_for(self, lane: int):
        """`allgather(send: bytes) -> bytes` for prover lane `lane` (the same id on every
        rank): every rank's bytes concatenated in rank order."""
        def allgather(data: bytes) -> bytes:
            req = _Request(bytes(data))
            with self.cv:
                if self.error is not None:
                    raise RuntimeError(f"exchange service failed: {self.error!r}")
                if self.closing:
                    raise RuntimeError("exchange service closed")
                self.pending.setdefault(lane, deque()).append(req)
                self.arrivals.append(lane)
                self.cv.notify_all()
            req.done.wait()
            if req.error is not None:
                raise RuntimeError(f"exchange failed: {req.error!r}")
            return req.result
        return allgather

    # -- exchange thread -----------------------------------------------------------------
    def _tensor(self, arr):
        t = self.torch.from_numpy(arr)
        return t.to(self.device) if self.device is not None else t

    def _plan(self):
        """Rank 0: (lanes, sizes) to serve next, or None to stop."""
        with self.cv:
            while not self.arrivals and not (self.closing and not self._any_pending()):
                self.cv.wait()
            if not self.arrivals:
                return None
            lanes, seen = [], set()
            while self.arrivals and len(lanes) < self.MAX_BATCH:
                ln = self.arrivals[0]
                if ln in seen:  # a lane's next request waits for the next all-gather
                    break
                self.arrivals.popleft()
                seen.add(ln)
                lanes.append(ln)
            return lanes, [len(self.pending[ln][0].data) for ln in lanes]

    def _any_pending(self):
        return any(self.pending.values())

    def _run(self):
        torch, dist = self.torch, self.dist
        header = np.zeros(1 + 2 * self.MAX_BATCH, dtype=np.int64)
        stream = torch.cuda.Stream(device=self.device) if self.device is not None else None
        try:
            while True:
                if self.rank == 0:
                    plan = self._plan()
                    header[:] = 0
                    if plan is None:
                        header[0] = -1
                    else:
                        lanes, sizes = plan
                        header[0] = len(lanes)
                        header[1:1 + len(lanes)] = lanes
                        header[1 + self.MAX_BATCH:1 + self.MAX_BATCH + len(lanes)] = sizes
                with (torch.cuda.stream(stream) if stream is not None else _nullctx()):
                    h = self._tensor(header.copy())
                    dist.broadcast(h, src=self.src, group=self.group)
                    hdr = h.cpu().numpy()
                    cnt = int(hdr[0])
                    if cnt < 0:
                        return
                    lanes = [int(x) for x in hdr[1:1 + cnt]]
                    sizes = [int(x) for x in hdr[1 + self.MAX_BATCH:1 + self.MAX_BATCH + cnt]]
                    reqs = []
                    with self.cv:
                        for ln in lanes:
                            deadline = time.monotonic() + self.REQUEST_TIMEOUT_S
                            while not self.pending.get(ln):
                                left = deadline - time.monotonic()
                                if left <= 0:  # the ranks' lane sequences diverged
                                    raise RuntimeError(f"lane {ln}'s exchange never arrived "
                                                       f"on rank {self.rank}")
                                self.cv.wait(left)
                            reqs.append(self.pending[ln].popleft())
                        if self.rank != 0:  # keep the arrival log bounded off rank 0
                            self.arrivals.clear()
                    for r, sz in zip(reqs, sizes):
                        if len(r.data) != sz:
                            raise RuntimeError(f"lane exchange size differs across ranks "
                                               f"({len(r.data)} here, {sz} on rank 0)")
                    payload = b"".join(r.data for r in reqs)
                    total = len(payload)
                    t = self._tensor(np.frombuffer(payload, dtype=np.uint8).copy())
                    out = torch.empty(self.world * total, dtype=torch.uint8, device=t.device)
                    dist.all_gather_into_tensor(out, t, group=self.group)
                    allb = out.cpu().numpy().tobytes()
                self.exchanges += 1
                self.requests += len(reqs)
                off = 0
                for r, sz in zip(reqs, sizes):
                    r.result = b"".join(allb[q * total + off: q * total + off + sz]
                                        for q in range(self.world))
                    off += sz
                    r.done.set()
        except BaseException as e:  # noqa: BLE001 — every waiting lane must wake
            with self.cv:
                self.error = e
                for dq in self.pending.values():
                    for r in dq:
                        r.error = e
                        r.done.set()
                    dq.clear()
                self.cv.notify_all()
            # peers may be blocked in this group's next collective: tear the group down so
            # theirs fails (or times out after GROUP_TIMEOUT_S) instead of waiting forever
            try:
                dist.destroy_process_group(self.group)
            except Exception:  # noqa: BLE001 — already torn down / backend refused
                pass

    def close(self, timeout: float | None = 120.0):
        """Stop the exchange thread (call on every rank once its lanes are done)."""
        with self.cv:
            self.closing = True
            self.cv.notify_all()
        self.thread.join(timeout)
        if self.thread.is_alive():
            raise RuntimeError("exchange thread did not stop")
        if self.error is not None:
            raise RuntimeError(f"exchange service failed: {self.error!r}")


class _nullctx:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


def srs_slice(tau, n_points: int, world: int, rank: int, ctx=None):
    """(slice start, PlonkParams) of rank `rank`'s share of the first `n_points` SRS
    powers of `tau` (plk_srs_setup_range on its GPU, window table included)."""
    lo, hi = shard_range(n_points, world, rank)
    return lo, PlonkParams.setup_range(tau, lo, hi - lo, ctx)


def shard_prover_lane(lane, tau, n_points: int, group=None, device=None, ctx=None,
                      slice_=None, exchange: ExchangeService | None = None, lane_id: int = 0,
                      mode: str = "slices"):
    """Split every commit of `lane` (a prover.ProverLane) over the ranks of `group`, one
    all-gather per commit group, two ways:

    * mode "slices" (rounds 2-5, plk_prover_shard): this rank's slice of the first `n_points`
      SRS powers of `tau`; `slice_` = (start, PlonkParams) from srs_slice lets several lanes
      share one slice (the SRS is read-only; each lane brings its own MSM workspace);
    * mode "buckets" (round 6, plk_prover_shard_buckets): the key's own whole SRS, this rank
      keeping bucket range `rank` of `world` of every commit (its sort, accumulation and
      bucket reduction cover 1/world of the buckets; no slice is built). Needs a power-of-two
      world and a wide bucket set with >= 2^14 buckets per part (bucket_parts_ok);
    * mode "auto": buckets where the key's SRS allows the split, slices otherwise (the same
      decision on every rank: it depends only on the SRS size and the world).

    With several lanes per rank pass `exchange` (one ExchangeService per rank) and a `lane_id`
    that names the same lane on every rank: all lanes' exchanges then share one communicator
    and one issuing thread. A lone lane may use the group's all-gather directly. Returns the
    slice (start, PlonkParams), or None in bucket mode."""
    import torch.distributed as dist

    if mode not in ("slices", "buckets", "auto"):
        raise ValueError(f"shard_prover_lane: mode {mode!r}")
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    ag = exchange.allgather_for(lane_id) if exchange is not None else torch_allgather(group, device)
    if mode == "buckets" or (mode == "auto" and bucket_parts_ok(lane.prover.pp.n, world)):
        lane.shard(None, 0, rank, world, ag, buckets=True)
        return None
    lo, sl = slice_ if slice_ is not None else srs_slice(tau, n_points, world, rank, ctx)
    lane.shard(sl, lo, rank, world, ag)
    return lo, sl


def window_bits(n_points: int) -> int:
    """The MSM window size c an SRS of n_points runs with: srs.hip choose_c (including its
    PLK_MSM_C override, which accepts 8..22 except 21) and msm_prepare_srs's mapping of a c
    whose every window would be c - 1 bits wide (c = 18) to c - 1 (oracle/pyref.py
    msm_effective_c)."""
    import os
    c = 0
    env = os.environ.get("PLK_MSM_C")
    if env:
        try:
            v = int(env)
        except ValueError:
            v = 0
        if 8 <= v <= 22 and v != 21:
            c = v
    if not c:
        c = (20 if n_points >= 1 << 20 else 17 if n_points >= 1 << 16 else
             15 if n_points >= 1 << 15 else 13 if n_points >= 1 << 14 else
             12 if n_points >= 1 << 13 else 10 if n_points >= 1 << 10 else 8)
    return c - 1 if (c - 1) * ((255 + c - 1) // c) == 255 else c


def bucket_parts_ok(n_points: int, parts: int) -> bool:
    """Whether plk_commit_batch_dev_part accepts `parts` bucket ranges on an SRS of n_points
    (msm.hip msm_commit_batch_part): a power of two, a wide bucket set (2^(c-1) above the
    32 K LDS buckets, c >= 17) and >= 2^14 buckets per part."""
    c = window_bits(n_points)
    return (parts >= 1 and parts & (parts - 1) == 0
            and (parts == 1 or (c >= 17 and (1 << (c - 1)) // parts >= 1 << 14)))


class ShardedPlonkParams:
    """PlonkParams whose MSM work is spread over the ranks of a process group, two ways:

    * mode "points" (rounds 1-4): the G1 powers are split into contiguous SRS slices, rank r
      holds slice r (``PlonkParams.setup_range``) and runs the whole Pippenger over its slice
      of every polynomial. The accumulation divides by G; each rank still sorts into and
      reduces the FULL bucket set (2^19 buckets at 2^20), a fixed cost that does not shrink.
    * mode "buckets" (round 5, SURVEY §8e "partial bucket sums for a single large MSM"): every
      rank holds the whole SRS and window table, reads every scalar, and keeps only the
      digits of its bucket range [r, r + 1) x 2^(c-1) / G (plk_commit_batch_dev_part): its
      sort, accumulation AND run-sum / bit-sum reduction cover 1/G of the buckets. The rank's
      share sum_{b in range} (b + 1) S_b is one point; the shares are all-gathered and folded
      exactly as the slices' partials are. G must be a power of two with 2^(c-1) / G >=
      2^14 (c = 20 from 2^20 points: up to 32 ranks; c = 17: up to 4); "auto" takes it then
      and the point slices otherwise.

    Outputs are identical in both modes (canonical affine, the fold order is irrelevant)."""

    def __init__(self, k: int, tau, n_points: int | None = None, ctx=None, group=None,
                 mode: str = "points"):
        import torch.distributed as dist

        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.n = n_points if n_points is not None else (1 << k) + PlonkParams.SLACK
        if mode not in ("points", "buckets", "auto"):
            raise ValueError(f"ShardedPlonkParams: mode {mode!r}")
        if mode in ("buckets", "auto"):
            ok = bucket_parts_ok(self.n, self.world)
            if mode == "buckets" and not ok:
                raise ValueError(f"ShardedPlonkParams: {self.world} bucket ranges need a power-of-"
                                 f"two world and 2^(c-1) / world >= 2^14 (SRS of {self.n} points)")
            mode = "buckets" if ok else "points"
        self.mode = mode
        if mode == "buckets":
            self.lo, self.hi = 0, self.n
            self.local = PlonkParams.setup(k, tau, ctx, n_points=self.n)
        else:
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
        if self.mode == "buckets":
            part = self.local.commit_batch_dev(list(ptrs_lens), stream, raise_on_error=False,
                                               part=self.rank, parts=self.world)
        else:
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


__all__ = ["ExchangeService", "ShardedPlonkParams", "bucket_parts_ok", "gather_fold", "shard_range",
           "shard_prover_lane", "srs_slice", "torch_allgather", "PLK_E_DEGREE"]
