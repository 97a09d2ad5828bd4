"""Multi-process tests of the sharded single MSM.

CPU (gloo, world_size 2): shard ranges, the all-gather of per-rank partial points and the
host fold (plk_g1_sum, no GPU needed) are the product code; the per-rank partial MSM is
computed by the C oracle (test infrastructure) since this container has no GPU.
GPU: two ranks on one card run the real path (SRS shards on the GPU, commits on the GPU,
gather over gloo) against the unsharded commit.
"""
import os
import socket
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parent.parent


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_shard_range_partitions():
    sys.path.insert(0, str(ROOT))
    from dusk_plonk_amd.parallel import shard_range
    for n in (1, 7, 64, 1000, (1 << 20) + 8):
        for world in (1, 2, 3, 8):
            spans = [shard_range(n, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            sizes = [h - l for l, h in spans]
            assert max(sizes) - min(sizes) <= 1


def test_g1_sum_host(plk, oracle, golden):
    g = golden["msm"]
    srs = g["srs"]
    ones = np.tile(np.asarray(__import__("pyref").fr_vec_to_np([1])[0]), (srs.shape[0], 1))
    assert np.array_equal(plk.plonk.g1_sum(srs).words, oracle.msm(srs, ones))
    assert plk.plonk.g1_sum(srs[:0]).is_identity
    # P + (-P) = identity
    neg = srs[:1].copy()
    import pyref as P
    x, y = P.g1_vec_from_np(neg)[0]
    both = P.g1_vec_to_np([(x, y), (x, (-y) % P.P_MOD)])
    assert plk.plonk.g1_sum(both).is_identity


def _cpu_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, str(ROOT))
    sys.path.insert(0, str(ROOT / "tests"))
    sys.path.insert(0, str(ROOT / "oracle"))
    import torch.distributed as dist
    import oracle_lib
    from dusk_plonk_amd.parallel import gather_fold, shard_range
    import dusk_plonk_amd as plk

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        orc = oracle_lib.load()
        g = dict(np.load(ROOT / "tests" / "golden" / "msm_golden.npz", allow_pickle=False))
        srs = g["srs"]
        n = srs.shape[0]
        lo, hi = shard_range(n, world, rank)
        slots = ["random", "sparse", "minus_one"]
        parts = np.stack([orc.msm(srs[lo:hi], g[f"{s}_scalars"][lo:hi]) for s in slots])
        res = gather_fold(parts, [plk.PLK_OK] * len(slots))
        ok = all(np.array_equal(r.words, g[f"{s}_result"]) for r, s in zip(res, slots))
        # a degree error on one rank is seen by every rank
        st = [plk.PLK_OK, plk.PLK_E_DEGREE if rank == world - 1 else plk.PLK_OK, plk.PLK_OK]
        res2 = gather_fold(parts, st)
        ok &= isinstance(res2[1], plk.PlonkError) and res2[1].status == plk.PLK_E_DEGREE
        ok &= np.array_equal(res2[0].words, g["random_result"])
        q.put((rank, bool(ok)))
    finally:
        dist.destroy_process_group()


def _spawn(fn, world, *args):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=fn, args=(r, world, port, q, *args)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
    out = dict(q.get(timeout=5) for _ in range(world))
    for p in procs:
        assert p.exitcode == 0
    return out


def test_sharded_msm_gather_fold_gloo_world2():
    out = _spawn(_cpu_worker, 2)
    assert out == {0: True, 1: True}


class _FakePartParams:
    """CPU stand-in for a rank's PlonkParams in ShardedPlonkParams' bucket mode: its
    commit_batch_dev(part=, parts=) returns the bucket-range shares of the restated split
    (oracle/pyref.py msm_bucket_part, window c = 20) — `ptr` indexes host scalar arrays."""

    def __init__(self, points, polys, c=20):
        self.points, self.polys, self.c = points, polys, c
        self.calls = []

    def commit_batch_dev(self, ptrs_lens, stream=0, raise_on_error=True, part=0, parts=1):
        import pyref as P
        import dusk_plonk_amd as plk
        self.calls.append((part, parts))
        out = []
        for ptr, length in ptrs_lens:
            sc = P.fr_vec_from_np(self.polys[ptr][:length])
            share = P.msm_bucket_part(self.points[:length], sc, self.c, part, parts)
            out.append(plk.Commitment(P.g1_vec_to_np([share])[0]))
        return out


def _cpu_bucket_worker(rank, world, port, q):
    """ShardedPlonkParams.commit_batch_dev in bucket mode over gloo: each rank's share of its
    bucket range (the restated split), one all-gather, host fold (plk_g1_sum)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, str(ROOT))
    sys.path.insert(0, str(ROOT / "tests"))
    sys.path.insert(0, str(ROOT / "oracle"))
    import torch.distributed as dist
    import pyref as P
    from dusk_plonk_amd.parallel import ShardedPlonkParams, bucket_parts_ok

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g = dict(np.load(ROOT / "tests" / "golden" / "msm_golden.npz", allow_pickle=False))
        pts = P.g1_vec_from_np(g["srs"])
        slots = ["random", "minus_one", "sparse"]
        sh = object.__new__(ShardedPlonkParams)  # no GPU: the rank's params are the fake
        sh.group, sh.world, sh.rank, sh.mode = None, world, rank, "buckets"
        sh.lo, sh.hi, sh.n = 0, len(pts), len(pts)
        sh.local = _FakePartParams(pts, [g[f"{s}_scalars"] for s in slots])
        res = sh.commit_batch_dev([(i, len(pts)) for i in range(len(slots))])
        ok = all(np.array_equal(r.words, g[f"{s}_result"]) for r, s in zip(res, slots))
        ok &= sh.local.calls == [(rank, world)]
        ok &= bucket_parts_ok(1 << 20, world) and not bucket_parts_ok(1 << 20, 3)
        ok &= bucket_parts_ok(1 << 16, 4) and not bucket_parts_ok(1 << 16, 8)
        q.put((rank, bool(ok)))
    finally:
        dist.destroy_process_group()


def test_bucket_split_gather_fold_gloo_world2():
    """The bucket-range split of a single MSM on 2 gloo ranks, CPU only."""
    out = _spawn(_cpu_bucket_worker, 2)
    assert out == {0: True, 1: True}


def _gpu_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, str(ROOT))
    sys.path.insert(0, str(ROOT / "tests"))
    import torch
    import torch.distributed as dist
    from oracle_lib import random_fr
    import dusk_plonk_amd as plk
    from dusk_plonk_amd.parallel import ShardedPlonkParams

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        k = 12
        tau = random_fr(1, seed=77)[0]
        ctx = plk.Context.default(0)
        sh = ShardedPlonkParams(k, tau, ctx=ctx)
        full = plk.PlonkParams.setup(k, tau, ctx)
        n = (1 << k) + 8
        polys = [random_fr(m, seed=300 + i) for i, m in enumerate([n, n - 5, 33, 1 << k])]
        devs = [torch.from_numpy(p.view(np.int64)).cuda() for p in polys]
        bad = torch.from_numpy(random_fr(n + 40, seed=9).view(np.int64)).cuda()
        torch.cuda.synchronize()
        s = torch.cuda.current_stream().cuda_stream
        res = sh.commit_batch_dev([(d.data_ptr(), d.shape[0]) for d in devs] +
                                  [(bad.data_ptr(), bad.shape[0])], s)
        ok = all(np.array_equal(r.words, full.commit(plk.Coefficients(p)).words)
                 for r, p in zip(res, polys))
        ok &= isinstance(res[-1], plk.PlonkError) and res[-1].status == plk.PLK_E_DEGREE
        q.put((rank, bool(ok)))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_sharded_commit_two_ranks_one_gpu(plk, gpu_ctx):
    out = _spawn(_gpu_worker, 2)
    assert out == {0: True, 1: True}


@pytest.mark.gpu
def test_msm_sharded_single_process(plk, gpu_ctx):
    """plk_msm_sharded: one process, consecutive SRS slices (PlonkParams.setup_range; here
    all on the one visible device), even and uneven cuts, full and partial scalar lengths,
    against the unsharded MSM."""
    from oracle_lib import random_fr
    from dusk_plonk_amd.plonk import msm_sharded
    n = 1 << 12
    tau = random_fr(1, seed=41)[0]
    full = plk.PlonkParams.setup(12, tau, gpu_ctx, n_points=n)
    sc = random_fr(n, seed=42)
    for cuts in ([0, n // 2, n], [0, 1000, 1001, n]):
        shards = [plk.PlonkParams.setup_range(tau, lo, hi - lo, gpu_ctx)
                  for lo, hi in zip(cuts, cuts[1:])]
        for m in (n, 1500, 1000, 1):
            assert np.array_equal(msm_sharded(shards, sc[:m]).words, full.msm(sc[:m]).words), (cuts, m)


def _sharded_prover_worker(rank, world, port, q, logn, mode="slices"):
    """BASELINE configs[4] at a test size: every rank proves the same circuit with its
    commits split by SRS slice (plk_prover_shard) and exchanges partials over gloo; the
    proof must equal the unsharded plk_prove's byte for byte on every rank."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, str(ROOT))
    sys.path.insert(0, str(ROOT / "tests"))
    import torch.distributed as dist
    from oracle_lib import random_fr
    import dusk_plonk_amd as plk
    from dusk_plonk_amd.parallel import shard_prover_lane
    from dusk_plonk_amd.prover import Plonk, PlonkKey

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        tau = random_fr(1, seed=91)[0]
        ctx = plk.Context.default(0)
        pp = plk.PlonkParams.setup(logn, tau, ctx)

        def circ(seed):
            cs = Plonk()
            cs.synthetic_chain((1 << logn) - 15, seed)
            cs.append_public(seed + 7)
            return cs
        prover, _ = PlonkKey.compile_composer(pp, b"shard", circ(1))
        lane = prover.lane()
        shard_prover_lane(lane, tau, pp.n, None, None, ctx, mode=mode)
        ok = True
        for seed in (3, 4):
            want = prover.prove_composer(circ(seed + 10), seed)[0].raw_bytes()
            got, pi = lane.prove_composer(circ(seed + 10), seed)
            ok &= got.raw_bytes() == want and len(pi) == 1
        # an unsatisfied circuit fails with the degree error on every rank
        bad = circ(20)
        bad.set_witness(5, 12345)  # breaks one gate of the chain
        try:
            lane.prove_composer(bad, 1)
            ok = False
        except plk.PlonkError as e:
            ok &= e.status == plk.PLK_E_DEGREE
        lane.close()
        q.put((rank, bool(ok)))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_sharded_prover_two_ranks_one_gpu(plk, gpu_ctx):
    out = _spawn(_sharded_prover_worker, 2, 12)
    assert out == {0: True, 1: True}


@pytest.mark.gpu
def test_sharded_prover_two_ranks_wide_slices(plk, gpu_ctx):
    """2^17: each rank's SRS slice holds over 2^16 points, so the sharded commits run the
    MSM's wide-bucket path (c = 17: two-level sort, run-sum reduction) on every rank."""
    out = _spawn(_sharded_prover_worker, 2, 17)
    assert out == {0: True, 1: True}


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 4])
def test_sharded_prover_bucket_split(plk, gpu_ctx, world):
    """plk_prover_shard_buckets (round 6): every commit of a 2^17 proof split by bucket range
    (c = 17: 2 or 4 parts of 2^15 / 2^14 buckets) over gloo ranks sharing the card; proofs equal
    plk_prove's bytes and an unsatisfied circuit fails with the degree error on every rank."""
    out = _spawn(_sharded_prover_worker, world, 17, "buckets")
    assert out == {r: True for r in range(world)}


def _bucket_refusal_worker(rank, world, port, q):
    """mode "buckets" is refused (PLK_E_ARG) where the key's SRS has no wide bucket set
    (2^12: c = 10); mode "auto" then shards by slice and proves the same bytes."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path[:0] = [str(ROOT), str(ROOT / "tests")]
    import torch.distributed as dist
    from oracle_lib import random_fr
    import dusk_plonk_amd as plk
    from dusk_plonk_amd.parallel import shard_prover_lane
    from dusk_plonk_amd.prover import Plonk, PlonkKey

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        tau = random_fr(1, seed=95)[0]
        ctx = plk.Context.default(0)
        pp = plk.PlonkParams.setup(12, tau, ctx)
        cs = Plonk()
        cs.synthetic_chain((1 << 12) - 15, 3)
        prover, _ = PlonkKey.compile_composer(pp, b"refuse", cs)
        lane = prover.lane()
        ok = False
        try:
            shard_prover_lane(lane, tau, pp.n, mode="buckets")
        except plk.PlonkError as e:
            ok = e.status == plk.PLK_E_ARG
        ok &= shard_prover_lane(lane, tau, pp.n, ctx=ctx, mode="auto") is not None  # a slice
        ok &= lane.prove_composer(cs, 9)[0].raw_bytes() == prover.prove_composer(cs, 9)[0].raw_bytes()
        lane.close()
        q.put((rank, bool(ok)))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_sharded_prover_bucket_split_refused_small_srs(plk, gpu_ctx):
    out = _spawn(_bucket_refusal_worker, 2)
    assert out == {0: True, 1: True}


@pytest.mark.gpu
def test_sharded_prover_three_ranks_uneven(plk, gpu_ctx):
    out = _spawn(_sharded_prover_worker, 3, 10)
    assert out == {0: True, 1: True, 2: True}


def _allgather_cb_worker(rank, world, port, q):
    """The byte all-gather behind plk_allgather_fn (parallel.torch_allgather) driven through
    the same ctypes callback the C++ prover calls, and the host fold of exchanged partial
    points (plk_g1_sum): the sharded prover's exchange without a GPU (gloo, world 2). The
    per-rank partial MSMs come from the C oracle (test infrastructure)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, str(ROOT))
    sys.path.insert(0, str(ROOT / "tests"))
    import ctypes as C
    import torch.distributed as dist
    import oracle_lib
    import dusk_plonk_amd as plk
    from dusk_plonk_amd.parallel import shard_range, torch_allgather
    from dusk_plonk_amd.prover import ALLGATHER_FN

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        orc = oracle_lib.load()
        g = dict(np.load(ROOT / "tests" / "golden" / "msm_golden.npz", allow_pickle=False))
        srs = g["srs"]
        lo, hi = shard_range(srs.shape[0], world, rank)
        ag = torch_allgather()
        recv_holder = {}

        def cb(_u, send, nbytes, recv):
            data = ag(C.string_at(send, nbytes))
            C.memmove(recv, data, len(data))
            recv_holder["n"] = len(data)
            return 0
        fn = ALLGATHER_FN(cb)
        slots = ["random", "sparse", "minus_one"]
        send = np.zeros((len(slots), 14), dtype=np.uint64)  # 13 point words + status
        for i, sname in enumerate(slots):
            send[i, :13] = orc.msm(srs[lo:hi], g[f"{sname}_scalars"][lo:hi])
        recv = np.zeros((world, len(slots), 14), dtype=np.uint64)
        rc = fn(None, send.ctypes.data, send.nbytes, recv.ctypes.data)
        ok = rc == 0 and recv_holder["n"] == world * send.nbytes
        for i, sname in enumerate(slots):
            ok &= np.array_equal(plk.plonk.g1_sum(recv[:, i, :13]).words, g[f"{sname}_result"])
        q.put((rank, bool(ok)))
    finally:
        dist.destroy_process_group()


def test_sharded_prover_exchange_gloo_world2():
    out = _spawn(_allgather_cb_worker, 2)
    assert out == {0: True, 1: True}


def _bucket_exchange_worker(rank, world, port, q):
    """The bucket-split prover's exchange (plk_prover_shard_buckets) without a GPU: each
    rank's payload is its bucket-range shares of several commits (restated split,
    oracle/pyref.py msm_bucket_part at c = 20), 13 point words + a status word each, sent
    through the same ctypes all-gather callback the C++ prover calls and folded with
    plk_g1_sum; a degree status on one rank must reach every rank."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path[:0] = [str(ROOT), str(ROOT / "tests"), str(ROOT / "oracle")]
    import ctypes as C
    import torch.distributed as dist
    import pyref as P
    import dusk_plonk_amd as plk
    from dusk_plonk_amd.parallel import torch_allgather
    from dusk_plonk_amd.prover import ALLGATHER_FN

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g = dict(np.load(ROOT / "tests" / "golden" / "msm_golden.npz", allow_pickle=False))
        pts = P.g1_vec_from_np(g["srs"])
        ag = torch_allgather()

        def cb(_u, send, nbytes, recv):
            data = ag(C.string_at(send, nbytes))
            C.memmove(recv, data, len(data))
            return 0
        fn = ALLGATHER_FN(cb)
        slots = ["random", "sparse", "high_bits"]
        send = np.zeros((len(slots) + 1, 14), dtype=np.uint64)
        for i, sname in enumerate(slots):
            sc = P.fr_vec_from_np(g[f"{sname}_scalars"])
            send[i, :13] = P.g1_vec_to_np([P.msm_bucket_part(pts, sc, 20, rank, world)])[0]
        send[-1, 12] = 1
        send[-1, 13] = plk.PLK_E_DEGREE if rank == world - 1 else plk.PLK_OK
        recv = np.zeros((world, len(slots) + 1, 14), dtype=np.uint64)
        ok = fn(None, send.ctypes.data, send.nbytes, recv.ctypes.data) == 0
        for i, sname in enumerate(slots):
            ok &= np.array_equal(plk.plonk.g1_sum(recv[:, i, :13]).words, g[f"{sname}_result"])
        ok &= int(recv[:, -1, 13].max()) == plk.PLK_E_DEGREE
        q.put((rank, bool(ok)))
    finally:
        dist.destroy_process_group()


def test_bucket_split_prover_exchange_gloo_world2():
    out = _spawn(_bucket_exchange_worker, 2)
    assert out == {0: True, 1: True}


def _exchange_service_worker(rank, world, port, q):
    """parallel.ExchangeService (the sharded prover's exchange with several lanes per rank):
    3 lanes per rank, each a thread doing its own sequence of all-gathers of varying size,
    with lane timing skewed differently on every rank (so the lanes reach their exchanges in
    a different order on each rank) and one lane driven through the same ctypes callback type
    the C++ prover calls (plk_allgather_fn). Every result must be the rank-ordered
    concatenation; the service must then stop cleanly. gloo, CPU only."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, str(ROOT))
    import ctypes as C
    import random
    import threading
    import time
    import torch.distributed as dist
    from dusk_plonk_amd.parallel import ExchangeService
    from dusk_plonk_amd.prover import ALLGATHER_FN

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        svc = ExchangeService()
        L, counts = 3, [9, 7, 4]  # lanes stop after different numbers of exchanges

        def payload(r, lane, j):
            n = 14 * 8 * (1 + (lane + j) % 4)
            return bytes(((r * 131 + lane * 17 + j * 7 + i) & 0xFF) for i in range(n))

        errors = []

        def lane_thread(lane):
            ag = svc.allgather_for(lane)
            rng = random.Random(1000 * rank + lane)
            if lane == 1:  # through the C callback type, as prover.hip calls it
                def cb(_u, send, nbytes, recv):
                    data = ag(C.string_at(send, nbytes))
                    C.memmove(recv, data, len(data))
                    return 0
                fn = ALLGATHER_FN(cb)

                def call(data):
                    src = C.create_string_buffer(data, len(data))
                    dst = C.create_string_buffer(world * len(data))
                    if fn(None, C.cast(src, C.c_void_p), len(data), C.cast(dst, C.c_void_p)) != 0:
                        raise RuntimeError("callback failed")
                    return dst.raw
            else:
                call = ag
            for j in range(counts[lane]):
                # skew: rank 0 runs lane 0 slow and lane 2 fast, rank 1 the reverse
                slow = (lane == 0) if rank == 0 else (lane == 2)
                time.sleep(rng.uniform(0.0, 0.03) + (0.02 if slow else 0.0))
                got = call(payload(rank, lane, j))
                want = b"".join(payload(r, lane, j) for r in range(world))
                if got != want:
                    errors.append((lane, j))
        ts = [threading.Thread(target=lane_thread, args=(ln,)) for ln in range(L)]
        for t in ts:
            t.start()
        # the caller's own collectives on the default group run concurrently with the
        # service's (bench.py's barriers / timing reductions): they must not interleave
        import torch
        for _ in range(5):
            dist.barrier()
            x = torch.ones(1)
            dist.all_reduce(x)
            time.sleep(0.01 * (1 + rank))
        for t in ts:
            t.join(120)
        ok = not errors and not any(t.is_alive() for t in ts)
        svc.close()
        ok &= svc.requests == sum(counts) and svc.exchanges <= sum(counts)
        q.put((rank, bool(ok)))
    finally:
        dist.destroy_process_group()


def test_exchange_service_skewed_lanes_gloo_world2():
    out = _spawn(_exchange_service_worker, 2)
    assert out == {0: True, 1: True}


def _sharded_lanes_worker(rank, world, port, q, logn, lanes, srs_mult):
    """configs[4]'s multi-lane form: `lanes` prover lanes per rank, each sharded over the
    ranks through ONE parallel.ExchangeService, proving concurrently with rank-dependent
    skew. The SRS holds srs_mult x (n + 8) points, so with srs_mult >= 4 the last rank's
    slice starts past the trimmed SRS (the t_4 tail check must still run there), and the
    full SRS and the slices take different MSM window sizes: lane 0 proves once unsharded
    (full SRS, c = 17 wide buckets) before it is sharded (slices, c = 15), so its MSM
    workspace changes shape. Every proof must equal the unsharded plk_prove's bytes; an
    unsatisfied circuit fails with the degree error on every rank."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, str(ROOT))
    sys.path.insert(0, str(ROOT / "tests"))
    import random
    import threading
    import time
    import torch.distributed as dist
    from oracle_lib import random_fr
    import dusk_plonk_amd as plk
    from dusk_plonk_amd.parallel import ExchangeService, shard_prover_lane, srs_slice
    from dusk_plonk_amd.prover import Plonk, PlonkKey

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        tau = random_fr(1, seed=93)[0]
        ctx = plk.Context.default(0)
        n = 1 << logn
        pp = plk.PlonkParams.setup(logn, tau, ctx, n_points=srs_mult * (n + 8))

        def circ(seed):
            cs = Plonk()
            cs.synthetic_chain(n - 15, seed)
            cs.append_public(seed + 7)
            return cs
        prover, _ = PlonkKey.compile_composer(pp, b"lanes", circ(1))
        seeds = list(range(3, 3 + 2 * lanes))
        want = {s: prover.prove_composer(circ(s + 10), s)[0].raw_bytes() for s in seeds}
        lns = [prover.lane() for _ in range(lanes)]
        ok = lns[0].prove_composer(circ(seeds[0] + 10), seeds[0])[0].raw_bytes() == want[seeds[0]]
        svc = ExchangeService()
        sl = srs_slice(tau, pp.n, world, rank, ctx)
        for i, ln in enumerate(lns):
            shard_prover_lane(ln, tau, pp.n, slice_=sl, exchange=svc, lane_id=i)
        results, errors = {}, []

        def drive(i):
            rng = random.Random(100 * rank + i)
            try:
                for s in seeds[i::lanes]:
                    time.sleep(rng.uniform(0, 0.05) * (1 + (i + rank) % 2))
                    results[s] = lns[i].prove_composer(circ(s + 10), s)[0].raw_bytes()
                if i == lanes - 1:  # an unsatisfied circuit: the degree error everywhere
                    bad = circ(20)
                    bad.set_witness(5, 12345)
                    try:
                        lns[i].prove_composer(bad, 1)
                        errors.append("bad circuit proved")
                    except plk.PlonkError as e:
                        if e.status != plk.PLK_E_DEGREE:
                            errors.append(f"status {e.status}")
            except Exception as e:  # noqa: BLE001
                errors.append(repr(e))
        ts = [threading.Thread(target=drive, args=(i,)) for i in range(lanes)]
        for t in ts:
            t.start()
        for t in ts:
            t.join(600)
        svc.close()
        ok &= not errors and all(results.get(s) == want[s] for s in seeds)
        for ln in lns:
            ln.close()
        q.put((rank, bool(ok)))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_sharded_prover_lanes_exchange_service(plk, gpu_ctx):
    """2 ranks x 3 lanes through one ExchangeService per rank; SRS 4x the circuit's."""
    out = _spawn(_sharded_lanes_worker, 2, 14, 3, 4)
    assert out == {0: True, 1: True}


@pytest.mark.gpu
def test_sharded_prover_three_ranks_large_srs(plk, gpu_ctx):
    """3 ranks x 2 lanes, SRS 5x the circuit's: two ranks' slices lie past the trimmed SRS."""
    out = _spawn(_sharded_lanes_worker, 3, 12, 2, 5)
    assert out == {0: True, 1: True, 2: True}


def _sharded_2_20_worker(rank, world, port, q, mode="slices"):
    """BASELINE configs[4] at its own size: the headline 2^20 bench circuit proved with every
    commit split over the ranks (plk_prover_shard, gloo on one card here; RCCL over xGMI on a
    node), byte for byte against the committed oracle fixture tests/golden/proof_2_20.npz."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path[:0] = [str(ROOT), str(ROOT / "tests"), str(ROOT / "tests" / "golden")]
    import torch.distributed as dist
    import dusk_plonk_amd as plk
    from dusk_plonk_amd.parallel import ExchangeService, shard_prover_lane
    from dusk_plonk_amd.prover import PlonkKey
    from make_proof_2_20 import BLIND_SEED, LABEL, LOG_N, TAU_SEED, circuit
    from test_prover_oracle import tau_for

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g = dict(np.load(ROOT / "tests" / "golden" / "proof_2_20.npz", allow_pickle=False))
        tau, _ = tau_for(TAU_SEED)
        ctx = plk.Context.default(0)
        pp = plk.PlonkParams.setup(LOG_N, tau, ctx)
        cs = circuit()
        prover, vd = PlonkKey.compile_composer(pp, LABEL, cs)
        ok = np.array_equal(vd.comms, g["vk"])
        lane = prover.lane()
        svc = ExchangeService()
        shard_prover_lane(lane, tau, pp.n, ctx=ctx, exchange=svc, lane_id=0, mode=mode)
        proof, _ = lane.prove_composer(cs, BLIND_SEED)
        svc.close()
        ok &= proof.to_bytes() == g["scale"].tobytes()
        lane.close()
        q.put((rank, bool(ok)))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_sharded_prover_2_20_equals_fixture(plk, gpu_ctx):
    out = _spawn(_sharded_2_20_worker, 2)
    assert out == {0: True, 1: True}


@pytest.mark.gpu
def test_sharded_prover_2_20_bucket_split_equals_fixture(plk, gpu_ctx):
    """configs[4] with every commit split by bucket range (plk_prover_shard_buckets: c = 20,
    2 parts of 2^18 buckets), byte for byte against the committed 2^20 oracle proof."""
    out = _spawn(_sharded_2_20_worker, 2, "buckets")
    assert out == {0: True, 1: True}


def _rccl_world1_worker(rank, world, port, q, logn, lanes):
    """The RCCL data path of the sharded prover on the one GPU: torch.distributed over
    `nccl` (RCCL) at world size 1 on cuda:0. Exercises what the gloo rehearsals cannot:
    communicator init on the exchange thread, its torch.cuda.Stream, device staging of the
    payloads and `.cpu()` syncs while other lanes' kernels hold the CUs; plus the device
    forms of torch_allgather and gather_fold (ShardedPlonkParams). Every sharded proof must
    equal plk_prove's bytes (reference commit groups: prover.rs:133-136,194,262-265,440,452)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, str(ROOT))
    sys.path.insert(0, str(ROOT / "tests"))
    import threading
    import torch
    import torch.distributed as dist
    from oracle_lib import random_fr
    import dusk_plonk_amd as plk
    from dusk_plonk_amd.parallel import (ExchangeService, ShardedPlonkParams, shard_prover_lane,
                                         srs_slice, torch_allgather)
    from dusk_plonk_amd.prover import Plonk, PlonkKey

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    checks = {}
    try:
        checks["backend"] = dist.get_backend() == "nccl"
        ag = torch_allgather(None, dev)  # the byte all-gather's device path
        checks["allgather"] = ag(b"\x01\x02\x03") == b"\x01\x02\x03"
        tau = random_fr(1, seed=71)[0]
        ctx = plk.Context.default(0)
        n = 1 << logn
        pp = plk.PlonkParams.setup(logn, tau, ctx)
        # the sharded single MSM with its partials gathered from HBM
        spp = ShardedPlonkParams(logn, tau, ctx=ctx)
        coef = torch.from_numpy(random_fr(n, 9).view(np.int64)).to(dev)
        s = torch.cuda.current_stream().cuda_stream
        got = spp.commit_dev(coef.data_ptr(), n, s, dev)
        want = pp.commit_dev(coef.data_ptr(), n, s)
        checks["sharded_commit"] = np.array_equal(got.words, want.words)

        def circ(seed):
            cs = Plonk()
            cs.synthetic_chain(n - 15, seed)
            cs.append_public(seed + 7)
            return cs
        prover, _ = PlonkKey.compile_composer(pp, b"rccl", circ(1))
        seeds = list(range(5, 5 + 2 * lanes))
        want = {s_: prover.prove_composer(circ(s_ + 10), s_)[0].raw_bytes() for s_ in seeds}
        lns = [prover.lane() for _ in range(lanes)]
        svc = ExchangeService(None, dev)
        sl = srs_slice(tau, pp.n, world, rank, ctx)
        for i, ln in enumerate(lns):
            shard_prover_lane(ln, tau, pp.n, device=dev, slice_=sl, exchange=svc, lane_id=i)
        results, errors = {}, []

        def drive(i):
            try:
                for s_ in seeds[i::lanes]:
                    results[s_] = lns[i].prove_composer(circ(s_ + 10), s_)[0].raw_bytes()
            except Exception as e:  # noqa: BLE001
                errors.append(repr(e))
        ts = [threading.Thread(target=drive, args=(i,)) for i in range(lanes)]
        for t in ts:
            t.start()
        for t in ts:
            t.join(300)
        svc.close()
        checks["errors"] = errors
        checks["proofs"] = [results.get(s_) == want[s_] for s_ in seeds]
        checks["requests"] = (svc.requests, svc.exchanges)  # 4 commit groups per proof
        for ln in lns:
            ln.close()
        q.put((rank, checks))
    except Exception as e:  # noqa: BLE001
        checks["exception"] = repr(e)
        q.put((rank, checks))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_sharded_prover_rccl_world1(plk, gpu_ctx):
    """3 lanes sharded over an RCCL world of one (the device-tensor exchange runs for real)."""
    c = _spawn(_rccl_world1_worker, 1, 14, 3)[0]
    print(c)
    assert "exception" not in c, c
    assert c["backend"] and c["allgather"] and c["sharded_commit"], c
    assert not c["errors"] and all(c["proofs"]) and len(c["proofs"]) == 6, c
    assert c["requests"][0] == 4 * 6 and 1 <= c["requests"][1] <= 4 * 6, c


@pytest.mark.gpu
def test_rccl_in_process_device_exchange(plk, gpu_ctx):
    """RCCL (torch.distributed `nccl`) in the test process itself at world size 1: the
    device-tensor paths of the exchange (torch_allgather, gather_fold, ExchangeService with a
    device) run over librccl here, then the group is torn down."""
    import threading
    import torch
    import torch.distributed as dist
    from dusk_plonk_amd.parallel import ExchangeService, gather_fold, torch_allgather
    if dist.is_initialized():
        pytest.skip("a process group already exists in this process")
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()))
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        assert dist.get_backend() == "nccl"
        assert torch_allgather(None, dev)(b"rccl") == b"rccl"
        g = dict(np.load(ROOT / "tests" / "golden" / "msm_golden.npz", allow_pickle=False))
        part = np.stack([g["random_result"], g["sparse_result"]])
        res = gather_fold(part, [plk.PLK_OK, plk.PLK_OK], None, dev)
        assert np.array_equal(res[0].words, g["random_result"])
        assert np.array_equal(res[1].words, g["sparse_result"])
        svc = ExchangeService(None, dev)
        out = {}

        def lane(i):
            ag = svc.allgather_for(i)
            out[i] = [ag(bytes([i, j]) * (j + 1)) for j in range(5)]
        ts = [threading.Thread(target=lane, args=(i,)) for i in range(3)]
        for t in ts:
            t.start()
        for t in ts:
            t.join(60)
        svc.close()
        assert all(out[i] == [bytes([i, j]) * (j + 1) for j in range(5)] for i in range(3))
        assert svc.requests == 15
    finally:
        dist.destroy_process_group()


def test_window_bits_mirror_choose_c(monkeypatch):
    """parallel.window_bits / bucket_parts_ok follow srs.hip choose_c + msm_prepare_srs
    (round-5 advisor: PLK_MSM_C = 18 runs as 17, 21 / 23 are refused, 2^14 / 2^13 points take
    c = 13 / 12), checked against pyref.msm_effective_c."""
    import pyref as P
    from dusk_plonk_amd.parallel import bucket_parts_ok, window_bits

    monkeypatch.delenv("PLK_MSM_C", raising=False)
    for n, c in [((1 << 20) + 8, 20), ((1 << 16) + 8, 17), (1 << 15, 15), ((1 << 14) + 8, 13),
                 (1 << 13, 12), (1 << 12, 10), (1 << 9, 8)]:
        assert window_bits(n) == c
    monkeypatch.setenv("PLK_MSM_C", "18")
    assert window_bits(1 << 10) == 17 == P.msm_effective_c(18)
    assert bucket_parts_ok(1 << 10, 4) and not bucket_parts_ok(1 << 10, 8)
    for bad in ("21", "23", "7", "x"):
        monkeypatch.setenv("PLK_MSM_C", bad)
        assert window_bits(1 << 20) == 20 and window_bits(1 << 14) == 13
    monkeypatch.setenv("PLK_MSM_C", "20")
    assert bucket_parts_ok(1 << 10, 8) and not bucket_parts_ok(1 << 10, 64)
    monkeypatch.delenv("PLK_MSM_C")
    assert bucket_parts_ok(1 << 14, 1) and not bucket_parts_ok(1 << 14, 2)
