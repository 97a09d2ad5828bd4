#!/usr/bin/env python3
"""bench.py — the BASELINE.json metric: PLONK prover constraints/s (BLS12-381) on MI355X.

Default step (mode "prove"): every prover lane of every rank completes ONE full
`Prover::create_proof` (src/prover.rs:67-474) at n = 2^k (default k = 20) on the synthetic
arithmetic-chain circuit of SURVEY §8d item 4 plus one public input: host synthesis of a fresh
witness (C++ composer, overlapped with the previous proof) + the five rounds + both openings
on the GPU, proof back on the host. The key (PlonkKey::compile) and the SRS are built once per
GPU outside the timed region and shared by the GPU's lanes (plk_prover). Per proof the GPU
runs 13 transforms (6 idft(n): 4 wires, z, PI; 6 coset_dft(8n): z, 4 wires, PI; 1
coset_idft(8n)) and 11 MSMs; the reference's other 6 transforms are per-key constants here
(4 sigma dft(n): the key holds their Lagrange values; L1's idft(n) + coset_dft(8n)).

value = constraints/s = n * proofs / max-over-ranks time.
  * default: proof batches — every rank proves its own proofs (weak scaling, no
    data-path collective; torch.distributed only for the barrier and the max reduction);
  * --shard-msm (BASELINE configs[4]): every rank proves the SAME proofs and each commit is
    split over the ranks by bucket range (plk_prover_shard_buckets, round 6) or, where the
    SRS does not allow that split, by SRS slice (plk_prover_shard): one RCCL all-gather of
    partial points per commit group, host fold — strong scaling of proof latency.
After the timed region the prove line also carries (unless --no-extras) `msm_shard`: one 2^k
MSM split over ALL ranks by bucket range (RCCL all-gather + host fold, checked against the
unsplit commit; at world 1 the lone MSM against the oracle) — the north star's MSM scaling
curve, one point per run — and `n_2_16`: the metric's second size, a short 2^16 prove run.
Every line carries `build_id` (plk_build_info, checked against this tree before anything runs).
`--gpus N` without a launcher starts N ranks itself (torch.distributed.run, 127.0.0.1).
Other modes: hotpath (only the NTT/MSM calls of one proof), ntt / msm (BASELINE configs[1] /
[2], checked bit-exact against the oracle after the timed loop).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)
# The accumulation's own ceiling: v_mad_u64_u32 issue rate. The guide lists no integer-mad
# peak; this one is MEASURED by tools/ubench_mad.hip (3.53e13/s chip-wide at 4 waves/SIMD,
# 3.2e13 at 2; dependent latency = issue cost).
VALU_MAD_PEAK = 3.53e13
# The VALU issue ceiling: every SIMD issuing every cycle at the chip's max clock
# (MI355X_MICROARCH.md: 256 CUs x 4 SIMDs, 2400 MHz). A loop's demand is its compiled
# instruction mix priced at the measured issue cost of each instruction (tools/ubench_issue.hip,
# profiles/r03_ubench_issue.txt: 64-bit ops and v_mad_u64_u32 ~4.3-4.5 cycles, 32-bit ALU ~2.3).
SIMD_CYCLES_PEAK = 1024 * 2.4e9
FR_MUL_PEAK = 1.64e11  # ffr.hpp Fr multiplies/s chip-wide, tools/ubench_limbs.hip (measured)
VALU_MAD_PEAK_SOURCE = ("measured by tools/ubench_mad.hip (independent v_mad_u64_u32 chains, "
                        "4 waves/SIMD, whole chip); MI355X_MICROARCH.md lists no integer-mad peak")
# Formula count of one XYZZ mixed addition in the redundant Fp form (ffr.hpp / g1r.hpp):
# 8 products x 196 + 2 squares x 105 + 9 Montgomery reductions x 196; used only when the
# compiled count (tools/isa_count.py on libplk.so) cannot be read.
MADS_PER_MIXED_ADD = 8 * 196 + 2 * 105 + 9 * 196
_ISA = {}


# k_accumulate's two instantiations (csrc/msm_acc.hip k_accumulate<HAS_INF, LONE>): prover
# lanes run the grouped-product form at 2 waves per SIMD, lone commits the plain chains at 3
ACC_LANE = ("k_accumulateILb0ELb0E", "k_accumulate<false, false>")
ACC_LONE = ("k_accumulateILb0ELb1E", "k_accumulate<false, true>")


def compiled_loop(kernel: str = ACC_LANE[0]) -> dict:
    """The kernel's loop body as compiled (largest basic block of its gfx950 code in
    libplk.so, tools/isa_count.py): v_mad_u64_u32 count, instruction count and the VALU issue
    cycles of the mix at the measured per-instruction costs (tools/ubench_issue.hip)."""
    if kernel not in _ISA:
        try:
            sys.path.insert(0, str(ROOT / "tools"))
            import isa_count
            lib = os.environ.get("PLK_LIB") or str(ROOT / "dusk-plonk_amd" / "libplk.so")
            r = isa_count.largest_block(Path(lib), kernel)
            _ISA[kernel] = ({"v_mad_u64_u32": r["v_mad_u64_u32"], "instructions": r["instructions"],
                             "valu_instructions": sum(n for op, n in r["mix"].items()
                                                      if op.startswith("v_")),
                             "s_nop": r["mix"].get("s_nop", 0),
                             "valu_cycles": isa_count.valu_cycles(r["mix"]),
                             "source": "compiled loop body (tools/isa_count.py on libplk.so)"}
                            if r else None)
        except Exception as e:  # noqa: BLE001 — llvm-objdump missing: formula fallback
            _ISA[kernel] = {"v_mad_u64_u32": MADS_PER_MIXED_ADD, "instructions": None,
                            "valu_cycles": MADS_PER_MIXED_ADD * 4.53 * 1.3,
                            "source": f"formula (compiled count unavailable: {e!r})"}
        if _ISA[kernel] is None:
            _ISA[kernel] = {"v_mad_u64_u32": MADS_PER_MIXED_ADD, "instructions": None,
                            "valu_cycles": MADS_PER_MIXED_ADD * 4.53 * 1.3,
                            "source": "formula (kernel not found in libplk.so)"}
    return _ISA[kernel]


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one per GPU). Without WORLD_SIZE in the environment and N > 1, "
                         "bench.py launches N ranks itself (torch.distributed.run); under a "
                         "launcher N must equal WORLD_SIZE")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--log-n", type=int, default=20)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="CPU baseline threads; 0 = OMP_NUM_THREADS if set (the GPU box's CPU "
                         "share per GPU), else every core in this process's affinity mask")
    ap.add_argument("--lanes", type=int, default=0,
                    help="concurrent prover lanes per GPU (prove mode): independent contexts "
                         "with their own streams, each driven by a host thread. 0 = 12 at "
                         "n >= 2^18, 14 at 2^15..2^17, 16 below (2 HIP hardware queues per "
                         "lane; round-3 / round-4 lane sweeps in DESIGN §6)")
    ap.add_argument("--fit-lanes", action="store_true",
                    help="prove mode: lower the lanes per GPU (same on every rank) when the "
                         "warmup's synthesis would need > 90 %% of a rank's CPU share")
    ap.add_argument("--hw-queues", type=int, default=0,
                    help="HIP hardware queues per process (GPU_MAX_HW_QUEUES, HIP default 4); "
                         "0 = min(32, 2 x lanes): more lanes than queues serialise on them")
    ap.add_argument("--mode", choices=["prove", "hotpath", "ntt", "msm"], default="prove",
                    help="prove: full Prover::create_proof (synthesis + 5 rounds + openings); "
                         "hotpath: only the 19 NTTs + 11 MSMs of one proof; ntt / msm: "
                         "BASELINE.json configs[1] / configs[2], the standalone 2^k dft+idft "
                         "pair or G1 MSM, bit-exact against the oracle after the timed loop")
    ap.add_argument("--dist-backend", choices=["nccl", "gloo"], default="nccl",
                    help="process group for the barrier / max-over-ranks timing (nccl = RCCL); "
                         "gloo only to rehearse several ranks on one GPU")
    ap.add_argument("--shard-msm", action="store_true",
                    help="BASELINE configs[4]: all ranks prove the same proofs, every commit "
                         "split over the ranks (--shard-split; RCCL all-gather of partial points "
                         "+ host fold); NTT / elementwise rounds replicated. With --mode msm: "
                         "ONE MSM per step split over the ranks (--msm-split)")
    ap.add_argument("--shard-split", choices=["auto", "buckets", "slices"], default="auto",
                    help="--shard-msm in prove mode: split every commit by bucket range "
                         "(plk_prover_shard_buckets: every rank holds the whole SRS and reduces "
                         "1/G of the buckets) or by SRS slice (plk_prover_shard); auto = buckets "
                         "where the SRS allows G parts (c >= 17, >= 2^14 buckets per part)")
    ap.add_argument("--msm-split", choices=["buckets", "points"], default="buckets",
                    help="--mode msm --shard-msm: by bucket range (each rank sorts, accumulates "
                         "and reduces 1/G of the buckets; plk_commit_batch_dev_part) or by SRS "
                         "slice (each rank the whole Pippenger over 1/G of the points)")
    ap.add_argument("--no-extras", action="store_true",
                    help="prove mode: skip the extra measurements attached to the line after the "
                         "timed region (n_2_16: the metric's second size; msm_shard: one 2^k MSM "
                         "split over all ranks by bucket range, the north star's MSM scaling curve)")
    ap.add_argument("--bucket-parts", type=int, default=1,
                    help="--mode msm on ONE GPU: run the MSM as P bucket-range parts one after "
                         "the other (what each of P GPUs would run under --shard-msm), timing "
                         "each part; the line reports the per-part times and checks the fold")
    return ap.parse_args()


def rand_fr_dev(torch, n: int, seed: int, device):
    """Uniform Fr (Montgomery limbs) generated on the host, moved to HBM once."""
    sys.path.insert(0, str(ROOT / "tests"))
    from oracle_lib import random_fr  # sampler only (numpy); no oracle arithmetic
    return torch.from_numpy(random_fr(n, seed).view(np.int64)).to(device)


class HotPath:
    def __init__(self, plk, torch, k: int, device, seed: int, shard: bool = False):
        self.plk, self.torch, self.k = plk, torch, k
        n = 1 << k
        self.n = n
        self.ctx = plk.Context.default(device.index or 0)
        self.fft = plk.Fft(k, self.ctx)
        self.fft8 = plk.Fft(k + 3, self.ctx)
        tau = np.asarray(np.random.default_rng(0x5EED).integers(1, 2**62, 4), dtype=np.uint64)
        tau[3] &= np.uint64(0x0FFFFFFFFFFFFFFF)
        self.shard = shard
        if shard:  # this rank's slice of the 2^k + 8 powers
            from dusk_plonk_amd.parallel import ShardedPlonkParams
            self.pp = ShardedPlonkParams(k, tau, ctx=self.ctx)
            # partials all-gathered from HBM over RCCL; from host memory under gloo
            self.device = device if torch.distributed.get_backend() == "nccl" else None
        else:
            self.pp = plk.PlonkParams.setup(k, tau, self.ctx)  # 2^k + 8 powers
        r = lambda s: rand_fr_dev(torch, n, seed + s, device)  # noqa: E731
        self.wire_vals = [r(i) for i in range(4)]
        self.sigma_coef = [r(10 + i) for i in range(4)]
        self.z_vals, self.pi_vals, self.l1_vals = r(20), r(21), r(22)
        e = lambda: torch.empty((n, 4), dtype=torch.int64, device=device)  # noqa: E731
        self.wire_coef = [e() for _ in range(4)]
        self.sigma_eval = [e() for _ in range(4)]
        self.z_coef, self.pi_coef, self.l1_coef = e(), e(), e()
        self.ev8 = [torch.empty((8 * n, 4), dtype=torch.int64, device=device) for _ in range(7)]
        self.quot8 = rand_fr_dev(torch, 8 * n, seed + 30, device)
        self.t_coef = torch.empty((8 * n, 4), dtype=torch.int64, device=device)
        torch.cuda.synchronize()
        self.ntt_ms = {"n": [], "8n": []}
        self.msm_acc_ms = []
        self.msm_adds = []

    def _ntt(self, fft, src, dst, length, direction, coset, key, s, timed):
        if timed:
            e0 = self.torch.cuda.Event(enable_timing=True)
            e1 = self.torch.cuda.Event(enable_timing=True)
            e0.record()
        fft.ntt_dev(src.data_ptr(), dst.data_ptr(), length, direction, coset, s)
        if timed:
            e1.record()
            self.ntt_ms[key].append((e0, e1))

    def _commit(self, bufs, length, s, timed):
        """One batch of independent commits (the reference's commit groups)."""
        if self.shard:
            cs = self.pp.commit_batch_dev([(b.data_ptr(), length) for b in bufs], s, self.device)
        else:
            cs = self.pp.commit_batch_dev([(b.data_ptr(), length) for b in bufs], s)
        if timed:
            ms, adds, _ = (self.pp.local if self.shard else self.pp).last_msm_stats()
            self.msm_acc_ms.append(ms)
            self.msm_adds.append(adds)
        return cs

    def step(self, timed=False):
        n, s = self.n, self.torch.cuda.current_stream().cuda_stream
        coms = []
        for w in range(4):  # round 1
            self._ntt(self.fft, self.wire_vals[w], self.wire_coef[w], n, -1, False, "n", s, timed)
        coms += self._commit(self.wire_coef, n, s, timed)  # 4 wire commits, one batch
        for i in range(4):  # round 2
            self._ntt(self.fft, self.sigma_coef[i], self.sigma_eval[i], n, 1, False, "n", s, timed)
        self._ntt(self.fft, self.z_vals, self.z_coef, n, -1, False, "n", s, timed)
        coms += self._commit([self.z_coef], n, s, timed)
        self._ntt(self.fft, self.pi_vals, self.pi_coef, n, -1, False, "n", s, timed)  # round 3
        self._ntt(self.fft, self.l1_vals, self.l1_coef, n, -1, False, "n", s, timed)
        srcs = [self.z_coef, *self.wire_coef, self.pi_coef, self.l1_coef]
        for i, src in enumerate(srcs):
            self._ntt(self.fft8, src, self.ev8[i], n, 1, True, "8n", s, timed)
        self._ntt(self.fft8, self.quot8, self.t_coef, 8 * n, -1, True, "8n", s, timed)
        coms += self._commit([self.t_coef[j * n:(j + 1) * n] for j in range(4)], n, s, timed)
        # the two opening witnesses are independent (both v challenges are drawn before
        # either commit, prover.rs:422-452): one batch, same length as the real witnesses
        coms += self._commit(self.wire_coef[:2], n, s, timed)
        return coms


BENCH_TAU_SEED = 0x5EED


def bench_tau():
    tau = np.asarray(np.random.default_rng(BENCH_TAU_SEED).integers(1, 2**62, 4), dtype=np.uint64)
    tau[3] &= np.uint64(0x0FFFFFFFFFFFFFFF)
    return tau


def bench_circuit(Plonk, chain_gates: int, seed: int):
    """The bench circuit: Plonk::initialize (6 gates), `chain_gates` chained gates
    x' = x*y + x (fresh SplitMix64 witness from `seed`) and one public input (lib.rs:708-719),
    so the per-proof PI transforms the reference runs (prover.rs:229, quotient_poly.rs:145)
    are in the step."""
    cs = Plonk()
    cs.synthetic_chain(chain_gates, seed)
    cs.append_public((seed * 0x9E3779B97F4A7C15 + 12345) % (1 << 250))
    return cs


class ProverBase:
    """Per GPU, built once outside the timed region: the SRS (2^k + 8 powers, window table
    in HBM) and the compiled proving key, shared by all of this GPU's prover lanes."""

    def __init__(self, plk, k: int, ctx):
        from dusk_plonk_amd.prover import PlonkKey, Plonk
        self.plk, self.k, self.n, self.ctx = plk, k, 1 << k, ctx
        self.Plonk = Plonk
        self.chain = self.n - 8 - 6 - 1  # m = n - 8 gates: 6 initial + chain + 1 public
        self.tau = bench_tau()
        self.pp = plk.PlonkParams.setup(k, self.tau, ctx=ctx)
        self.prover, self.vd = PlonkKey.compile_composer(
            self.pp, b"bench", bench_circuit(Plonk, self.chain, 1))
        self.gates = self.prover.m


class ProofLane:
    """One concurrent prover (plk_prover over the shared key: own stream, MSM workspace and
    scratch) with its own synthesis thread: synthesis of proof k+1 (host C++ composer, GIL
    released in ctypes) overlaps the GPU proving of proof k, as in a proof server; both are
    inside the timed loop."""

    def __init__(self, base: ProverBase, seed: int):
        import concurrent.futures as cf
        self.base = base
        self.lane = base.prover.lane()
        self.seed = seed
        self.synth_s, self.prove_s, self.synth_all = [], [], []
        self.last = None  # (seed, raw proof bytes) of this lane's latest proof
        self.pool = cf.ThreadPoolExecutor(1)
        self.next = self.pool.submit(self._synth, self.seed + 1)

    def _synth(self, seed):
        t0 = time.perf_counter()
        cs = bench_circuit(self.base.Plonk, self.base.chain, seed)  # a fresh witness
        return cs, time.perf_counter() - t0

    def step(self, timed=False):
        self.seed += 1
        cs, ts = self.next.result()
        self.next = self.pool.submit(self._synth, self.seed + 1)
        t1 = time.perf_counter()
        proof, pi = self.lane.prove_composer(cs, self.seed)
        t2 = time.perf_counter()
        self.synth_all.append(ts)
        self.last = (self.seed, proof.raw_bytes())
        if timed:
            self.synth_s.append(ts)
            self.prove_s.append(t2 - t1)
        return proof


def recheck_proofs(lanes, checker) -> tuple[int, list]:
    """The credited configuration checked byte for byte: every lane's last timed proof
    (circuit and blinding from its seed) proved again on `checker` with no other lane
    running. A race between concurrent lanes (shared window table, per-lane workspaces,
    readback stamps) would make the concurrent proof differ from the lone one."""
    bad = []
    for ln in lanes:
        seed, got = ln.last
        cs = bench_circuit(ln.base.Plonk, ln.base.chain, seed)
        want = checker.lane.prove_composer(cs, seed)[0].raw_bytes()
        if want != got:
            bad.append(seed)
    return len(lanes), bad


def host_core_budget(dist, world, lanes, step_s, share=None) -> dict:
    """Host cores the proof server needs against the cores it has. Each lane synthesises one
    fresh witness per step beside the GPU work (synthesis time measured in the warmup), so a
    rank needs lanes x synth_s / step_s cores. The GPU box gives every GPU its own CPU share
    (cpu_share: affinity, cgroup quota and the OMP_NUM_THREADS share), so each rank's need is
    compared with ITS OWN share; `ratio` is the largest need / share over the ranks (the same
    on every rank), and the per-host sums are reported beside it."""
    import socket
    ts = [s for ln in lanes for s in ln.synth_all]
    synth = float(np.mean(ts)) if ts else 0.0
    need = len(lanes) * synth / max(step_s, 1e-9)
    share = share or cpu_share()
    avail = float(share["available"])
    mine = {"host": socket.gethostname(), "need": need, "available": avail}
    ranks = [mine]
    if world > 1:
        ranks = [None] * world
        dist.all_gather_object(ranks, mine)
    hosts = {}
    for r in ranks:
        h = hosts.setdefault(r["host"], {"ranks": 0, "need": 0.0, "available": 0.0})
        h["ranks"] += 1
        h["need"] += r["need"]
        h["available"] += r["available"]
    ratio = max(r["need"] / max(r["available"], 1e-9) for r in ranks)
    return {"needed_per_rank": need, "available_per_rank": avail, "ratio": ratio,
            "oversubscribed": ratio > 0.9, "per_host": hosts}


def cpu_baseline(k: int, pp, threads: int):
    """Restated reference CPU path (oracle/plk_oracle.c, OpenMP) on a bounded sample:
    one MSM(2^k) on the same SRS, one dft(2^k), one coset_dft(2^(k+3)); the per-proof
    hot-path time is 11*msm + 11*ntt(n) + 8*ntt(8n)."""
    sys.path.insert(0, str(ROOT / "tests"))
    import oracle_lib
    orc = oracle_lib.load()
    n = 1 << k
    pts = pp.points(0, n)
    sc = oracle_lib.random_fr(n, 77)
    v8 = oracle_lib.random_fr(8 * n, 78)
    t0 = time.perf_counter()
    orc.msm(pts, sc, threads)
    t_msm = time.perf_counter() - t0
    t0 = time.perf_counter()
    orc.dft(sc, k, threads)
    t_ntt = time.perf_counter() - t0
    t0 = time.perf_counter()
    orc.coset_dft(v8, k + 3, threads)
    t_ntt8 = time.perf_counter() - t0
    per_proof = 11 * t_msm + 11 * t_ntt + 8 * t_ntt8
    return {
        "value": n / per_proof, "unit": "constraints/s", "cores": threads, "kind": "port",
        "host": host_info(),
        "sample": (f"oracle/plk_oracle.c (restated reference CPU path, OpenMP {threads} threads): "
                   f"1x MSM(2^{k}) {t_msm:.2f}s, 1x dft(2^{k}) {t_ntt:.3f}s, "
                   f"1x coset_dft(2^{k + 3}) {t_ntt8:.3f}s; per-proof hot path = "
                   f"11*msm + 11*ntt(n) + 8*ntt(8n) = {per_proof:.2f}s"),
    }


def cpu_share() -> dict:
    """Cores this process may use: the affinity mask, capped by a cgroup CPU quota (the GPU
    box gives each GPU a share of the machine), and the whole machine's count."""
    hi = host_info()
    usable = hi["usable_cores"] or 1
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        pass
    avail = max(1, min(usable, int(quota))) if quota else usable
    # the GPU box allots each GPU a CPU share and says so in OMP_NUM_THREADS: worker pools
    # stay within it (the rest of the machine belongs to the other GPUs' jobs)
    env = os.environ.get("OMP_NUM_THREADS", "")
    share = int(env) if env.isdigit() and int(env) > 0 else None
    if share:
        avail = min(avail, share)
    return {"available": avail, "affinity": usable, "cgroup_quota_cpus": quota,
            "omp_num_threads": share, "machine_cores": hi["nproc"], "cpu_model": hi["cpu_model"]}


def cpu_concurrent(gates, wit, srs, vk, procs: int, n: int) -> dict:
    """MEASURED concurrent CPU proof throughput: `procs` independent restated-reference proofs
    (tests/oracle_worker.py, one OS process and one thread each — the throughput-optimal way
    to use cores for a prover whose quotient loop is sequential) started together.
    rate_sum = sum of n / create_proof time over the processes (their proofs run at once);
    window = procs * n / (last end - first create_proof start), which also charges any
    non-overlap."""
    import subprocess
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        f = Path(d) / "inputs.npz"
        np.savez(f, gates=gates, witness=wit, srs=srs, vk=vk)
        env = dict(os.environ, OMP_NUM_THREADS="1")
        ps = [subprocess.Popen([sys.executable, str(ROOT / "tests" / "oracle_worker.py"), str(f),
                                "1", str(100 + i)], stdout=subprocess.PIPE, text=True, env=env)
              for i in range(procs)]
        outs = []
        for p in ps:
            o, _ = p.communicate(timeout=900)
            if p.returncode != 0:
                raise RuntimeError(f"oracle worker failed ({p.returncode})")
            outs.append(json.loads(o.strip().splitlines()[-1]))
    rate_sum = sum(n / o["create_proof_s"] for o in outs)
    window = max(o["end"] for o in outs) - min(o["prove_start"] for o in outs)
    return {"value": rate_sum, "unit": "constraints/s", "procs": procs, "n": n,
            "create_proof_s": [round(o["create_proof_s"], 3) for o in outs],
            "window_value": procs * n / window, "window_s": window}


def cpu_baseline_full(k: int, pp, threads: int, k_sample: int = 16, gpu_value=None,
                      gpu_value_16=None):
    """Restated reference CPU prover (oracle/plk_prover_oracle.c: key compile + create_proof
    in the reference's order and cost structure, OpenMP where the reference uses rayon,
    sequential where it is sequential — notably the quotient loop's one v_h inversion per 8n
    point, quotient_poly.rs:99-107), two ways:
      * value (MEASURED throughput): as many independent single-thread proofs at 2^k_sample as
        this process has cores, run at once (cpu_concurrent) — the CPU used as a proof server
        uses it. Per-constraint CPU cost grows with n (MSM window, NTT depth), so the 2^16
        rate bounds the CPU's 2^20 throughput from above: the GPU/CPU ratio is conservative;
      * latency: ONE proof on `threads` threads (the reference's rayon prover on the GPU's
        CPU share): a full proof at 2^k_sample timed by phase, composed to 2^k with MSM / NTT
        timed at the 2^k sizes; the direct 2^20 timing is profiles/r02_cpu_full_n20.json."""
    sys.path.insert(0, str(ROOT / "tests"))
    import oracle_lib
    from dusk_plonk_amd.prover import Plonk
    orc = oracle_lib.load()
    ks = min(k, k_sample)
    n, ns = 1 << k, 1 << ks
    cs = bench_circuit(Plonk, ns - 15, 77)
    gates, wit = cs.export()
    trim = (1 << (gates.shape[0] + 6 - 1).bit_length()) + 8
    srs = pp.points(0, trim)
    res = orc.prove(gates, wit, srs, b"cpu-baseline", 5, threads)
    tm = res["timing_ns"].astype(np.float64) / 1e9
    prove_s, msm_s, ntt_s = tm[6], tm[1], tm[2]
    other_s = prove_s - msm_s - ntt_s  # quotient loop, grand product, openings, transcript
    if ks == k:
        t_msm = msm_s / 11
        per_proof = prove_s
        t_ntt = t_ntt8 = float("nan")
    else:
        pts = pp.points(0, n)
        sc = oracle_lib.random_fr(n, 77)
        v8 = oracle_lib.random_fr(8 * n, 78)
        t0 = time.perf_counter()
        orc.msm(pts, sc, threads)
        t_msm = time.perf_counter() - t0
        t0 = time.perf_counter()
        orc.dft(sc, k, threads)
        t_ntt = time.perf_counter() - t0
        t0 = time.perf_counter()
        orc.coset_dft(v8, k + 3, threads)
        t_ntt8 = time.perf_counter() - t0
        per_proof = 11 * t_msm + 11 * t_ntt + 8 * t_ntt8 + other_s * (n / ns)
    share = cpu_share()
    conc = cpu_concurrent(gates, wit, srs, res["vk"], share["available"], ns)
    direct = None
    f = ROOT / "profiles" / "r02_cpu_full_n20.json"
    if k == 20 and f.exists():
        try:
            direct = json.loads(f.read_text())
        except ValueError:
            direct = None
    # the concurrent 2^20 throughput measured directly on the GPU box (tools/cpu_node_n20.py:
    # 16 single-thread 2^20 proofs at once, ~5 minutes, too long for every bench run)
    node20 = None
    f20 = ROOT / "profiles" / "r03_cpu_node_n20.json"
    if k == 20 and f20.exists():
        try:
            d20 = json.loads(f20.read_text())
            node20 = {"value": d20["window_constraints_per_s"], "unit": "constraints/s",
                      "procs": d20["procs"], "n": d20["n"],
                      "create_proof_s": [min(d20["create_proof_s"]), max(d20["create_proof_s"])],
                      "window_s": d20["window_s"], "latency_16_threads_s": d20.get("latency_create_proof_s"),
                      "source": "profiles/r03_cpu_node_n20.json (stored measurement, tools/cpu_node_n20.py)"}
        except (ValueError, KeyError):
            node20 = None
    out = {
        "value": conc["value"], "unit": "constraints/s", "cores": conc["procs"], "kind": "port",
        "value_log_n": ks,
        "value_note": (f"`value` is measured in this run at n=2^{ks}" + (
            f", not at the line's 2^{k}: {conc['procs']} concurrent 2^{k} proofs take ~5 minutes "
            "(too long for every run); the stored 2^20 measurement of the same kind is "
            "`concurrent_2_20` (ratio `gpu_over_measured_2_20_share`), and `gpu_16_over_cpu_16` "
            "compares the line's own 2^16 figure (n_2_16) with `value` at the same size"
            if ks != k else "")),
        "measure": (f"MEASURED throughput of {conc['procs']} concurrent independent proofs at "
                    f"n=2^{ks} (one process and thread each, every core of this process's "
                    "share); an upper bound of the CPU's 2^20 throughput"),
        "host": share,
        "concurrent": conc,
        "concurrent_2_20": node20,
        "latency": {
            "value": n / per_proof, "unit": "constraints/s", "threads": threads, "n": n,
            "seconds_per_proof": per_proof, "composed": ks != k,
            "direct_2_20": ({"seconds": direct.get("create_proof_s", direct.get("seconds")),
                             "source": "profiles/r02_cpu_full_n20.json"} if direct else None),
            "note": "ONE proof on `threads` threads: the reference's own constraints/s reading"},
        "sample": (f"oracle/plk_prover_oracle.c (restated reference CPU prover): "
                   f"{conc['procs']} concurrent single-thread proofs at 2^{ks}, create_proof "
                   f"{min(conc['create_proof_s']):.1f}-{max(conc['create_proof_s']):.1f} s each; "
                   f"one 2^{ks} proof on {threads} threads = {prove_s:.2f} s (MSM {msm_s:.2f} s, "
                   f"NTT {ntt_s:.2f} s, quotient loop {tm[3]:.2f} s, grand product {tm[4]:.2f} s, "
                   f"openings {tm[5]:.2f} s)" + (
                       "" if ks == k else
                       f"; latency at 2^{k} = 11 x MSM(2^{k}) {t_msm:.2f} s + 11 x dft(2^{k}) "
                       f"{t_ntt:.3f} s + 8 x coset_dft(2^{k + 3}) {t_ntt8:.3f} s + O(n) phases x "
                       f"{n // ns} = {per_proof:.1f} s")),
    }
    mc = share["machine_cores"] or conc["procs"]
    out["node_projection"] = {
        "value": conc["value"] * mc / conc["procs"], "cores": mc,
        "note": f"the measured per-core throughput x all {mc} cores of the machine (independent "
                "processes; not measured beyond this process's share)"}
    if gpu_value:
        out["ratio"] = {"gpu_over_cpu_share": gpu_value / conc["value"],
                        "gpu_over_node_projection": gpu_value / out["node_projection"]["value"],
                        "gpu_over_latency": gpu_value / out["latency"]["value"]}
        if node20:
            out["ratio"]["gpu_over_measured_2_20_share"] = gpu_value / node20["value"]
        if gpu_value_16:
            out["ratio"]["gpu_16_over_cpu_16"] = gpu_value_16 / conc["value"]
    return out


def stored_cpu_baseline(k: int, world: int, gpu_value: float):
    """A multi-rank line's CPU baseline: the STORED measurement of the restated reference
    prover on one GPU's CPU share (profiles/r03_cpu_node_n20.json: 16 concurrent
    single-thread 2^20 proofs, tools/cpu_node_n20.py), not re-measured at world > 1 (each
    rank's host share is busy synthesising its lanes' witnesses). The N-GPU comparison is
    against N such shares."""
    f = ROOT / "profiles" / "r03_cpu_node_n20.json"
    try:
        d = json.loads(f.read_text())
    except (OSError, ValueError):
        return {"source": "stored (unavailable)", "value": None, "unit": "constraints/s"}
    per_share = d["window_constraints_per_s"]
    return {"source": f"stored: {f.relative_to(ROOT)} (tools/cpu_node_n20.py, measured on the "
                      "GPU box)",
            "kind": "port", "unit": "constraints/s", "n": d.get("n"),
            "value": per_share * world, "cores": d["procs"] * world,
            "per_share": {"value": per_share, "cores": d["procs"]},
            "sample": (f"{d['procs']} concurrent single-thread restated-reference proofs at "
                       f"n=2^{int(d['n']).bit_length() - 1} per GPU share, x {world} shares"
                       + ("" if k == 20 else f" (stored at 2^20; this line is 2^{k})")),
            "ratio": {"gpu_over_cpu_shares": gpu_value / (per_share * world)}}


def host_info():
    """nproc, usable cores and the CPU model of the machine the baseline ran on."""
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        usable = len(os.sched_getaffinity(0))
    except AttributeError:
        usable = os.cpu_count()
    return {"nproc": os.cpu_count(), "usable_cores": usable, "cpu_model": model}


def stored_clock(form_name: str):
    """The stored DVFS reading of a k_accumulate form (profiles/r06_effective_clock.json: the
    effective shader clock from GRBM_GUI_ACTIVE and the VALU activity per wave from the SQ
    counters on the round-6 final code, one --pmc pass each, tools/recipes.py counters), or
    None."""
    f = Path(__file__).resolve().parent / "profiles" / "r06_effective_clock.json"
    try:
        d = json.loads(f.read_text()).get(form_name)
    except (OSError, ValueError):
        return None
    return d if isinstance(d, dict) and d.get("effective_ghz") else None


def valu_roofline(adds_per_s, form=ACC_LANE):
    """k_accumulate against its binding ceiling, VALU issue: each mixed addition's compiled
    instruction mix (of the instantiation that ran: `form`) priced at the measured
    per-instruction issue costs, per wave of 64 additions, against every SIMD issuing every
    cycle (SIMD-cycles/s). The v_mad_u64_u32 rate against its own measured peak is kept beside
    it."""
    isa = compiled_loop(form[0])
    achieved = adds_per_s / 64.0 * isa["valu_cycles"]
    mads = adds_per_s * isa["v_mad_u64_u32"]
    clk = stored_clock(form[1])
    dvfs = None
    if clk:  # the clock the chip holds under this kernel, and how busy its VALU is there
        ghz = clk["effective_ghz"]
        # (no frac against that clock: it was read in a profiled pass, which runs a few % below
        # the un-profiled clock of this line, MI355X_MICROARCH.md)
        dvfs = {"effective_clock_ghz": ghz,
                "sq_valu_active_per_wave": clk["valu_per_wave"],
                "waves_per_simd": clk["waves_per_simd"],
                "source": "stored profiles/r06_effective_clock.json (" + clk["run"] + "): clock = "
                          "GRBM_GUI_ACTIVE / 8 XCDs / dispatch time; SQ_ACTIVE_INST_VALU / "
                          "SQ_WAVE_CYCLES per wave (its product with the waves per SIMD is ~1.0 "
                          "here, but reads 1.3 for the NTT pass at 4 waves: the counter's active "
                          "cycles overlap across waves, so it bounds the VALU busy fraction from above)"}
    return {"bound": "valu", "achieved": achieved, "peak": SIMD_CYCLES_PEAK, "dvfs": dvfs,
            "unit": "SIMD issue-cycles/s", "frac": achieved / SIMD_CYCLES_PEAK,
            "peak_source": "1024 SIMDs x 2.4 GHz (MI355X_MICROARCH.md); per-instruction issue "
                           "costs measured by tools/ubench_issue.hip (profiles/r03_ubench_issue.txt)",
            "valu_cycles_per_wave_of_adds": isa["valu_cycles"],
            "mads_per_point_add": isa["v_mad_u64_u32"],
            "instructions_per_point_add": isa["instructions"],
            "valu_instructions_per_point_add": isa.get("valu_instructions"),
            "s_nop_per_point_add": isa.get("s_nop"), "mads_source": isa["source"],
            "kernel_form": form[1],
            "mad": {"achieved": mads, "peak": VALU_MAD_PEAK, "unit": "mad/s",
                    "frac": mads / VALU_MAD_PEAK, "peak_source": VALU_MAD_PEAK_SOURCE}}


def binding_roofline(valu: dict, hbm_achieved_gbs: float, alg_bytes: float, traffic,
                     kernel: str) -> dict:
    """The roofline object of the bench line: the BINDING (integer-VALU issue) roofline at top
    level (bound / achieved / peak / frac), HBM as the required secondary figure under `hbm`,
    and `traffic` = PMC-measured HBM bytes per launch."""
    return {"bound": "valu", "kernel": kernel, "achieved": valu["achieved"], "peak": valu["peak"],
            "unit": valu["unit"], "frac": valu["frac"], "peak_source": valu["peak_source"],
            "valu_cycles_per_wave_of_adds": valu["valu_cycles_per_wave_of_adds"],
            "mads_per_point_add": valu["mads_per_point_add"],
            "instructions_per_point_add": valu["instructions_per_point_add"],
            "valu_instructions_per_point_add": valu.get("valu_instructions_per_point_add"),
            "s_nop_per_point_add": valu.get("s_nop_per_point_add"),
            "mads_source": valu["mads_source"], "mad": valu["mad"], "dvfs": valu.get("dvfs"),
            "traffic": traffic,
            "hbm": {"achieved": hbm_achieved_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": hbm_achieved_gbs / HBM_PEAK_GBS,
                    "algorithmic_bytes_per_launch": alg_bytes,
                    "note": "secondary roofline: SURVEY §8d algorithmic bytes (128 B per MSM point)"
                            " over the average launch"}}


def load_pmc_traffic(kernel_substr: str, key: str = "hbm_bytes_per_launch",
                     fname: str = "pmc_traffic.json"):
    """HBM bytes per launch of a kernel from the committed rocprofv3 PMC summary
    (profiles/pmc_traffic.json, made by tools/gpu_pmc.sh + tools/pmc_summary.py from the
    default bench command). key "hbm_bytes_last_launch" = the run's last dispatch. A summary
    with a "units" field (tools/recipes.py configs: the transforms or MSMs its run performed)
    gives bytes per unit instead: all launches of the kernel / units."""
    f = ROOT / "profiles" / fname
    if not f.exists():
        return None
    try:
        d = json.loads(f.read_text())
        for name, rec in d.get("kernels", {}).items():
            if kernel_substr in name:
                if "units" in d:
                    return rec["hbm_bytes_per_launch"] * rec["launches"] / d["units"]
                return rec.get(key, rec.get("hbm_bytes_per_launch"))
    except Exception:
        return None
    return None


def max_over_ranks(torch, dist, elapsed: float, device) -> float:
    """The slowest rank's time (all_reduce MAX; a host tensor under gloo)."""
    on = device if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([elapsed], dtype=torch.float64, device=on)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def cpu_threads(args) -> int:
    """CPU baseline threads: --cpu-threads, else OMP_NUM_THREADS (set on the GPU box to the
    CPU share of one GPU), else every core in this process's affinity mask."""
    if args.cpu_threads:
        return args.cpu_threads
    env = os.environ.get("OMP_NUM_THREADS", "")
    if env.isdigit() and int(env) > 0:
        return int(env)
    return host_info()["usable_cores"] or 1


def acc_roofline(ms_total, launches, adds, points, label, form=ACC_LANE):
    """k_accumulate: algorithmic bytes (128 B per MSM point) and mixed additions
    per launch over the average launch duration (dispatch-stamped events)."""
    ms = ms_total / launches
    alg = 128.0 * points / launches
    return {"avg_launch_ms": ms, "launches": launches,
            "algorithmic_bytes_per_launch": alg,
            "achieved_gbs": alg / (ms * 1e-3) / 1e9,
            "point_adds_per_launch": adds / launches,
            "point_adds_per_s": adds / (ms_total * 1e-3),
            "valu": valu_roofline(adds / (ms_total * 1e-3), form), "timing": label}


def msm_shard_point(plk, torch, dist, world, rank, device, pp, k, steps, warmup, threads):
    """One point of the north star's MSM scaling curve per driver run: ONE 2^k MSM
    per step (uniform scalars, the same on every rank, resident in HBM; the bench SRS), split
    over ALL ranks by bucket range (plk_commit_batch_dev_part: rank r sorts, accumulates and
    reduces 1/G of the 2^(c-1) buckets of the whole MSM) with one all-gather of one point per
    rank and the host fold (parallel.gather_fold); at world 1 the lone MSM (the curve's N = 1
    point). Every rank holds the whole SRS (the proof batches' own), so each checks the fold
    against the unsplit commit of the same scalars; world 1 checks against the oracle."""
    from dusk_plonk_amd.parallel import bucket_parts_ok, gather_fold
    n = 1 << k
    gpu = torch.cuda.is_available()  # (False only in the CPU test of this function's logic)
    s = torch.cuda.current_stream().cuda_stream if gpu else 0
    sync = torch.cuda.synchronize if gpu else (lambda: None)
    x = rand_fr_dev(torch, n, 4343, device)
    split = world > 1 and bucket_parts_ok(pp.n, world)
    comm_dev = device if split and dist.get_backend() == "nccl" else None
    coms, part_s = [], []

    def one(timed):
        t0 = time.perf_counter()
        if split:
            part = pp.commit_batch_dev([(x.data_ptr(), n)], s, part=rank, parts=world)
            t1 = time.perf_counter()
            w = np.zeros((1, 13), dtype=np.uint64)
            w[0] = part[0].words
            com = gather_fold(w, [0], None, comm_dev)[0]
        else:
            com = pp.commit_dev(x.data_ptr(), n, s)
            t1 = time.perf_counter()
        if timed:
            coms.append(com)
            part_s.append(t1 - t0)

    for _ in range(warmup):
        one(False)
    sync()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        one(True)
    sync()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        elapsed = max_over_ranks(torch, dist, elapsed, device)
    want = pp.commit_dev(x.data_ptr(), n, s)  # unsplit, on this rank's whole SRS
    ok = all(c == want for c in coms)
    check = "every rank: the fold against its own unsplit commit of the same scalars"
    if world == 1:
        sys.path.insert(0, str(ROOT / "tests"))
        import oracle_lib
        orc = oracle_lib.load()
        ok = ok and np.array_equal(orc.msm(pp.points(0, n), x.cpu().numpy().view(np.uint64), threads),
                                   want.words)
        check = f"against the oracle's Pippenger (oracle/plk_oracle.c, {threads} threads)"
    mine = {"rank": rank, "part_ms": 1e3 * float(np.mean(part_s)), "ok": bool(ok)}
    allr = [mine]
    if world > 1:
        allr = [None] * world
        dist.all_gather_object(allr, mine)
    return {"n": n, "parts": world if split else 1,
            "split": ("bucket range" if split else
                      "none (lone MSM: the curve's N = 1 point)" if world == 1 else
                      f"none ({world} bucket ranges not valid for this SRS)"),
            "transport": transport(dist) if split else None,
            "ms_per_msm": elapsed * 1e3 / steps, "msm_per_s": steps / elapsed, "steps": steps,
            "points_per_s": n * steps / elapsed,
            "per_rank_part_ms": [r["part_ms"] for r in allr],
            "bit_exact": all(r["ok"] for r in allr), "check": check,
            "note": "strong scaling of ONE MSM over the ranks (the north star's 8-GPU MSM curve); "
                    "part_ms = a rank's own part, host-timed launch to readback; ms_per_msm includes "
                    "the all-gather and the fold, max over ranks"}


def run_second_size(args, plk, torch, dist, world, rank, device, k2: int):
    """The metric's second size (BASELINE: 'at n=2^16 and 2^20'): a short prove run at 2^k2
    with the default lanes for that size, proof batches on every rank (key and SRS built
    outside the timed region, fresh witnesses), every lane's last proof re-proved alone and
    byte-compared (proofs_checked)."""
    n2 = 1 << k2
    L = 12 if k2 >= 18 else 14 if k2 >= 15 else 16
    ctx = plk.Context.default(torch.cuda.current_device())
    base = ProverBase(plk, k2, ctx)
    lanes = [ProofLane(base, 1000 * rank + 23 + 101 * l) for l in range(L)]
    import concurrent.futures as cf
    drivers = cf.ThreadPoolExecutor(L)

    def run(count, which=None):
        for f in [drivers.submit(lambda ln: [ln.step() for _ in range(count)], ln)
                  for ln in (which or lanes)]:
            f.result()

    run(max(1, min(args.warmup, 3)))
    torch.cuda.synchronize()
    steps = args.steps
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    run(steps)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        elapsed = max_over_ranks(torch, dist, elapsed, device)
    checked, bad = recheck_proofs(lanes, lanes[0])
    for ln in lanes:
        ln.pool.shutdown(wait=True)
        ln.lane.close()
    drivers.shutdown()
    if bad:
        raise SystemExit(f"bench.py: 2^{k2}: {len(bad)} of {checked} concurrent proofs differ "
                         f"from the same proof made alone (seeds {bad})")
    return {"value": n2 * steps * L * world / elapsed, "unit": "constraints/s", "log_n": k2,
            "ms_per_step": elapsed * 1e3 / steps, "steps": steps, "lanes": L,
            "proofs_per_step": L * world, "proofs_checked": checked - len(bad),
            "hip_hw_queues": int(os.environ.get("GPU_MAX_HW_QUEUES", "4")),
            "note": f"same workload as the headline at n=2^{k2} (m = {base.gates} gates, 1 public "
                    "input), timed after it in the same process; HIP hardware queues as sized "
                    "for the headline's lanes"}


def run_full(args, plk, torch, dist, world, rank, device, k, n, shard):
    # `lanes` concurrent provers per GPU over ONE shared key and SRS (plk_prover: own
    # stream, MSM workspace, scratch), each driven by its own host thread: a proof server
    # keeps several proofs in flight so one proof's host phases and reduction tails overlap
    # another's kernels. One step = every lane completes one proof.
    L = max(1, args.lanes)
    ctx = plk.Context.default(torch.cuda.current_device())
    base = ProverBase(plk, k, ctx)
    # sharded: every rank proves the same proofs (same seeds), commits split by SRS slice
    lane_seed = (lambda l: 17 + 101 * l) if shard else (lambda l: 1000 * rank + 17 + 101 * l)
    lanes = [ProofLane(base, lane_seed(l)) for l in range(L)]
    exchange = None
    split = None
    if shard:
        from dusk_plonk_amd.parallel import (ExchangeService, bucket_parts_ok, shard_prover_lane,
                                             srs_slice)
        comm_dev = device if dist.get_backend() == "nccl" else None
        # the split of every commit: by bucket range where the key's SRS allows it (round 6:
        # each rank sorts, accumulates AND reduces 1/G of the buckets), else by SRS slice
        split = args.shard_split
        if split == "auto":
            split = "buckets" if bucket_parts_ok(base.pp.n, world) else "slices"
        sl = (srs_slice(base.tau, base.pp.n, world, rank, ctx)  # one slice per GPU, all lanes
              if split == "slices" else None)
        # every lane's exchanges on ONE communicator, issued by ONE thread per rank in the
        # order rank 0 sequences (parallel.ExchangeService: no concurrent collectives on
        # different communicators, so no cross-rank ordering deadlock)
        exchange = ExchangeService(None, comm_dev)
        for l, ln in enumerate(lanes):
            shard_prover_lane(ln.lane, base.tau, base.pp.n, None, comm_dev, ctx, slice_=sl,
                              exchange=exchange, lane_id=l, mode=split)
    import concurrent.futures as cf
    drivers = cf.ThreadPoolExecutor(L)

    def run(count, timed, which=None):
        def one(lane):
            for _ in range(count):
                lane.step(timed=timed)
        for f in [drivers.submit(one, ln) for ln in (which or lanes)]:
            f.result()

    tw = time.perf_counter()
    run(args.warmup, False)
    torch.cuda.synchronize()
    # host cores: each lane synthesises one fresh witness per step beside the GPU work. If the
    # node's ranks would need more cores than the node has, prove with fewer lanes per rank
    # rather than oversubscribe (the same count on every rank: the figures are all-reduced)
    warm_step = (time.perf_counter() - tw) / max(1, args.warmup)
    hc = host_core_budget(dist, world, lanes, warm_step)
    # --fit-lanes: prove with fewer lanes (the same count on every rank) when a rank's
    # synthesis would need more than 90 % of its CPU share; by default the lanes stay as
    # requested and the line says whether the host was oversubscribed
    L_run = L
    if args.fit_lanes and args.warmup and hc["oversubscribed"]:
        L_run = max(1, int(L * 0.9 / hc["ratio"]))
    active = lanes[:L_run]
    for ln in lanes:
        ln.lane.msm_stats(reset=True)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    run(args.steps, True, active)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        elapsed = max_over_ranks(torch, dist, elapsed, device)
    steps = args.steps
    lanes_all, lanes, L = lanes, active, L_run
    # k_accumulate inside the workload (all lanes' launches; they share the chip) ...
    acc_ms = launches = adds = points = 0
    for ln in lanes:
        m_, l_, a_, p_ = ln.lane.msm_stats(reset=True)
        acc_ms, launches, adds, points = acc_ms + m_, launches + l_, adds + a_, points + p_
    # ... and with the GPU to itself: one more proof on lane 0 after the timed region. The
    # solo durations are the kernel's own (the in-workload ones overlap other lanes' kernels)
    run(1, False, [lanes[0]])
    torch.cuda.synchronize()
    s_ms, s_l, s_a, s_p = lanes[0].lane.msm_stats(reset=True)
    cbits = base.pp.last_msm_stats()[2]
    # every lane's last timed proof, re-proved alone on lane 0 and compared byte for byte
    # (under --shard-msm every rank re-proves the same seeds in the same order)
    checked, mismatched = recheck_proofs(lanes, lanes[0])
    proofs = L if shard else L * world
    transforms = ("13 transforms (6 idft(n); 6 coset_dft and 1 coset_idft over the 6n quotient "
                  "domain, each as 3 coset blocks of 2n) + 11 MSMs")
    result = {
        "metric": "PLONK prover constraints/sec (BLS12-381) at n=2^16 and 2^20, 1/2/4/8 GPUs",
        "value": n * steps * proofs / elapsed,
        "unit": "constraints/s",
        "n_gpus": world,
        "steps": steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed * 1e3 / steps,
        "higher_is_better": True,
        "scaling": "strong" if shard else "weak",
        "vs_baseline": None,
        "dtype": "u32-limb Montgomery Fr/Fp (integer)",
        "data": "synthetic arithmetic-chain circuit x' = x*y + x + 1 public input, fresh "
                "SplitMix64 witness per proof",
        "config": {
            "workload": f"full Prover::create_proof at n=2^{k} (m = {base.gates} gates, 1 public "
                        f"input): synthesis + 5 rounds + 2 openings = {transforms} per proof "
                        "(the reference's 4 sigma dft(n) and L1's idft(n) + coset_dft(8n) are "
                        "per-key constants here; its 8n quotient coset is a 6n one here, same t "
                        "and proof bytes, DESIGN §3); host synthesis of the next proof overlaps "
                        "the current GPU proof"
                        + (f"; {L} proofs in flight per GPU (plk_prover lanes sharing one key "
                           "and SRS)" if L > 1 else "")
                        + (f"; every commit split over {world} GPU(s) by "
                           + ("bucket range" if split == "buckets" else "SRS slice")
                           + f" ({transport(dist)} all-gather of partial points + host fold), "
                           "NTT / elementwise rounds replicated on every GPU" if shard else ""),
            "n": n, "log_n": k, "proofs_per_step": proofs,
            "parallelism": (f"msm-shard x{world} ({split}) x {L} lane(s), partials all-gathered "
                            f"over {transport(dist)}" if shard else
                            f"proof-batch x{world * L} ({L} concurrent prover lane(s) per GPU)")
                           + (f"; lanes lowered from {len(lanes_all)} to {L} (--fit-lanes: host "
                              "CPU share)" if L < len(lanes_all) else ""),
            "msm_window_bits": cbits,
            "hip_hw_queues": int(os.environ.get("GPU_MAX_HW_QUEUES", "4")),
        },
        "breakdown_ms_per_step": {
            "synthesis_host_overlapped": 1e3 * sum(sum(ln.synth_s) for ln in lanes) / (steps * L),
            "prove_latency": 1e3 * sum(sum(ln.prove_s) for ln in lanes) / (steps * L),
        },
        "proofs_checked": checked - len(mismatched),
        "proofs_check": ("GPU against GPU: each lane's last timed proof re-proved alone on one "
                         "lane after the timed region, byte-identical (catches races between "
                         "concurrent lanes). The oracle check of this configuration (12 lanes "
                         "at 2^20 against the committed C-oracle proof) is the -m gpu test "
                         "tests/test_prover_lanes.py::test_twelve_lanes_2_20_concurrent_byte_exact"),
        "host_cores": {**hc, "lanes_requested": len(lanes_all), "lanes_run": L,
                       "note": "lanes x measured synthesis s / step s (warmup) per rank, against "
                               "that rank's own CPU share (cpu_share); ratio = the largest "
                               "need / share over the ranks; lanes are lowered only with "
                               "--fit-lanes"},
    }
    # roofline of the dominant kernel (k_accumulate, ~60 % of a proof's GPU time) from its
    # solo launches; the in-workload averages beside them
    if s_l and s_ms > 0:
        solo = acc_roofline(s_ms, s_l, s_a, s_p, "one proof with no other lane running, "
                            "dispatch-stamped events (outside the timed region)")
        inw = (acc_roofline(acc_ms, launches, adds, points, "all lanes inside the timed region; "
                            "durations overlap other lanes' kernels (not the kernel's own time)")
               if launches and acc_ms > 0 else None)
        traffic = load_pmc_traffic(ACC_LANE[1])
        traffic2 = load_pmc_traffic(ACC_LANE[1], "hbm_bytes_per_launch_stream_corrected")
        roof = binding_roofline(solo["valu"], solo["achieved_gbs"],
                                solo["algorithmic_bytes_per_launch"], traffic, "k_accumulate")
        roof.update({
            "traffic_fetch_doubled": traffic2,
            "traffic_source": ("stored profile profiles/pmc_traffic.json (rocprofv3 --pmc "
                               "FETCH_SIZE / WRITE_SIZE passes of the default bench command, "
                               "per-launch average over the run); `traffic` = raw FETCH + WRITE, "
                               "`traffic_fetch_doubled` applies the guide's gfx950 x2 for "
                               "16-B/lane streams — this kernel's 96-B random gathers are an "
                               "uncalibrated width, so the two bracket it")
            if traffic is not None else None,
            "avg_launch_ms": solo["avg_launch_ms"], "launches": solo["launches"],
            "point_adds_per_launch": solo["point_adds_per_launch"],
            "point_adds_per_s": solo["point_adds_per_s"],
            "solo": solo, "in_workload": inw,
            "note": "integer-VALU-bound (no MFMA): frac = VALU issue cycles of the solo launches' "
                    "mixed additions (compiled mix x measured costs) over every SIMD issuing every "
                    "cycle at 2.4 GHz; HBM under `hbm` (4 commit batches per proof: 4, 1, 4 and "
                    "2 MSMs)",
        })
        result["roofline"] = roof
    if world > 1 and "roofline" in result:
        # every rank's own k_accumulate figures (its lane 0's solo proof), gathered to the line
        r = result["roofline"]
        mine = {"rank": rank, "frac": r["frac"], "point_adds_per_s": r["point_adds_per_s"],
                "avg_launch_ms": r["avg_launch_ms"], "hbm_gbs": r["hbm"]["achieved"]}
        allr = [None] * world
        dist.all_gather_object(allr, mine)
        r["per_rank"] = allr
        r["note"] += "; per_rank: every rank's own solo figures (top level: rank 0's)"
    for ln in lanes_all:
        ln.pool.shutdown(wait=True)
        ln.lane.close()
    if exchange is not None:
        exchange.close()
    drivers.shutdown()
    if mismatched:
        if rank == 0:
            emit(result)
        raise SystemExit(f"bench.py: {len(mismatched)} of {checked} concurrent proofs differ "
                         f"from the same proof made alone (seeds {mismatched})")
    if not args.no_extras and not shard:
        # after the timed region: the north star's MSM curve point (one 2^k MSM over all ranks)
        # and the metric's second size
        result["msm_shard"] = msm_shard_point(plk, torch, dist, world, rank, device, base.pp, k,
                                              args.steps, max(1, min(args.warmup, 3)),
                                              cpu_threads(args))
        if not result["msm_shard"]["bit_exact"]:
            if rank == 0:
                emit(result)
            raise SystemExit("bench.py: the split MSM differs from the unsplit commit")
        if k != 16:
            result["n_2_16"] = run_second_size(args, plk, torch, dist, world, rank, device, 16)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline_full(
            k, base.pp, cpu_threads(args), gpu_value=result["value"],
            gpu_value_16=(result.get("n_2_16") or {}).get("value") if k != 16 else result["value"])
    elif rank == 0 and world > 1:
        result["cpu_baseline"] = stored_cpu_baseline(k, world, result["value"])
    if rank == 0:
        emit(result)
    if dist.is_initialized():
        dist.destroy_process_group()


BUILD_INFO: dict = {}


def emit(result: dict):
    """Print the line (rank 0), stamped with the library's build provenance (plk_build_info:
    hashes of the sources and flags it was compiled from, checked against this tree)."""
    if BUILD_INFO:
        result["build_id"] = {k: BUILD_INFO.get(k) for k in ("src", "flags", "variant", "tree_src")}
    print(json.dumps(result), flush=True)


def transport(dist) -> str:
    """The process group's transport, as the line reports it."""
    return "RCCL" if dist.get_backend() == "nccl" else "gloo (host memory)"


def run_kernel_mode(args, plk, torch, dist, world, rank, device, k, n):
    """BASELINE.json configs[1] (standalone 2^k BlsScalar NTT/iNTT) and configs[2]
    (standalone 2^k G1 MSM on SRS bases) on one GPU per rank, replicas only (each rank its
    own transform / MSM). Inputs are resident in HBM; one step = dft + idft (ntt) or one
    MSM (msm). After the timed loop the result is checked bit-exact against the oracle
    (tests/oracle_lib.py), whose timing on the same input is the cpu_baseline."""
    s = torch.cuda.current_stream().cuda_stream
    ctx = plk.Context.default(device.index or 0)
    # a split MSM (--shard-msm): every rank holds the same scalars; replicas: their own
    x = rand_fr_dev(torch, n, 4242 if args.shard_msm else 4242 + rank, device)
    ev = []
    if args.mode == "ntt":
        fft = plk.Fft(k, ctx)
        y, z = torch.empty_like(x), torch.empty_like(x)

        def step(timed):
            e = [torch.cuda.Event(enable_timing=True) for _ in range(3)] if timed else None
            if timed:
                e[0].record()
            fft.ntt_dev(x.data_ptr(), y.data_ptr(), n, 1, False, s)
            if timed:
                e[1].record()
            fft.ntt_dev(y.data_ptr(), z.data_ptr(), n, -1, False, s)
            if timed:
                e[2].record()
                ev.append(e)
        units = 2 * n
    else:
        tau = np.asarray(np.random.default_rng(0x5EED).integers(1, 2**62, 4), dtype=np.uint64)
        tau[3] &= np.uint64(0x0FFFFFFFFFFFFFFF)
        coms = []
        part_s = []  # per step: [seconds of each bucket-range part] (--bucket-parts / --shard-msm)
        if args.shard_msm:  # one MSM per step split over the ranks (strong scaling)
            from dusk_plonk_amd.parallel import ShardedPlonkParams
            spp = ShardedPlonkParams(k, tau, ctx=ctx, mode=args.msm_split)
            pp = spp.local
            comm_dev = device if dist.get_backend() == "nccl" else None

            def step(timed):
                from dusk_plonk_amd.parallel import gather_fold
                t0 = time.perf_counter()
                if spp.mode == "buckets":  # this rank's bucket range of the whole MSM
                    part = pp.commit_batch_dev([(x.data_ptr(), n)], s, raise_on_error=False,
                                               part=rank, parts=world)
                else:  # this rank's SRS slice: its span of the scalars against its points
                    off, m = spp._local_spans(n)
                    part = pp.commit_batch_dev([(x.data_ptr() + 32 * off, m)], s,
                                               raise_on_error=False)
                t1 = time.perf_counter()
                if isinstance(part[0], plk.PlonkError):
                    raise part[0]
                w = np.zeros((1, 13), dtype=np.uint64)
                w[0] = part[0].words
                coms.append(gather_fold(w, [0], None, comm_dev)[0])
                if timed:
                    ev.append(pp.last_msm_stats())
                    part_s.append([t1 - t0])
        elif args.bucket_parts > 1:  # the G parts of a bucket-split MSM, one after the other
            from dusk_plonk_amd.parallel import bucket_parts_ok
            P = args.bucket_parts
            pp = plk.PlonkParams.setup(k, tau, ctx)
            if not bucket_parts_ok(pp.n, P):
                raise SystemExit(f"bench.py: --bucket-parts {P} not valid for 2^{k} points")

            def step(timed):
                ts, pts, st = [], [], (0.0, 0, 0)
                for q in range(P):
                    t0 = time.perf_counter()
                    c = pp.commit_batch_dev([(x.data_ptr(), n)], s, part=q, parts=P)[0]
                    ts.append(time.perf_counter() - t0)
                    pts.append(c.words)
                    ms_q, adds_q, cb = pp.last_msm_stats()
                    st = (st[0] + ms_q, st[1] + adds_q, cb)
                coms.append(plk.g1_sum(np.stack(pts)))
                if timed:
                    ev.append(st)
                    part_s.append(ts)
        else:
            pp = plk.PlonkParams.setup(k, tau, ctx)

            def step(timed):
                coms.append(pp.commit_dev(x.data_ptr(), n, s))  # returns the affine point
                if timed:
                    ev.append(pp.last_msm_stats())
        units = n
    for _ in range(args.warmup):
        step(False)
    torch.cuda.synchronize()
    ev.clear()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        elapsed = max_over_ranks(torch, dist, elapsed, device)
    steps = args.steps
    if args.mode == "ntt":
        t_dft = sum(e[0].elapsed_time(e[1]) for e in ev) / steps
        t_idft = sum(e[1].elapsed_time(e[2]) for e in ev) / steps
        launch_ms = (t_dft + t_idft) / 2
        alg_bytes = 64.0 * n  # one read + one write of 32 B per point
        gbs = alg_bytes / (launch_ms * 1e-3) / 1e9
        muls = (n / 2) * k / (launch_ms * 1e-3)
        # binding roofline: the instruction side — the radix-2 butterflies' Fr multiplications
        # (algorithmic count, (N/2) log2 N) against the measured redundant-limb Fr multiply rate
        # (tools/ubench_limbs.hip); HBM (64 B per point) is the secondary figure under `hbm`
        roof = {"bound": "valu", "kernel": "k_ntt_pass (all passes of one transform)",
                "achieved": muls, "peak": FR_MUL_PEAK, "unit": "Fr mul/s", "frac": muls / FR_MUL_PEAK,
                "peak_source": "measured by tools/ubench_limbs.hip (ffr.hpp Fr multiply, whole chip)",
                "ops": "(N/2) log2 N butterfly multiplications per transform",
                "traffic": load_pmc_traffic("k_ntt_pass", fname=f"pmc_traffic_ntt{k}.json"),
                "avg_launch_ms": launch_ms, "dft_ms": t_dft, "idft_ms": t_idft,
                "hbm": {"achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": gbs / HBM_PEAK_GBS,
                        "algorithmic_bytes_per_launch": alg_bytes},
                "note": "per transform (all its Stockham passes; traffic summed over them); "
                        "instruction-bound: the lone transform's passes load, compute and store in "
                        "lockstep, see DESIGN §3"}
        metric = f"standalone BlsScalar dft+idft points/s at n=2^{k} (BASELINE configs[1])"
        workload = f"Fft::dft + Fft::idft of one 2^{k}-point Fr vector, device-resident"
    else:
        launch_ms = sum(e[0] for e in ev) / steps
        adds = sum(e[1] for e in ev) / steps
        alg_bytes = 128.0 * n  # N * (32 B scalar + 96 B base)
        gbs = alg_bytes / (launch_ms * 1e-3) / 1e9
        roof = binding_roofline(valu_roofline(adds / (launch_ms * 1e-3), ACC_LONE), gbs, alg_bytes,
                                load_pmc_traffic(ACC_LONE[1], fname=f"pmc_traffic_msm{k}.json"),
                                "k_accumulate")
        roof.update({"avg_launch_ms": launch_ms, "point_adds_per_launch": adds,
                     "point_adds_per_s": adds / (launch_ms * 1e-3),
                     "note": "integer-VALU-bound (no MFMA); HBM is the secondary roofline"})
        metric = f"standalone G1 MSM points/s at n=2^{k} (BASELINE configs[2])"
        workload = f"KZG10 commit: one 2^{k}-point G1 MSM, random Fr scalars, SRS bases"
        if part_s:
            per = np.asarray(part_s) * 1e3  # [steps, parts] ms
            roof["bucket_parts"] = {
                "parts": per.shape[1] if not args.shard_msm else world,
                "part_ms_mean": [float(v) for v in per.mean(axis=0)],
                "part_ms_max": float(per.mean(axis=0).max()),
                "note": ("each part = plk_commit_batch_dev_part on this GPU: reads every scalar "
                         "and the whole window table, sorts / accumulates / reduces only its "
                         "bucket range; host-timed (launch to readback). Under --shard-msm the "
                         "rank's own part; with --bucket-parts the parts ran one after the other "
                         "on one GPU, each as one of G GPUs would run it")}
            if args.shard_msm:
                workload += (f"; split over {world} GPU(s) by "
                             + ("bucket range" if spp.mode == "buckets" else "SRS slice")
                             + f" ({transport(dist)} all-gather of one point per rank + host fold)")
            else:
                workload += (f"; run as {per.shape[1]} bucket-range parts one after the other on "
                             "one GPU (the per-GPU work of a split over that many GPUs) + host fold")
    if "frac" not in roof:
        roof["frac"] = roof["achieved"] / roof["peak"]
    result = {
        "metric": metric,
        "value": units * steps * (1 if (args.shard_msm and args.mode == "msm") else world) / elapsed,
        "unit": "points/s",
        "n_gpus": world, "steps": steps, "warmup": args.warmup,
        "ms_per_step": elapsed * 1e3 / steps, "higher_is_better": True,
        "scaling": "strong" if (args.shard_msm and args.mode == "msm") else "weak",
        "vs_baseline": None, "dtype": "u32-limb Montgomery Fr/Fp (integer)",
        "data": "synthetic (uniform Fr)",
        "config": {"workload": workload, "n": n, "log_n": k,
                   "parallelism": (f"msm-split x{world} ({args.msm_split})"
                                   if (args.shard_msm and args.mode == "msm") else
                                   f"replicas x{world}")},
        "roofline": roof,
    }
    if args.mode == "msm" and args.shard_msm and world > 1:
        # the folded commitment against an unsplit commit of the same scalars on a whole SRS
        # (buckets: every rank's own; points: one built for the check), on every rank
        full = spp.local if spp.mode == "buckets" else plk.PlonkParams.setup(k, tau, ctx)
        want = full.commit_dev(x.data_ptr(), n, s)
        ok = all(c == want for c in coms)
        on = device if dist.get_backend() == "nccl" else "cpu"
        flag = torch.tensor([1 if ok else 0], dtype=torch.int32, device=on)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        result["bit_exact_vs_unsplit"] = bool(flag.item())
        if not result["bit_exact_vs_unsplit"]:
            if rank == 0:
                emit(result)
            raise SystemExit("bench.py: the split MSM's fold differs from the unsplit commit")
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        threads = cpu_threads(args)
        sys.path.insert(0, str(ROOT / "tests"))
        import oracle_lib
        orc = oracle_lib.load()
        xh = x.cpu().numpy().view(np.uint64)
        if args.mode == "ntt":
            t0 = time.perf_counter()
            want = orc.dft(xh, k, threads)
            t1 = time.perf_counter()
            back = orc.idft(want, k, threads)
            t2 = time.perf_counter()
            exact = (np.array_equal(y.cpu().numpy().view(np.uint64), want)
                     and np.array_equal(z.cpu().numpy().view(np.uint64), back)
                     and np.array_equal(back, xh))
            cpu_s = t2 - t0
            sample = (f"oracle/plk_oracle.c orc_ntt (OpenMP {threads} threads): dft(2^{k}) "
                      f"{t1 - t0:.3f}s + idft(2^{k}) {t2 - t1:.3f}s on the same input")
        else:
            t0 = time.perf_counter()
            want = orc.msm(pp.points(0, n), xh, threads)
            cpu_s = time.perf_counter() - t0
            exact = all(np.array_equal(c.words, want) for c in coms)
            sample = (f"oracle/plk_oracle.c orc_msm (Pippenger, OpenMP {threads} threads): "
                      f"one MSM(2^{k}) on the same SRS and scalars {cpu_s:.2f}s")
        result["bit_exact_vs_oracle"] = bool(exact)
        result["cpu_baseline"] = {"value": units / cpu_s, "unit": "points/s", "cores": threads,
                                  "kind": "port", "host": host_info(), "sample": sample}
        if not exact:
            emit(result)
            raise SystemExit("GPU result differs from the oracle")
    if rank == 0:
        emit(result)
    if dist.is_initialized():
        dist.destroy_process_group()


def launch_ranks(n: int) -> int:
    """`--gpus N` without a launcher: start N ranks of this same command under
    torch.distributed.run (127.0.0.1) as a child process and return its exit code. Called
    before anything touches the GPU (no exec from a GPU-initialised process)."""
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={n}", "--master-addr", "127.0.0.1", f"--master-port={port}",
           str(Path(__file__).resolve()), *sys.argv[1:]]
    return subprocess.run(cmd).returncode


def main():
    args = parse()
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None and args.gpus and args.gpus > 1:
        raise SystemExit(launch_ranks(args.gpus))
    if world_env is not None and args.gpus is not None and args.gpus != int(world_env):
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world_env}")
    if args.lanes <= 0:
        # round-3 sweep (profiles/r03_lanes20_sweep.txt): 2^20 30.2 / 30.3 / 30.7 / 31.4 M at 6 / 8 /
        # 10 / 12 lanes; 2^16 24.0 / 24.6 / 25.1 / 22.0 M at 10 / 12 / 14 / 16; 2^12 5.4 / 5.9
        # M at 12 / 16
        args.lanes = 12 if args.log_n >= 18 else 14 if args.log_n >= 15 else 16
    if args.mode == "prove":
        # before the HIP runtime starts (the torch import below): each lane's stream gets a
        # hardware queue of its own
        q = args.hw_queues or min(32, 2 * args.lanes)
        os.environ["GPU_MAX_HW_QUEUES"] = str(min(32, q))
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 or args.shard_msm:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if world == 1 and "MASTER_PORT" not in os.environ:  # --shard-msm on one GPU, no launcher
            import socket
            with socket.socket() as sk:
                sk.bind(("127.0.0.1", 0))
                os.environ["MASTER_PORT"] = str(sk.getsockname()[1])
        # one rank per GPU; ranks beyond the device count share GPUs (a gloo rehearsal of
        # the multi-rank path on a one-GPU box: RCCL refuses two ranks on one device)
        local %= max(1, torch.cuda.device_count())
        torch.cuda.set_device(local)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local),
                                    rank=rank, world_size=world)
        else:
            dist.init_process_group("gloo", rank=rank, world_size=world)
    else:
        torch.cuda.set_device(0)
    device = torch.device("cuda", torch.cuda.current_device())

    import dusk_plonk_amd as plk

    # the library must come from this tree's sources (fails loudly otherwise); the line
    # carries the ids
    BUILD_INFO.update(plk.check_build())
    k = args.log_n
    n = 1 << k
    # An explicit stream: torch's default stream has handle 0, which the ABI maps to the
    # context's own stream, so events recorded by torch would not bracket our kernels.
    stream = torch.cuda.Stream(device=device)
    torch.cuda.set_stream(stream)
    if args.mode in ("ntt", "msm"):
        return run_kernel_mode(args, plk, torch, dist, world, rank, device, k, n)
    # --shard-msm at world 1 runs the sharded path's whole exchange (communicator, device
    # staging, the exchange thread) with one slice: the configs[4] form on one GPU
    shard = args.shard_msm
    if args.mode == "prove":
        return run_full(args, plk, torch, dist, world, rank, device, k, n, shard)
    hp = HotPath(plk, torch, k, device, seed=1 if shard else 1000 * rank + 1, shard=shard)
    for _ in range(args.warmup):
        hp.step()
    torch.cuda.synchronize()
    hp.ntt_ms = {"n": [], "8n": []}
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        hp.step(timed=True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        elapsed = max_over_ranks(torch, dist, elapsed, device)

    ntt_n = [a.elapsed_time(b) for a, b in hp.ntt_ms["n"]]
    ntt_8n = [a.elapsed_time(b) for a, b in hp.ntt_ms["8n"]]
    acc = hp.msm_acc_ms
    steps = args.steps
    ms_per_step = elapsed * 1e3 / steps
    # per-kernel time shares (HIP events on the launching stream)
    t_ntt_n = sum(ntt_n) / steps
    t_ntt_8n = sum(ntt_8n) / steps
    t_acc = sum(acc) / steps
    # dominant kernel: MSM bucket accumulation vs coset NTT(8n)
    if t_acc >= t_ntt_8n:
        # one k_accumulate launch per commit batch; algorithmic bytes of the MSMs it covers
        launch_ms = sum(acc) / len(acc)
        alg_bytes = 128.0 * n * 11 / len(acc) * steps  # N*(32 B + 96 B) per MSM
        kname = "k_accumulate"
    else:
        launch_ms = sum(ntt_8n) / len(ntt_8n)
        alg_bytes = 2.0 * 8 * n * 32  # one read + one write of the 8n vector
        kname = "k_ntt_pass"
    achieved = alg_bytes / (launch_ms * 1e-3) / 1e9
    traffic = load_pmc_traffic(ACC_LONE[1] if kname == "k_accumulate" else kname)
    result = {
        "metric": "PLONK prover constraints/sec (BLS12-381) at n=2^16 and 2^20, 1/2/4/8 GPUs",
        "value": n * steps * (1 if shard else world) / elapsed,
        "unit": "constraints/s",
        "n_gpus": world,
        "steps": steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "strong" if shard else "weak",
        "vs_baseline": None,
        "dtype": "u32-limb Montgomery Fr/Fp (integer)",
        "data": "synthetic (uniform Fr wires/polys, SRS [tau^i]G1 from a fixed tau)",
        "config": {
            "workload": f"create_proof hot path at n=2^{k}: 7 idft(n) + 4 dft(n) + 7 coset_dft(8n) "
                        f"+ 1 coset_idft(8n) + 11 KZG commits (MSM n, in the reference's 4 independent groups)",
            "n": n, "log_n": k, "hot_path_only": True, "proofs_per_step": 1 if shard else world,
            "parallelism": (f"msm-shard x{world} (SRS slices, {transport(dist)} all-gather of partials)"
                            if shard else f"proof-batch x{world} (one proof per GPU per step)"),
            "msm_window_bits": (hp.pp.local if shard else hp.pp).last_msm_stats()[2],
        },
        "breakdown_ms_per_step": {
            "ntt_n_x11": t_ntt_n, "ntt_8n_x8": t_ntt_8n, "msm_accumulate_4_batches": t_acc,
            "other": ms_per_step - t_ntt_n - t_ntt_8n - t_acc,
        },
    }
    if kname == "k_ntt_pass":  # the binding (Fr-multiply issue) roofline at top level
        k8 = k + 3
        muls = (8 * n / 2) * k8 / (launch_ms * 1e-3)
        result["roofline"] = {
            "bound": "valu", "kernel": "k_ntt_pass (all passes of one 8n coset transform)",
            "achieved": muls, "peak": FR_MUL_PEAK, "unit": "Fr mul/s", "frac": muls / FR_MUL_PEAK,
            "peak_source": "measured by tools/ubench_limbs.hip (ffr.hpp Fr multiply, whole chip)",
            "ops": "(N/2) log2 N butterfly multiplications per transform, N = 8n",
            "traffic": traffic, "avg_launch_ms": launch_ms,
            "hbm": {"achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": achieved / HBM_PEAK_GBS, "algorithmic_bytes_per_launch": alg_bytes},
            "note": "integer-VALU-bound path (no MFMA); HBM is the secondary roofline"}
    if kname == "k_accumulate" and acc:  # the binding (VALU issue) roofline at top level
        adds = sum(hp.msm_adds) / len(hp.msm_adds)
        roof = binding_roofline(valu_roofline(adds / (launch_ms * 1e-3), ACC_LONE), achieved,
                                alg_bytes, traffic, kname)
        roof.update({"avg_launch_ms": launch_ms, "point_adds_per_launch": adds,
                     "point_adds_per_s": adds / (launch_ms * 1e-3),
                     "note": "integer-VALU-bound (no MFMA); HBM is the secondary roofline"})
        result["roofline"] = roof
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(k, hp.pp, cpu_threads(args))
    if rank == 0:
        emit(result)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
