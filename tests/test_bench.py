"""bench.py's output contract (the driver parses one JSON line from rank 0): the CLI on the
CPU, and on the GPU the three single-rank modes at small sizes — prove (default), and the
standalone NTT / MSM lines of BASELINE configs[1] / [2], which check their own result
bit-exact against the oracle before printing."""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
CONTRACT = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
            "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config", "roofline")
ROOFLINE = ("bound", "achieved", "peak", "unit", "frac", "traffic")


def run_bench(*args, timeout=100):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    p = subprocess.run([sys.executable, "bench.py", *args], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    return json.loads(lines[0])


def check_contract(d, steps, warmup, n_gpus=1):
    for k in CONTRACT:
        assert k in d, k
    for k in ROOFLINE:
        assert k in d["roofline"], k
    assert d["value"] > 0 and d["ms_per_step"] > 0
    assert d["n_gpus"] == n_gpus and d["steps"] == steps and d["warmup"] == warmup
    assert d["higher_is_better"] is True and d["vs_baseline"] is None
    assert "workload" in d["config"]
    assert d["roofline"]["frac"] == pytest.approx(d["roofline"]["achieved"] / d["roofline"]["peak"])


def test_cli_lists_modes():
    p = subprocess.run([sys.executable, "bench.py", "--help"], cwd=ROOT, capture_output=True,
                       text=True, timeout=60)
    assert p.returncode == 0
    for flag in ("--gpus", "--steps", "--warmup", "--mode", "--lanes", "--dist-backend"):
        assert flag in p.stdout
    for mode in ("prove", "hotpath", "ntt", "msm"):
        assert mode in p.stdout


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["ntt", "msm"])
def test_kernel_mode_line_is_bit_exact(mode):
    d = run_bench("--mode", mode, "--log-n", "12", "--steps", "3", "--warmup", "1",
                  "--cpu-threads", "4")
    check_contract(d, 3, 1)
    assert d["unit"] == "points/s" and d["config"]["log_n"] == 12
    assert d["bit_exact_vs_oracle"] is True
    cb = d["cpu_baseline"]
    assert cb["kind"] == "port" and cb["cores"] == 4 and cb["value"] > 0
    # both kernels are instruction-bound: the binding (VALU) roofline at top level, HBM beside
    assert d["roofline"]["bound"] == "valu" and d["roofline"]["hbm"]["unit"] == "GB/s"


@pytest.mark.gpu
def test_prove_mode_line():
    d = run_bench("--log-n", "12", "--steps", "2", "--warmup", "1", "--lanes", "2",
                  "--no-cpu-baseline", "--no-extras")
    check_contract(d, 2, 1)
    assert d["unit"] == "constraints/s" and d["scaling"] == "weak"
    # value counts every lane's proof: n * steps * lanes / time
    assert d["value"] == pytest.approx(4096 * 2 * 2 / (d["ms_per_step"] * 2e-3), rel=1e-6)


def test_compiled_loop_mads():
    """bench.py's mads per mixed addition come from the compiled k_accumulate loop in
    libplk.so (tools/isa_count.py), not from the formula constant."""
    sys.path.insert(0, str(ROOT))
    import bench
    for form in (bench.ACC_LANE, bench.ACC_LONE):  # both k_accumulate instantiations
        isa = bench.compiled_loop(form[0])
        assert "compiled" in isa["source"], (form, isa)
        assert 3000 < isa["v_mad_u64_u32"] < isa["instructions"] < 6000
        assert isa["v_mad_u64_u32"] * 4 < isa["valu_cycles"] < isa["instructions"] * 5
    # the lane form's interleaved product groups: fewer VALU instructions than the plain chains
    lane, lone = bench.compiled_loop(bench.ACC_LANE[0]), bench.compiled_loop(bench.ACC_LONE[0])
    assert lane["v_mad_u64_u32"] == lone["v_mad_u64_u32"]
    assert lane["valu_instructions"] < lone["valu_instructions"]


def test_valu_roofline_carries_stored_clock():
    """The VALU roofline of each k_accumulate form carries the stored DVFS reading
    (profiles/r06_effective_clock.json: effective clock from GRBM_GUI_ACTIVE, the SQ VALU
    activity per wave): the top-level frac is priced at the nominal 2.4 GHz."""
    sys.path.insert(0, str(ROOT))
    import bench
    for form in (bench.ACC_LANE, bench.ACC_LONE):
        r = bench.valu_roofline(7.0e9, form)
        d = r["dvfs"]
        assert d is not None, form
        assert 1.0 < d["effective_clock_ghz"] < 2.5
        assert 0.2 < d["sq_valu_active_per_wave"] < 1.0 and d["waves_per_simd"] in (2, 3)
        assert "r06_effective_clock.json" in d["source"]


def test_gpus_flag_must_match_launcher():
    """Under a launcher (WORLD_SIZE set) --gpus must agree with it: no silent n_gpus: 1."""
    env = dict(os.environ, WORLD_SIZE="3", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--steps", "1"], cwd=ROOT,
                       env=env, capture_output=True, text=True, timeout=60)
    assert p.returncode != 0 and "WORLD_SIZE=3" in (p.stderr + p.stdout)


@pytest.mark.gpu
def test_prove_mode_line_has_solo_roofline():
    d = run_bench("--log-n", "12", "--steps", "2", "--warmup", "1", "--lanes", "2",
                  "--no-cpu-baseline", "--no-extras")
    r = d["roofline"]
    assert r["kernel"] == "k_accumulate" and r["solo"]["launches"] == 4  # one proof
    assert r["avg_launch_ms"] == r["solo"]["avg_launch_ms"]
    assert r["in_workload"]["launches"] == 2 * 2 * 4
    # the binding roofline at top level, HBM as the secondary figure
    assert r["bound"] == "valu" and r["hbm"]["unit"] == "GB/s" and r["mad"]["unit"] == "mad/s"
    assert r["mads_per_point_add"] > 3000 and "compiled" in r["mads_source"]
    assert "13 transforms" in d["config"]["workload"] and "1 public input" in d["config"]["workload"]


@pytest.mark.gpu
def test_gpus_2_shard_msm_launches_ranks_itself():
    """`bench.py --gpus 2 --shard-msm` without a launcher starts two ranks (here sharing the
    box's one GPU over gloo) and prints ONE full-proof line with n_gpus 2 (configs[4] form)."""
    d = run_bench("--gpus", "2", "--shard-msm", "--dist-backend", "gloo", "--log-n", "12",
                  "--steps", "2", "--warmup", "1", "--lanes", "2", "--no-cpu-baseline",
                  timeout=300)
    check_contract(d, 2, 1, n_gpus=2)
    assert d["scaling"] == "strong" and d["config"]["proofs_per_step"] == 2
    assert d["config"]["parallelism"].startswith("msm-shard x2 (slices)")  # c = 10: no bucket split
    # all ranks prove the same proofs: value counts each once
    assert d["value"] == pytest.approx(4096 * 2 * 2 / (d["ms_per_step"] * 2e-3), rel=1e-6)


@pytest.mark.gpu
def test_prove_mode_checks_its_proofs():
    """The prove line re-proves every lane's last timed proof alone and compares bytes."""
    d = run_bench("--log-n", "12", "--steps", "2", "--warmup", "1", "--lanes", "3",
                  "--no-cpu-baseline", "--no-extras")
    assert d["proofs_checked"] == 3
    hc = d["host_cores"]
    assert hc["lanes_run"] == 3 and hc["needed_per_rank"] > 0 and hc["available_per_rank"] >= 1
    assert "oversubscribed" in hc and len(hc["per_host"]) == 1


@pytest.mark.gpu
def test_shard_msm_world1_over_rccl():
    """`bench.py --shard-msm` at world 1 under nccl: the configs[4] form with its whole RCCL
    exchange on the one GPU (no launcher), one line, transport named."""
    d = run_bench("--shard-msm", "--log-n", "12", "--steps", "2", "--warmup", "1", "--lanes",
                  "2", "--no-cpu-baseline", timeout=200)
    check_contract(d, 2, 1)
    assert d["scaling"] == "strong" and "RCCL" in d["config"]["parallelism"]
    assert d["proofs_checked"] == 2


class _Lane:
    def __init__(self, synth):
        self.synth_all = synth


def _budget_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, str(ROOT))
    import torch.distributed as dist
    import bench

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # rank 0: 12 lanes x 0.05 s synthesis per 0.4 s step = 1.5 cores of a 16-core share;
        # rank 1: 12 x 0.5 / 0.4 = 15 cores of a 16-core share (oversubscribed at > 90 %)
        share = {"available": 16}
        lanes = [_Lane([0.05 if rank == 0 else 0.5])] * 12
        hc = bench.host_core_budget(dist, world, lanes, 0.4, share=share)
        ok = abs(hc["needed_per_rank"] - (1.5 if rank == 0 else 15.0)) < 1e-9
        ok &= hc["available_per_rank"] == 16
        ok &= abs(hc["ratio"] - 15.0 / 16) < 1e-9 and hc["oversubscribed"]
        host = next(iter(hc["per_host"].values()))
        ok &= host["ranks"] == 2 and abs(host["need"] - 16.5) < 1e-9 and host["available"] == 32
        # a node of 8 GPUs at ~2.5 cores each against 16-core shares: not oversubscribed
        # (round 4 compared the node's sum with ONE share and would have cut lanes to ~8)
        hc2 = bench.host_core_budget(dist, world, [_Lane([0.083])] * 12, 0.4, share=share)
        ok &= not hc2["oversubscribed"]
        q.put((rank, bool(ok)))
    finally:
        dist.destroy_process_group()


def test_host_core_budget_per_rank_share_gloo_world2():
    """each rank's synthesis need is compared with its own CPU share (the GPU box
    gives every GPU one), not the node's summed need with one share."""
    import socket
    import torch.multiprocessing as mp
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_budget_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
    out = dict(q.get(timeout=5) for _ in range(2))
    assert out == {0: True, 1: True}
    for p in procs:
        assert p.exitcode == 0


@pytest.mark.gpu
def test_prove_line_world2_self_describing():
    """A multi-rank prove line (2 ranks sharing the card over gloo) carries every rank's
    roofline and the stored CPU baseline (bench.py stored_cpu_baseline), labelled as stored."""
    d = run_bench("--gpus", "2", "--dist-backend", "gloo", "--log-n", "12", "--steps", "2",
                  "--warmup", "1", "--lanes", "2", "--no-cpu-baseline", "--no-extras", timeout=300)
    check_contract(d, 2, 1, n_gpus=2)
    cb = d["cpu_baseline"]
    assert cb["source"].startswith("stored") and cb["value"] > 0 and cb["cores"] == 32
    pr = d["roofline"]["per_rank"]
    assert [r["rank"] for r in pr] == [0, 1] and all(r["frac"] > 0 for r in pr)
    assert d["host_cores"]["lanes_run"] == 2


@pytest.mark.gpu
def test_msm_bucket_parts_line_is_bit_exact():
    """`--mode msm --bucket-parts 4`: the 2^16 MSM run as 4 bucket-range parts on one GPU (what
    each of 4 GPUs runs under --shard-msm), folded, checked against the oracle; per-part times."""
    d = run_bench("--mode", "msm", "--log-n", "16", "--steps", "2", "--warmup", "1",
                  "--bucket-parts", "4", "--cpu-threads", "4")
    check_contract(d, 2, 1)
    assert d["bit_exact_vs_oracle"] is True
    bp = d["roofline"]["bucket_parts"]
    assert bp["parts"] == 4 and len(bp["part_ms_mean"]) == 4 and bp["part_ms_max"] > 0


@pytest.mark.gpu
def test_msm_split_over_ranks_lines():
    """`--mode msm --shard-msm`: ONE MSM per step split over the ranks by bucket range — at
    world 1 over RCCL (checked against the oracle) and on 2 gloo ranks sharing the card."""
    d = run_bench("--mode", "msm", "--shard-msm", "--log-n", "16", "--steps", "2", "--warmup",
                  "1", "--cpu-threads", "4")
    assert d["bit_exact_vs_oracle"] is True and d["scaling"] == "strong"
    assert d["config"]["parallelism"] == "msm-split x1 (buckets)"
    d2 = run_bench("--gpus", "2", "--mode", "msm", "--shard-msm", "--dist-backend", "gloo",
                   "--log-n", "16", "--steps", "2", "--warmup", "1", timeout=300)
    assert d2["n_gpus"] == 2 and d2["scaling"] == "strong"
    assert d2["config"]["parallelism"] == "msm-split x2 (buckets)"
    assert d2["roofline"]["bucket_parts"]["parts"] == 2
    # one MSM per step whatever the world: value = n * steps / time
    assert d2["value"] == pytest.approx(65536 * 2 / (d2["ms_per_step"] * 2e-3), rel=1e-6)
    assert d2["bit_exact_vs_unsplit"] is True  # the fold against an unsplit commit, every rank


@pytest.mark.gpu
def test_msm_split_points_over_ranks_line():
    """`--msm-split points` on 2 gloo ranks (round-5 advisor: each rank commits ITS span of the
    scalars against its SRS slice, not the whole vector), checked against an unsplit commit."""
    d = run_bench("--gpus", "2", "--mode", "msm", "--shard-msm", "--msm-split", "points",
                  "--dist-backend", "gloo", "--log-n", "16", "--steps", "2", "--warmup", "1",
                  timeout=300)
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "msm-split x2 (points)"
    assert "SRS slice" in d["config"]["workload"] and d["bit_exact_vs_unsplit"] is True


class _FakeSplitParams:
    """CPU stand-in for the bench SRS in msm_shard_point: commit_batch_dev(part=, parts=)
    returns the bucket-range share of the restated split (oracle/pyref.py msm_bucket_part,
    c = 20), commit_dev the double-and-add MSM; scalars are read from the host pointer."""

    def __init__(self, points):
        self.points, self.n, self.parts_seen = points, len(points), []

    @staticmethod
    def _scalars(ptr, length):
        import ctypes
        import numpy as np
        import pyref as P
        a = np.ctypeslib.as_array((ctypes.c_uint64 * (4 * length)).from_address(ptr))
        return P.fr_vec_from_np(a.reshape(length, 4).copy())

    def commit_batch_dev(self, ptrs_lens, stream=0, raise_on_error=True, part=0, parts=1):
        import pyref as P
        import dusk_plonk_amd as plk
        self.parts_seen.append((part, parts))
        (ptr, length), = ptrs_lens
        share = P.msm_bucket_part(self.points[:length], self._scalars(ptr, length), 20, part, parts)
        return [plk.Commitment(P.g1_vec_to_np([share])[0])]

    def commit_dev(self, ptr, length, stream=0):
        import pyref as P
        import dusk_plonk_amd as plk
        return plk.Commitment(P.g1_vec_to_np([P.msm_naive(self.points[:length],
                                                          self._scalars(ptr, length))])[0])


def _msm_shard_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), PLK_MSM_C="20")
    sys.path[:0] = [str(ROOT), str(ROOT / "tests"), str(ROOT / "oracle")]
    import numpy as np
    import torch
    import torch.distributed as dist
    import bench
    import pyref as P

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g = dict(np.load(ROOT / "tests" / "golden" / "msm_golden.npz", allow_pickle=False))
        pp = _FakeSplitParams(P.g1_vec_from_np(g["srs"]))
        r = bench.msm_shard_point(None, torch, dist, world, rank, "cpu", pp, 6, 2, 1, 1)
        ok = r["parts"] == world and r["split"] == "bucket range" and r["bit_exact"] is True
        ok &= len(r["per_rank_part_ms"]) == world and r["ms_per_msm"] > 0
        ok &= r["points_per_s"] > 0 and set(pp.parts_seen) == {(rank, world)}
        q.put((rank, bool(ok)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_msm_shard_point_gloo(world):
    """The msm_shard field of the default multi-rank line (the north star's MSM curve): ONE
    MSM per step split over 2 / 4 gloo ranks by bucket range, shares all-gathered and folded,
    the fold checked against the unsplit commit on every rank (CPU: the split restated by
    pyref)."""
    import socket
    import torch.multiprocessing as mp
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_msm_shard_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
    out = dict(q.get(timeout=5) for _ in range(world))
    assert out == {r: True for r in range(world)}
    for p in procs:
        assert p.exitcode == 0


@pytest.mark.gpu
def test_prove_line_extras_world1():
    """The default line's extras at world 1: msm_shard = the lone 2^k MSM (the curve's N = 1
    point) checked against the oracle; n_2_16 = the metric's second size, proofs re-checked;
    build_id = the library's source hash, equal to the tree's."""
    d = run_bench("--log-n", "14", "--steps", "2", "--warmup", "1", "--lanes", "2",
                  "--no-cpu-baseline", timeout=300)
    m = d["msm_shard"]
    assert m["parts"] == 1 and m["bit_exact"] is True and "oracle" in m["check"]
    assert m["ms_per_msm"] > 0 and m["n"] == 1 << 14
    s = d["n_2_16"]
    assert s["log_n"] == 16 and s["value"] > 0 and s["proofs_checked"] == s["lanes"] == 14
    assert d["build_id"]["src"] == d["build_id"]["tree_src"]


@pytest.mark.gpu
def test_prove_line_msm_curve_world2():
    """At world 2 (two gloo ranks sharing the card) the line's msm_shard is ONE 2^16 MSM split
    by bucket range over both ranks, folded and checked against the unsplit commit."""
    d = run_bench("--gpus", "2", "--dist-backend", "gloo", "--log-n", "16", "--steps", "2",
                  "--warmup", "1", "--lanes", "2", "--no-cpu-baseline", timeout=400)
    m = d["msm_shard"]
    assert m["parts"] == 2 and m["split"] == "bucket range" and m["bit_exact"] is True
    assert len(m["per_rank_part_ms"]) == 2 and "n_2_16" not in d


@pytest.mark.gpu
def test_gpus_2_shard_msm_bucket_split():
    """configs[4] with the bucket-range split (plk_prover_shard_buckets): 2^16 (c = 17, 2 parts
    of 2^15 buckets), two gloo ranks sharing the card, every lane's proof re-checked alone."""
    d = run_bench("--gpus", "2", "--shard-msm", "--dist-backend", "gloo", "--log-n", "16",
                  "--steps", "2", "--warmup", "1", "--lanes", "2", "--no-cpu-baseline",
                  timeout=400)
    check_contract(d, 2, 1, n_gpus=2)
    assert d["config"]["parallelism"].startswith("msm-shard x2 (buckets)")
    assert "bucket range" in d["config"]["workload"] and d["proofs_checked"] == 2
