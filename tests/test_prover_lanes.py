"""Prover lanes (plk_prover): several proofs in flight over ONE key and SRS, each lane with
its own stream, MSM workspace and scratch — the reference's `Prover: Clone` +
`create_proof(&self)` run concurrently. Also the key/circuit structure check
(a circuit that does not match the key is refused with PLK_E_ARG) and the SCALE round trip
of a real GPU proof."""
import concurrent.futures as cf

import numpy as np
import pytest

from oracle_lib import random_fr
from verifier import verify

pytestmark = pytest.mark.gpu


def chain_pi(cs, gates, seed):
    cs.synthetic_chain(gates, seed)
    cs.append_public((seed * 0x9E3779B97F4A7C15 + 12345) % (1 << 250))


def setup_key(plk, logn, seed=5):
    from dusk_plonk_amd.prover import Plonk, PlonkKey, fr_int
    tau = random_fr(1, seed=seed)[0]
    pp = plk.PlonkParams.setup(logn, tau)
    gates = (1 << logn) - 15
    cs = Plonk()
    chain_pi(cs, gates, 1)
    prover, vd = PlonkKey.compile_composer(pp, b"lanes", cs)
    return fr_int(tau), pp, prover, vd, gates


def fresh(gates, seed):
    from dusk_plonk_amd.prover import Plonk
    cs = Plonk()
    chain_pi(cs, gates, seed)
    return cs


def test_lanes_share_key_and_match_plk_prove(plk):
    tau, pp, prover, vd, gates = setup_key(plk, 12)
    seeds = [11, 12, 13, 14, 15, 16]
    want = {s: prover.prove_composer(fresh(gates, s + 100), s)[0].raw_bytes() for s in seeds}
    lanes = [prover.lane() for _ in range(3)]
    assert len({ln.stream for ln in lanes}) == 3

    def run(i):
        out = {}
        for s in seeds[i::3]:
            p, pi = lanes[i].prove_composer(fresh(gates, s + 100), s)
            out[s] = (p, pi)
        return out

    got = {}
    with cf.ThreadPoolExecutor(3) as ex:  # three lanes proving at the same time
        for d in ex.map(run, range(3)):
            got.update(d)
    for s in seeds:
        p, pi = got[s]
        assert p.raw_bytes() == want[s], s
    verify(vd, got[11][0], got[11][1], tau)
    ms, launches, adds, points = lanes[0].msm_stats()
    assert launches == 2 * 4 and adds > 0 and points > 0  # 4 commit batches per proof
    for ln in lanes:
        ln.close()


def test_structure_mismatch_is_refused(plk):
    """the key's wire gather indices stand for the proving circuit's wires, so a
    circuit with another structure (same gate count) or too few witnesses is refused."""
    from dusk_plonk_amd.prover import Constraint, Plonk
    _, pp, prover, vd, gates = setup_key(plk, 10)
    other = Plonk()  # same gate count, different wiring (no copy chain)
    for i in range(gates):
        w = other.append_witness(i + 3)
        other.append_gate(Constraint().left(1).a(w).constant(-(i + 3)))
    other.append_public(5)
    assert other.m() == prover.m
    with pytest.raises(plk.PlonkError) as e:
        prover.prove_composer(other, 1)
    assert e.value.status == plk.PLK_E_ARG
    # a circuit whose public input is at another gate: different structure as well
    moved = Plonk()
    moved.append_public((1 * 0x9E3779B97F4A7C15 + 12345) % (1 << 250))
    moved.synthetic_chain(gates, 1)
    assert moved.m() == prover.m
    with pytest.raises(plk.PlonkError) as e:
        prover.prove_composer(moved, 1)
    assert e.value.status == plk.PLK_E_ARG
    # the same structure with other witness values proves
    p, pi = prover.prove_composer(fresh(gates, 77), 1)
    assert len(pi) == 1


def test_gpu_proof_scale_round_trip(plk):
    from dusk_plonk_amd.prover import PROOF_SCALE_BYTES, Proof
    tau, pp, prover, vd, gates = setup_key(plk, 9)
    p, pi = prover.prove_composer(fresh(gates, 5), 3)
    data = p.to_bytes()
    assert len(data) == PROOF_SCALE_BYTES
    q = Proof.from_bytes(data)
    assert q == p
    verify(vd, q, pi, tau)


def test_twelve_lanes_2_20_concurrent_byte_exact(plk):
    """The credited bench configuration byte-checked: ONE key at n = 2^20 (the fixture's
    circuit and tau) and 12 prover lanes proving concurrently on the wide-bucket MSM path
    (c = 20), 2 proofs each. Lane 0's first proof is the fixture's (circuit, blinding seed 7)
    and must equal tests/golden/proof_2_20.npz (the restated CPU prover's bytes); every other
    proof must equal the same (circuit, seed) proved afterwards on one lane alone. A race in
    the shared window table, the per-lane workspaces or the readback generation stamps would
    show here (reference: `Prover: Clone`, concurrent create_proof(&self), prover.rs:67-474)."""
    import sys
    from pathlib import Path
    gold = Path(__file__).resolve().parent / "golden"
    sys.path.insert(0, str(gold))
    from make_proof_2_20 import BLIND_SEED, LABEL, LOG_N, TAU_SEED, circuit
    from dusk_plonk_amd.prover import PlonkKey
    from test_prover_oracle import bench_chain, build, tau_for
    g = dict(np.load(gold / "proof_2_20.npz", allow_pickle=False))
    tau_limbs, _ = tau_for(TAU_SEED)
    pp = plk.PlonkParams.setup(LOG_N, tau_limbs)
    prover, vd = PlonkKey.compile_composer(pp, LABEL, circuit())
    assert np.array_equal(vd.comms, g["vk"])
    L, per = 12, 2
    lanes = [prover.lane() for _ in range(L)]
    chain = (1 << LOG_N) - 15
    jobs = {i: [(200 + i * per + j, 300 + i * per + j) for j in range(per)] for i in range(L)}
    jobs[0][0] = (None, BLIND_SEED)  # the fixture's circuit (chain seed 77) and blinding

    def circ(cseed):
        return circuit() if cseed is None else build(bench_chain(chain, cseed))

    def run(i):
        out = {}
        for cseed, bseed in jobs[i]:
            cs = circ(cseed)
            out[(cseed, bseed)] = lanes[i].prove_composer(cs, bseed)[0]
        return out

    got = {}
    with cf.ThreadPoolExecutor(L) as ex:  # twelve lanes proving at the same time
        for d in ex.map(run, range(L)):
            got.update(d)
    assert len(got) == L * per
    assert got[(None, BLIND_SEED)].to_bytes() == g["scale"].tobytes()
    alone = lanes[1]
    for (cseed, bseed), p in got.items():
        if cseed is None:
            continue
        want = alone.prove_composer(circ(cseed), bseed)[0]
        assert p.raw_bytes() == want.raw_bytes(), (cseed, bseed)
    for ln in lanes:
        ln.close()
