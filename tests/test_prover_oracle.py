"""Full-proof parity: the C restatement of PlonkKey::compile + Prover::create_proof
(oracle/plk_prover_oracle.c) against the restated verifier (CPU, this file's first half)
and against the GPU prover byte for byte (second half, `gpu`).

The reference holds no proof vector (transcript and proof bytes are unpinned),
so the chain of evidence is: merlin's published vector pins both transcripts
(tests/test_transcript.py); oracle proofs are accepted by tests/verifier.py (a restatement
of proof.rs / verifier.rs / commitment_scheme.rs) and tampering is rejected; the GPU proof
equals the oracle proof on the same circuit, SRS, label and blinding seed.
"""
import numpy as np
import pytest

from oracle_lib import random_fr
from verifier import VerificationError, verify

COMMS = ["a_comm", "b_comm", "c_comm", "d_comm", "z_comm", "t_low_comm", "t_mid_comm",
         "t_high_comm", "t_4_comm", "w_z_chall_comm", "w_z_chall_w_comm"]
EVALS = ["a_eval", "b_eval", "c_eval", "d_eval", "a_next_eval", "b_next_eval", "d_next_eval",
         "q_arith_eval", "q_c_eval", "q_l_eval", "q_r_eval", "s_sigma_1_eval",
         "s_sigma_2_eval", "s_sigma_3_eval", "r_poly_eval", "perm_eval"]


class OracleProof:
    def __init__(self, res):
        from dusk_plonk_amd.prover import fr_int
        for i, c in enumerate(COMMS):
            setattr(self, c, res["comms"][i])
        for i, e in enumerate(EVALS):
            setattr(self, e, fr_int(res["evals"][i]))


def tau_for(seed):
    from dusk_plonk_amd.prover import fr_int
    t = random_fr(1, seed=seed)[0]
    return t, fr_int(t)


def n_trim(m):
    k = max(0, (m + 6 - 1).bit_length())
    return (1 << k) + 8


def build(circuit_fn):
    from dusk_plonk_amd.prover import Plonk
    cs = Plonk()
    circuit_fn(cs)
    return cs


def boolean(a):
    def f(cs):
        cs.component_boolean(cs.append_witness(a))
    return f


def public_sum(a, b, c):
    def f(cs):
        from dusk_plonk_amd.prover import Constraint
        wa, wb = cs.append_witness(a), cs.append_witness(b)
        wc = cs.gate_add(Constraint().left(1).right(1).a(wa).b(wb))
        cs.assert_equal_constant(wc, 0, -c)
    return f


def chain(gates, seed):
    def f(cs):
        cs.synthetic_chain(gates, seed)
    return f


def public_and_chain(gates, seed, pub):
    def f(cs):
        w = cs.append_public(pub)
        cs.synthetic_chain(gates, seed)
        from dusk_plonk_amd.prover import Constraint
        cs.gate_add(Constraint().left(1).right(1).a(w).b(w))
    return f


def ranged(a, bits):
    """tests/range.rs DummyCircuit: component_range(append_witness(a), bits)."""
    def f(cs):
        cs.component_range(cs.append_witness(a), bits)
    return f


R_MOD = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001

CASES = [
    ("range_u64max_76", ranged(2**64 - 1, 76), 31),
    ("range_7_76", ranged(7, 76), 32),
    ("range_odd_77", ranged(1, 77), 33),
    ("range_full_254", ranged(2**250 + 12345, 254), 34),
    ("boolean1", boolean(1), 11),
    ("boolean0", boolean(0), 12),
    ("public_sum", public_sum(10, 20, 30), 5),
    ("chain_2^6", chain((1 << 6) - 14, 3), 7),
    ("chain_2^9", chain((1 << 9) - 14, 4), 8),
    ("public_chain", public_and_chain(300, 9, 1234567), 21),
]


def oracle_prove(oracle, cs, label, seed, tau_limbs):
    gates, wit = cs.export()
    srs = oracle.srs(tau_limbs, n_trim(gates.shape[0]))
    return oracle.prove(gates, wit, srs, label, seed)


def vd_for(res, cs, label):
    from dusk_plonk_amd.prover import VerifierData
    gates, _ = cs.export()
    m = gates.shape[0]
    n = 1 << max(0, (m - 1).bit_length())
    _, idx = cs.public_inputs()
    return VerifierData(label, n, m, res["vk"], idx)


@pytest.mark.parametrize("name,fn,seed", CASES, ids=[c[0] for c in CASES])
def test_oracle_proof_verifies(plk, oracle, name, fn, seed):
    from dusk_plonk_amd.prover import fr_int
    tau_limbs, tau = tau_for(seed + 100)
    cs = build(fn)
    res = oracle_prove(oracle, cs, b"oracle", seed, tau_limbs)
    proof = OracleProof(res)
    pis = [fr_int(p) for p in res["pis"]]
    vd = vd_for(res, cs, b"oracle")
    verify(vd, proof, pis, tau)
    proof.b_eval = (proof.b_eval + 1) % (2**255)
    with pytest.raises(VerificationError):
        verify(vd, proof, pis, tau)


@pytest.mark.parametrize("fn", [boolean(2), ranged((R_MOD - 2**77) % R_MOD, 76),
                                ranged(2**76, 76)], ids=["boolean2", "range_neg", "range_2^76"])
def test_oracle_rejects_unsatisfied(plk, oracle, fn):
    tau_limbs, _ = tau_for(1)
    cs = build(fn)
    with pytest.raises(RuntimeError, match="status 2"):  # ORC_E_DEGREE at the t commit
        oracle_prove(oracle, cs, b"oracle", 1, tau_limbs)


@pytest.mark.gpu
@pytest.mark.parametrize("name,fn,seed", CASES, ids=[c[0] for c in CASES])
def test_gpu_proof_equals_oracle(plk, oracle, name, fn, seed):
    from dusk_plonk_amd.prover import PlonkKey
    tau_limbs, _ = tau_for(seed + 100)
    cs = build(fn)
    gates, _ = cs.export()
    k = max(0, (n_trim(gates.shape[0]) - 8 - 1).bit_length())
    pp = plk.PlonkParams.setup(k, tau_limbs)
    srs = pp.points(0, n_trim(gates.shape[0]))
    gates, wit = cs.export()
    ref = oracle.prove(gates, wit, srs, b"parity", seed)
    prover, vd = PlonkKey.compile_composer(pp, b"parity", cs)
    assert np.array_equal(vd.comms, ref["vk"]), "verifier key commitments differ"
    proof, pis = prover.prove_composer(cs, seed)
    for i, c in enumerate(COMMS):
        assert np.array_equal(getattr(proof, c), ref["comms"][i]), c
    raw = np.frombuffer(proof.to_bytes(), dtype=np.uint64)
    evals = raw[11 * 13:].reshape(16, 4)
    assert np.array_equal(evals, ref["evals"]), "evaluations differ"
    from dusk_plonk_amd.prover import fr_int
    assert pis == [fr_int(p) for p in ref["pis"]]
