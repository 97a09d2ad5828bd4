"""Full-proof parity: the C restatement of PlonkKey::compile + Prover::create_proof
(oracle/plk_prover_oracle.c) against the restated verifier (CPU, this file's first half)
and against the GPU prover byte for byte (second half, `gpu`).

The reference holds no proof vector (transcript and proof bytes are unpinned),
so the chain of evidence is: merlin's published vector pins both transcripts
(tests/test_transcript.py); oracle proofs are accepted by tests/verifier.py (a restatement
of proof.rs / verifier.rs / commitment_scheme.rs) and tampering is rejected; the GPU proof
equals the oracle proof on the same circuit, SRS, label and blinding seed.
"""
from pathlib import Path

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


def decomposition(a, n, flip=None):
    """tests/decomposition.rs DummyCircuit<N>: witness bits asserted equal to
    component_decomposition(a); `flip` corrupts one bit (the negative case)."""
    def f(cs):
        w_a = cs.append_witness(a)
        bits = [(a >> i) & 1 for i in range(n)]
        if flip is not None:
            bits[flip] ^= 1
        w_bits = [cs.append_witness(b) for b in bits]
        for w, b in zip(w_bits, cs.component_decomposition(w_a, n)):
            cs.assert_equal(w, b)
    return f


def selects(bit, a, b):
    """component_select / _one / _zero outputs pinned with assert_equal_constant."""
    def f(cs):
        wb, wa, wv = cs.append_witness(bit), cs.append_witness(a), cs.append_witness(b)
        cs.component_boolean(wb)
        s = cs.component_select(wb, wa, wv)
        cs.assert_equal_constant(s, a if bit else b)
        s1 = cs.component_select_one(wb, wa)
        cs.assert_equal_constant(s1, a if bit else 1)
        s0 = cs.component_select_zero(wb, wa)
        cs.assert_equal_constant(s0, a if bit else 0)
    return f

def logic(a, b, bits, xor, wrong=False):
    """tests/logic.rs DummyCircuit: append_logic_and / _xor of the low `bits` bits, asserted
    equal to the expected value (`wrong` asserts a different value: the negative case)."""
    def f(cs):
        mask = (1 << bits) - 1
        aa, bb = a & mask, b & mask
        c = (aa ^ bb) if xor else (aa & bb)
        c >>= bits & 1  # odd counts: 2-bit quads cover the top bits - 1 bits (lib.rs:291)
        if wrong:
            c ^= 1
        wa, wb, wc = cs.append_witness(aa), cs.append_witness(bb), cs.append_witness(c)
        wx = cs.append_logic_xor(wa, wb, bits) if xor else cs.append_logic_and(wa, wb, bits)
        cs.assert_equal(wc, wx)
    return f


def readme_circuit(a, b, c, d, e, f=None):
    """README.md:28-70 TestCircuit: a + b = c (public), a < 2^6, b < 2^5, a * b = d
    (public), e * G = f (public point) via component_mul_generator."""
    def fn(cs):
        from dusk_plonk_amd.prover import (JUBJUB_GENERATOR, Constraint, jubjub_mul)
        ff = f if f is not None else jubjub_mul(JUBJUB_GENERATOR, e)
        wa, wb = cs.append_witness(a), cs.append_witness(b)
        cs.append_gate(Constraint().left(1).right(1).public(-c).a(wa).b(wb))
        cs.component_range(wa, 1 << 6)
        cs.component_range(wb, 1 << 5)
        cs.append_gate(Constraint().mult(1).public(-d).a(wa).b(wb))
        we = cs.append_witness(e)
        p = cs.component_mul_generator(we, JUBJUB_GENERATOR)
        cs.assert_equal_public_point(p, ff)
    return fn


def mul_generator(a, wrong=False):
    """tests/ecc.rs:20-60: component_mul_generator(a) == append_point(a G)."""
    def fn(cs):
        from dusk_plonk_amd.prover import JUBJUB_GENERATOR, jubjub_mul
        b = jubjub_mul(JUBJUB_GENERATOR, a + (1 if wrong else 0))
        wa, wb = cs.append_witness(a), cs.append_point(b)
        cs.assert_equal_point(cs.component_mul_generator(wa, JUBJUB_GENERATOR), wb)
    return fn


def add_point(a, b, wrong=False):
    """tests/ecc.rs:111-160: component_add_point(aG, bG) == (a + b) G."""
    def fn(cs):
        from dusk_plonk_amd.prover import JUBJUB_GENERATOR, jubjub_mul
        pa, pb = jubjub_mul(JUBJUB_GENERATOR, a), jubjub_mul(JUBJUB_GENERATOR, b)
        pc = jubjub_mul(JUBJUB_GENERATOR, a + b + (1 if wrong else 0))
        wa, wb, wc = cs.append_point(pa), cs.append_point(pb), cs.append_point(pc)
        cs.assert_equal_point(cs.component_add_point(wa, wb), wc)
    return fn


def mul_point(a, b):
    """tests/ecc.rs:236-285: component_mul_point(a, bG) == (a b) G (variable base)."""
    def fn(cs):
        from dusk_plonk_amd.prover import JUBJUB_GENERATOR, jubjub_mul
        pb = jubjub_mul(JUBJUB_GENERATOR, b)
        pc = jubjub_mul(pb, a)
        wa, wb, wc = cs.append_witness(a), cs.append_point(pb), cs.append_point(pc)
        cs.assert_equal_point(cs.component_mul_point(wa, wb), wc)
    return fn


JJ_A = 0x0A5B3C2D1E0F9A8B7C6D5E4F3A2B1C0D9E8F7A6B5C4D3E2F1A0B9C8D7E6F5A4
JJ_B = 0x03F2E1D0C9B8A7968574635241302F1E0D1C2B3A49586776A5B4C3D2E1F0A1B

A_RND = 0x3A5F0E29B8C1D47265E0F1A2B3C4D5E6F708192A3B4C5D6E7F8091A2B3C4D5E6
B_RND = 0x2F1E3D4C5B6A79881726354453627180A9B8C7D6E5F40312233445566778899A

CASES = [
    ("test_circuit_default", readme_circuit(0, 0, 0, 0, 0, f=(0, 1)), 61),
    ("test_circuit_20_5", readme_circuit(20, 5, 25, 100, 2), 62),
    ("mul_generator", mul_generator(JJ_A), 63),
    ("add_point", add_point(JJ_A, JJ_B), 64),
    ("mul_point", mul_point(JJ_A, JJ_B), 65),
    ("and_254", logic(A_RND, B_RND, 254, False), 51),
    ("and_30", logic(A_RND, B_RND, 30, False), 52),
    ("and_0", logic(A_RND, B_RND, 0, False), 53),
    ("and_55", logic(A_RND, B_RND, 55, False), 54),
    ("xor_254", logic(A_RND, B_RND, 254, True), 55),
    ("xor_30", logic(A_RND, B_RND, 30, True), 56),
    ("decomposition_256", decomposition(0x1234567890ABCDEF1122334455667788 * 7919, 256), 41),
    ("select_1", selects(1, 77, 99), 42),
    ("select_0", selects(0, 77, 99), 43),
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
                                ranged(2**76, 76),
                                decomposition(0x1234567890ABCDEF * 31337, 256, flip=10),
                                logic(A_RND, B_RND, 254, False, wrong=True),
                                logic(A_RND, B_RND, 64, True, wrong=True),
                                mul_generator(JJ_A, wrong=True), add_point(JJ_A, JJ_B, wrong=True),
                                readme_circuit(20, 5, 26, 100, 2)],
                         ids=["boolean2", "range_neg", "range_2^76", "decomposition_flip",
                              "and_wrong", "xor_wrong", "mul_generator_wrong", "add_point_wrong",
                              "test_circuit_wrong_c"])
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
    raw = np.frombuffer(proof.raw_bytes(), dtype=np.uint64)
    evals = raw[11 * 13:].reshape(16, 4)
    assert np.array_equal(evals, ref["evals"]), "evaluations differ"
    from dusk_plonk_amd.prover import fr_int
    assert pis == [fr_int(p) for p in ref["pis"]]


def bench_chain(chain_gates, seed):
    """bench.py's circuit (bench_circuit): Plonk::initialize + chain + one public input."""
    def f(cs):
        cs.synthetic_chain(chain_gates, seed)
        cs.append_public((seed * 0x9E3779B97F4A7C15 + 12345) % (1 << 250))
    return f


@pytest.mark.gpu
def test_gpu_proof_equals_oracle_bench_2_16(plk, oracle):
    """BASELINE configs[3] at its full size: the bench circuit at n = 2^16 (m = n - 8 gates,
    one public input, so the PI idft / coset_dft run), GPU proof byte for byte against the
    restated CPU prover on the same SRS, label and blinding seed."""
    import os
    from dusk_plonk_amd.prover import PlonkKey, fr_int
    k = 16
    tau_limbs, _ = tau_for(0x5EED)
    cs = build(bench_chain((1 << k) - 15, 77))
    gates, wit = cs.export()
    assert gates.shape[0] == (1 << k) - 8
    pp = plk.PlonkParams.setup(k, tau_limbs)
    srs = pp.points(0, n_trim(gates.shape[0]))
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    ref = oracle.prove(gates, wit, srs, b"bench", 7, threads)
    prover, vd = PlonkKey.compile_composer(pp, b"bench", cs)
    assert np.array_equal(vd.comms, ref["vk"])
    proof, pis = prover.prove_composer(cs, 7)
    raw = np.frombuffer(proof.raw_bytes(), dtype=np.uint64)
    assert np.array_equal(raw[: 11 * 13].reshape(11, 13), ref["comms"])
    assert np.array_equal(raw[11 * 13:].reshape(16, 4), ref["evals"])
    assert len(pis) == 1 and pis == [fr_int(p) for p in ref["pis"]]


@pytest.mark.gpu
@pytest.mark.parametrize("k", [13, 14])
def test_gpu_proof_equals_oracle_bench_small(plk, oracle, k):
    """The bench circuit at the sizes whose commits take c = 12 / 13 (srs.hip choose_c,
    round 5: balanced windows on the narrow bucket path, k_hist + k_sort_small + k_scatter),
    GPU proof byte for byte against the restated CPU prover."""
    import os
    from dusk_plonk_amd.prover import PlonkKey
    tau_limbs, _ = tau_for(0x5EED + k)
    cs = build(bench_chain((1 << k) - 15, 78))
    gates, wit = cs.export()
    assert gates.shape[0] == (1 << k) - 8
    pp = plk.PlonkParams.setup(k, tau_limbs)
    srs = pp.points(0, n_trim(gates.shape[0]))
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    ref = oracle.prove(gates, wit, srs, b"bench", 11, threads)
    prover, vd = PlonkKey.compile_composer(pp, b"bench", cs)
    assert np.array_equal(vd.comms, ref["vk"])
    proof, _ = prover.prove_composer(cs, 11)
    raw = np.frombuffer(proof.raw_bytes(), dtype=np.uint64)
    assert np.array_equal(raw[: 11 * 13].reshape(11, 13), ref["comms"])
    assert np.array_equal(raw[11 * 13:].reshape(16, 4), ref["evals"])


GOLD_2_20 = Path(__file__).resolve().parent / "golden" / "proof_2_20.npz"


def test_fixture_2_20_shape():
    """The committed 2^20 headline fixture (tests/golden/make_proof_2_20.py: the restated CPU
    prover on bench.py's circuit) is a complete proof: VK, 11 commitments, 16 evaluations,
    one public input, and SCALE bytes that are the restated encoding of those words."""
    import sys
    sys.path.insert(0, str(GOLD_2_20.parent))
    from make_proof_scale import scale_bytes
    g = dict(np.load(GOLD_2_20, allow_pickle=False))
    assert g["vk"].shape == (15, 13) and g["comms"].shape == (11, 13)
    assert g["evals"].shape == (16, 4) and g["pis"].shape == (1, 4)
    assert list(g["meta"]) == [20, 77, 7, 0x5EED]
    assert scale_bytes(g["comms"], g["evals"]) == g["scale"].tobytes()
    assert not any(int(c[12]) for c in g["comms"])  # no identity commitments


@pytest.mark.gpu
def test_gpu_proof_equals_oracle_fixture_2_20(plk):
    """BASELINE's headline workload (n = 2^20, the bench circuit) pinned byte for byte: the
    GPU proof equals the restated CPU prover's (committed fixture, /root/reference/src/
    prover.rs:67-474 order) — verifier key, commitments, evaluations, public input and the
    SCALE bytes of the Proof."""
    import sys
    sys.path.insert(0, str(GOLD_2_20.parent))
    from make_proof_2_20 import BLIND_SEED, LABEL, LOG_N, TAU_SEED, circuit
    from dusk_plonk_amd.prover import PlonkKey, fr_int
    g = dict(np.load(GOLD_2_20, allow_pickle=False))
    tau_limbs, _ = tau_for(TAU_SEED)
    cs = circuit()
    pp = plk.PlonkParams.setup(LOG_N, tau_limbs)
    prover, vd = PlonkKey.compile_composer(pp, LABEL, cs)
    assert np.array_equal(vd.comms, g["vk"]), "verifier key commitments differ"
    proof, pis = prover.prove_composer(cs, BLIND_SEED)
    raw = np.frombuffer(proof.raw_bytes(), dtype=np.uint64)
    assert np.array_equal(raw[: 11 * 13].reshape(11, 13), g["comms"])
    assert np.array_equal(raw[11 * 13:].reshape(16, 4), g["evals"])
    assert pis == [fr_int(p) for p in g["pis"]]
    assert proof.to_bytes() == g["scale"].tobytes()
