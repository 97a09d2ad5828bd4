"""End-to-end PLONK proofs on the GPU (PlonkKey::compile + Prover::create_proof through the
C ABI), accepted by the restated verifier (tests/verifier.py), and the reference's
negative path: an unsatisfied circuit fails in create_proof at the quotient commit
(PLK_E_DEGREE), as tests/boolean.rs:88-90, tests/range.rs:82-84, tests/ecc.rs:91-93
expect_err. Circuits restate the reference's integration tests where the gadget is
supported (boolean.rs: component_boolean; public inputs; arithmetic gates).
"""
import numpy as np
import pytest

from oracle_lib import random_fr
from verifier import VerificationError, verify

pytestmark = pytest.mark.gpu


def tau_and_params(plk, k, seed):
    from dusk_plonk_amd.prover import fr_int
    tau = random_fr(1, seed=seed)[0]
    return fr_int(tau), plk.PlonkParams.setup(k, tau)


class Boolean:
    """tests/boolean.rs:27-55 DummyCircuit: component_boolean(a)."""

    def __init__(self, a):
        self.a = a

    def synthesize(self, cs):
        w = cs.append_witness(self.a)
        cs.component_boolean(w)


class PublicSum:
    """a + b = c with c public (gate_add + assert_equal_constant with a public input)."""

    def __init__(self, a, b, c):
        self.a, self.b, self.c = a, b, c

    def synthesize(self, cs):
        from dusk_plonk_amd.prover import Constraint
        wa, wb = cs.append_witness(self.a), cs.append_witness(self.b)
        wc = cs.gate_add(Constraint().left(1).right(1).a(wa).b(wb))
        cs.assert_equal_constant(wc, 0, -self.c)


class Chain:
    def __init__(self, gates, seed):
        self.gates, self.seed = gates, seed

    def synthesize(self, cs):
        cs.synthetic_chain(self.gates, self.seed)


class Ranged:
    """tests/range.rs:27-55 DummyCircuit: component_range(a, bits)."""

    def __init__(self, a, bits):
        self.a, self.bits = a, bits

    def synthesize(self, cs):
        cs.component_range(cs.append_witness(self.a), self.bits)


def test_range_works(plk):
    """tests/range.rs:14-99: compile with the default circuit (7, 76 bits), prove u64::MAX,
    reject -2^77, and compile with 77 bits."""
    from dusk_plonk_amd.prover import PlonkKey
    r = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
    tau, pp = tau_and_params(plk, 6, 8349)
    prover, vd = PlonkKey.compile_with_circuit(pp, b"demo", Ranged(7, 76))
    proof, pi = prover.create_proof(1, Ranged(2**64 - 1, 76))
    verify(vd, proof, pi, tau)
    with pytest.raises(plk.PlonkError) as e:
        prover.create_proof(2, Ranged((r - 2**77) % r, 76))
    assert e.value.status == plk.PLK_E_DEGREE
    PlonkKey.compile_with_circuit(pp, b"demo", Ranged(1, 77))


def test_boolean_works(plk):
    from dusk_plonk_amd.prover import PlonkKey
    tau, pp = tau_and_params(plk, 4, 8349)
    prover, vd = PlonkKey.compile_with_circuit(pp, b"plonk", Boolean(1))
    assert vd.n == 8 and vd.m == 7
    for a, seed in ((1, 11), (0, 12)):
        proof, pi = prover.create_proof(seed, Boolean(a))
        verify(vd, proof, pi, tau)
    with pytest.raises(plk.PlonkError) as e:
        prover.create_proof(13, Boolean(2))
    assert e.value.status == plk.PLK_E_DEGREE


def test_public_inputs_and_tamper(plk):
    from dusk_plonk_amd.prover import PlonkKey
    tau, pp = tau_and_params(plk, 5, 7)
    prover, vd = PlonkKey.compile_with_circuit(pp, b"sum", PublicSum(2, 3, 5))
    proof, pi = prover.create_proof(1, PublicSum(10, 20, 30))
    assert len(pi) == 1
    verify(vd, proof, pi, tau)
    with pytest.raises(VerificationError):  # wrong public input
        verify(vd, proof, [(pi[0] + 1) % (2**255)], tau)
    proof.a_eval = (proof.a_eval + 1) % 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
    with pytest.raises(VerificationError):  # tampered evaluation
        verify(vd, proof, pi, tau)
    with pytest.raises(plk.PlonkError):  # unsatisfied: 10 + 20 != 31
        prover.create_proof(2, PublicSum(10, 20, 31))


def test_proofs_are_deterministic_per_seed(plk):
    from dusk_plonk_amd.prover import PlonkKey
    _, pp = tau_and_params(plk, 6, 3)
    prover, _ = PlonkKey.compile_with_circuit(pp, b"chain", Chain(40, 5))
    p1, _ = prover.create_proof(99, Chain(40, 5))
    p2, _ = prover.create_proof(99, Chain(40, 5))
    p3, _ = prover.create_proof(100, Chain(40, 5))
    assert p1.raw_bytes() == p2.raw_bytes()
    assert p1.raw_bytes() != p3.raw_bytes()


@pytest.mark.parametrize("logn", [6, 10, 12, 16, 20])
def test_chain_circuit_proves_and_verifies(plk, logn):
    """Including the benchmark's own sizes (2^16 and 2^20: c = 13 / 16 windows, pruned
    first NTT passes, multi-lane bucket sums): a fresh-witness proof the verifier accepts."""
    from dusk_plonk_amd.prover import PlonkKey
    tau, pp = tau_and_params(plk, logn, logn)
    gates = (1 << logn) - 8 - 6
    prover, vd = PlonkKey.compile_with_circuit(pp, b"chain", Chain(gates, 1))
    assert vd.n == 1 << logn
    proof, pi = prover.create_proof(7, Chain(gates, 2))  # another witness, same structure
    verify(vd, proof, pi, tau)
