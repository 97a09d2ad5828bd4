"""The Proof wire format: the SCALE encoding the reference derives for
Proof (src/prover/proof.rs:11,36), with the element encodings ASSUMED as documented at
plk_proof_encode (include/plk.h) — parity unpinned: the reference holds no encoded proof.

CPU: plk_proof_encode / plk_proof_decode are host code in libplk.so. The fixture
tests/golden/proof_scale.npz (tests/golden/make_proof_scale.py) freezes one oracle proof and
its SCALE bytes written by an independent struct-level restatement; the library must write
exactly those bytes, decode them back, and reject malformed input.
"""
from pathlib import Path

import numpy as np
import pytest

GOLD = Path(__file__).resolve().parent / "golden" / "proof_scale.npz"


@pytest.fixture(scope="module")
def fixture():
    return dict(np.load(GOLD, allow_pickle=False))


def test_fixture_reproduces(plk, fixture):
    """The oracle still produces the frozen proof, and the restated encoder its bytes."""
    import sys
    sys.path.insert(0, str(GOLD.parent))
    import make_proof_scale
    comms, evals, data = make_proof_scale.make()
    assert np.array_equal(comms, fixture["comms"]) and np.array_equal(evals, fixture["evals"])
    assert data == fixture["scale"].tobytes()


def test_encode_matches_fixture(plk, fixture):
    from dusk_plonk_amd.prover import PROOF_SCALE_BYTES, Proof
    p = Proof.from_words(fixture["comms"], fixture["evals"])
    data = p.to_bytes()
    assert len(data) == PROOF_SCALE_BYTES == 11 * 97 + 16 * 32
    assert data == fixture["scale"].tobytes()


def test_decode_round_trip(plk, fixture):
    from dusk_plonk_amd.prover import Proof
    data = fixture["scale"].tobytes()
    q = Proof.from_bytes(data)
    assert q == Proof.from_words(fixture["comms"], fixture["evals"])
    assert q.to_bytes() == data


def test_identity_commitment_round_trip(plk, fixture):
    from dusk_plonk_amd.prover import Proof
    comms = fixture["comms"].copy()
    comms[4] = 0
    comms[4, 12] = 1  # z_comm = identity (0, 0, true)
    p = Proof.from_words(comms, fixture["evals"])
    data = p.to_bytes()
    assert data[4 * 97 + 96] == 1 and data[4 * 97: 4 * 97 + 96] == bytes(96)
    assert Proof.from_bytes(data) == p


FP = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB


def test_identity_zkcrypto_encoding(plk, fixture):
    """The identity's second known encoding: zkcrypto-style (0, one, true) with one = 2^384
    mod p in Montgomery limbs decodes as the identity, normalised to (0, 0, 1)."""
    from dusk_plonk_amd.prover import Proof
    b = bytearray(fixture["scale"].tobytes())
    off = 4 * 97  # z_comm
    b[off: off + 48] = bytes(48)
    b[off + 48: off + 96] = ((1 << 384) % FP).to_bytes(48, "little")
    b[off + 96] = 1
    q = Proof.from_bytes(bytes(b))
    comms = fixture["comms"].copy()
    comms[4] = 0
    comms[4, 12] = 1
    assert q == Proof.from_words(comms, fixture["evals"])


@pytest.mark.parametrize("case", ["short", "long", "bool", "x_noncanonical", "off_curve",
                                  "identity_noncanonical", "identity_other_coords",
                                  "eval_noncanonical"])
def test_decode_rejects(plk, fixture, case):
    from dusk_plonk_amd.prover import Proof
    b = bytearray(fixture["scale"].tobytes())
    if case == "short":
        b = b[:-1]
    elif case == "long":
        b += b"\0"
    elif case == "bool":
        b[96] = 2
    elif case == "x_noncanonical":
        b[40:48] = (0xFFFFFFFFFFFFFFFF).to_bytes(8, "little")  # top limb of a_comm.x >= p
    elif case == "off_curve":
        b[0] ^= 1
    elif case == "identity_noncanonical":
        b[96] = 1
        b[40:48] = (0xFFFFFFFFFFFFFFFF).to_bytes(8, "little")
    elif case == "identity_other_coords":  # canonical, but neither (0, 0) nor (0, one)
        b[96] = 1
    elif case == "eval_noncanonical":
        off = 11 * 97
        b[off + 24: off + 32] = (0xFFFFFFFFFFFFFFFF).to_bytes(8, "little")
    with pytest.raises(plk.PlonkError) as e:
        Proof.from_bytes(bytes(b))
    assert e.value.status == plk.PLK_E_ARG
