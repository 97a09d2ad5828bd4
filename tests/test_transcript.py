"""The transcript (merlin over STROBE-128/Keccak) pinned to merlin's published test vector
(merlin crate, tests "equivalence_simple"), for the Python restatement used by the test
verifier; the C++ product transcript (csrc/transcript.hpp) is exercised end to end by the
GPU proofs, which the Python verifier only accepts if both transcripts agree byte for
byte."""
from transcript import Transcript


def test_merlin_published_vector():
    t = Transcript(b"test protocol")
    t.append_message(b"some label", b"some data")
    assert t.challenge_bytes(b"challenge", 32).hex() == \
        "d5a21972d0d5fe320c0d263fac7fffb8145aa640af6e9bca177c03c7efcf0615"


def test_long_messages_cross_the_rate():
    t = Transcript(b"rate")
    t.append_message(b"big", bytes(range(256)) * 3)  # > 166-byte STROBE rate
    a = t.challenge_bytes(b"c", 200)
    t2 = Transcript(b"rate")
    t2.append_message(b"big", bytes(range(256)) * 3)
    assert t2.challenge_bytes(b"c", 200) == a and len(a) == 200
