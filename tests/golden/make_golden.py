"""Generate the golden fixtures in tests/golden/*.npz from oracle/pyref.py (pure Python
big ints — an independent restatement of the math, not the GPU or C code).

Run:  python tests/golden/make_golden.py
Inputs come from SplitMix64 (seed 8349 = tests/boolean.rs:21 of the reference; tau from
seed 0x5EED). All Fr arrays are Montgomery-form uint64[n,4] (the ABI
layout), G1 arrays uint64[n,13].

Pinning: the reference holds no numeric NTT/MSM vector (its
poly-commit / zksnarks crates are not vendored); these fixtures pin the restatement to
the definitions (naive O(n^2) DFT at k <= 6, naive double-and-add MSM) and to the
reference's in-tree constants (lib.rs:583-588, permutation.rs:28-30), which the tests
check separately.
"""
from __future__ import annotations

import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parent.parent / "oracle"))
import pyref as P  # noqa: E402


def ntt_fixtures():
    rng = P.SplitMix64(8349)
    out = {}
    for k in (0, 1, 2, 3, 4, 5, 6, 8, 10):
        n = 1 << k
        x = [rng.fr() for _ in range(n)]
        part = [rng.fr() for _ in range(max(1, n // 2 + 1))][: n]  # zero-padded input
        dft = P.dft(x, k)
        if k <= 6:
            assert dft == P.dft_naive(x, k)
            assert P.idft(x, k) == P.dft_naive(x, k, inverse=True)
        out[f"k{k}_in"] = P.fr_vec_to_np(x)
        out[f"k{k}_part"] = P.fr_vec_to_np(part)
        out[f"k{k}_dft"] = P.fr_vec_to_np(dft)
        out[f"k{k}_idft"] = P.fr_vec_to_np(P.idft(x, k))
        out[f"k{k}_coset_dft"] = P.fr_vec_to_np(P.coset_dft(x, k))
        out[f"k{k}_coset_idft"] = P.fr_vec_to_np(P.coset_idft(x, k))
        out[f"k{k}_part_dft"] = P.fr_vec_to_np(P.dft(part, k))
        out[f"k{k}_part_coset_dft"] = P.fr_vec_to_np(P.coset_dft(part, k))
        out[f"k{k}_elements"] = P.fr_vec_to_np([pow(P.omega(k), i, P.R_MOD) for i in range(n)])
    # vanishing polynomial over the 8n coset for n = 2^2 (key.rs:291)
    out["vanish_k5_n4"] = P.fr_vec_to_np(P.vanishing_poly_over_coset(5, 4))
    np.savez_compressed(HERE / "ntt_golden.npz", **out)


def msm_fixtures():
    rng = P.SplitMix64(0x5EED)
    tau = rng.fr()
    n = 64
    srs = P.srs_setup(tau, n)
    rng = P.SplitMix64(8349)
    cases = {
        "random": [rng.fr() for _ in range(n)],
        "zeros": [0] * n,
        "ones": [1] * n,
        "minus_one": [P.R_MOD - 1] * n,
        "sparse": [(rng.fr() if i % 7 == 0 else 0) for i in range(n)],
        "small": [i * i for i in range(n)],
        "high_bits": [P.R_MOD - 1 - i for i in range(n)],
    }
    out = {"tau": P.fr_vec_to_np([tau])[0], "srs": P.g1_vec_to_np(srs)}
    for name, sc in cases.items():
        res = P.msm_naive(srs, sc)
        out[f"{name}_scalars"] = P.fr_vec_to_np(sc)
        out[f"{name}_result"] = P.g1_vec_to_np([res])[0]
    # prefix lengths of the random case (commit over an SRS prefix)
    for m in (1, 2, 3, 17, 33):
        out[f"random_prefix{m}_result"] = P.g1_vec_to_np([P.msm_naive(srs[:m], cases['random'][:m])])[0]
    np.savez_compressed(HERE / "msm_golden.npz", **out)


if __name__ == "__main__":
    ntt_fixtures()
    msm_fixtures()
    print("wrote", sorted(p.name for p in HERE.glob("*.npz")))
