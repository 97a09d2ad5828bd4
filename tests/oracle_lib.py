"""ctypes binding of the C oracle (oracle/plk_oracle.c, oracle/plk_prover_oracle.c) — test
infrastructure only."""
from __future__ import annotations

import ctypes as C
import subprocess
from pathlib import Path

import numpy as np

ORACLE_DIR = Path(__file__).resolve().parent.parent / "oracle"
LIB = ORACLE_DIR / "build" / "liboracle.so"


class Oracle:
    def __init__(self, lib):
        self.lib = lib
        vp, u32, u64, sz, i32 = C.c_void_p, C.c_uint32, C.c_uint64, C.c_size_t, C.c_int
        sig = {
            "orc_fr_mul": (None, [vp, vp, vp]), "orc_fr_add": (None, [vp, vp, vp]),
            "orc_fr_sub": (None, [vp, vp, vp]), "orc_fr_inv": (None, [vp, vp]),
            "orc_fp_mul": (None, [vp, vp, vp]), "orc_fr_omega": (None, [u32, vp]),
            "orc_elements": (None, [u32, vp, i32]), "orc_ntt": (i32, [vp, u32, i32, i32, i32]),
            "orc_vanishing": (None, [u32, u64, vp]), "orc_msm": (i32, [vp, vp, sz, vp, i32]),
            "orc_g1_mul": (None, [vp, vp, vp]), "orc_srs": (None, [vp, sz, vp, i32]),
            "orc_merlin_test": (None, [vp]),
            "orc_prove": (i32, [vp, sz, vp, sz, vp, sz, C.c_char_p, u64, i32, vp, vp, vp, vp,
                                vp, sz, C.POINTER(sz), vp]),
        }
        for name, (res, args) in sig.items():
            f = getattr(lib, name)
            f.restype, f.argtypes = res, args

    @staticmethod
    def _p(a):
        return a.ctypes.data_as(C.c_void_p)

    def ntt(self, vals: np.ndarray, k: int, direction: int, coset: bool, threads: int = 0):
        n = 1 << k
        buf = np.zeros((n, 4), dtype=np.uint64)
        v = np.asarray(vals, dtype=np.uint64).reshape(-1, 4)
        buf[: v.shape[0]] = v
        assert self.lib.orc_ntt(self._p(buf), k, direction, int(coset), threads) == 0
        return buf

    def dft(self, v, k, threads=0):
        return self.ntt(v, k, 1, False, threads)

    def idft(self, v, k, threads=0):
        return self.ntt(v, k, -1, False, threads)

    def coset_dft(self, v, k, threads=0):
        return self.ntt(v, k, 1, True, threads)

    def coset_idft(self, v, k, threads=0):
        return self.ntt(v, k, -1, True, threads)

    def elements(self, k, threads=0):
        out = np.zeros((1 << k, 4), dtype=np.uint64)
        self.lib.orc_elements(k, self._p(out), threads)
        return out

    def vanishing(self, k, deg):
        out = np.zeros((1 << k, 4), dtype=np.uint64)
        self.lib.orc_vanishing(k, deg, self._p(out))
        return out

    def msm(self, points, scalars, threads=0):
        pts = np.ascontiguousarray(np.asarray(points, dtype=np.uint64).reshape(-1, 13))
        sc = np.ascontiguousarray(np.asarray(scalars, dtype=np.uint64).reshape(-1, 4))
        assert pts.shape[0] >= sc.shape[0]
        out = np.zeros(13, dtype=np.uint64)
        assert self.lib.orc_msm(self._p(pts), self._p(sc), sc.shape[0], self._p(out), threads) == 0
        return out

    def srs(self, tau, n, threads=0):
        t = np.ascontiguousarray(np.asarray(tau, dtype=np.uint64).reshape(4))
        out = np.zeros((n, 13), dtype=np.uint64)
        self.lib.orc_srs(self._p(t), n, self._p(out), threads)
        return out

    def merlin_test(self) -> bytes:
        out = (C.c_uint8 * 32)()
        self.lib.orc_merlin_test(out)
        return bytes(out)

    def prove(self, gates: np.ndarray, witness: np.ndarray, srs: np.ndarray, label: bytes,
              seed: int, threads: int = 0, vk_in=None):
        """orc_prove: restated PlonkKey::compile + create_proof. gates: (m, 51) u64 words in
        plk_constraint layout; witness (nw, 4); srs (N, 13). Returns dict with vk (15, 13),
        comms (11, 13), evals (16, 4), pis (k, 4), timing_ns (8,)."""
        g = np.ascontiguousarray(gates, dtype=np.uint64)
        w = np.ascontiguousarray(witness, dtype=np.uint64).reshape(-1, 4)
        pts = np.ascontiguousarray(srs, dtype=np.uint64).reshape(-1, 13)
        vk = np.zeros((15, 13), dtype=np.uint64)
        comms = np.zeros((11, 13), dtype=np.uint64)
        evals = np.zeros((16, 4), dtype=np.uint64)
        pis = np.zeros((max(1, g.shape[0]), 4), dtype=np.uint64)
        npi = C.c_size_t()
        timing = np.zeros(8, dtype=np.uint64)
        vin = None
        if vk_in is not None:
            vin = np.ascontiguousarray(vk_in, dtype=np.uint64).reshape(15, 13)
        st = self.lib.orc_prove(self._p(g), g.shape[0], self._p(w), w.shape[0], self._p(pts),
                                pts.shape[0], label, seed, threads,
                                None if vin is None else self._p(vin), self._p(vk),
                                self._p(comms), self._p(evals), self._p(pis), pis.shape[0],
                                C.byref(npi), self._p(timing))
        if st != 0:
            raise RuntimeError(f"orc_prove status {st}")
        return {"vk": vk, "comms": comms, "evals": evals, "pis": pis[: npi.value],
                "timing_ns": timing}

    def fr_mul(self, a, b):
        a = np.ascontiguousarray(a, dtype=np.uint64)
        b = np.ascontiguousarray(b, dtype=np.uint64)
        r = np.zeros(4, dtype=np.uint64)
        self.lib.orc_fr_mul(self._p(a), self._p(b), self._p(r))
        return r


def load() -> Oracle:
    srcs = [ORACLE_DIR / "plk_oracle.c", ORACLE_DIR / "plk_prover_oracle.c"]
    if not LIB.exists() or any(LIB.stat().st_mtime < s.stat().st_mtime for s in srcs):
        subprocess.run(["make", "-C", str(ORACLE_DIR)], check=True, capture_output=True)
    return Oracle(C.CDLL(str(LIB)))


def random_fr(n: int, seed: int) -> np.ndarray:
    """Uniform Montgomery-form Fr vector (vectorised SplitMix64-free sampler for big n).

    Any uniform canonical value is a uniform Montgomery value, so we sample canonical
    255-bit words with rejection and store them directly as Montgomery limbs.
    """
    import sys
    sys.path.insert(0, str(ORACLE_DIR))
    import pyref
    rng = np.random.Generator(np.random.PCG64(seed))
    out = np.empty((n, 4), dtype=np.uint64)
    r_limbs = np.array(pyref.int_to_limbs(pyref.R_MOD, 4), dtype=np.uint64)
    filled = 0
    while filled < n:
        m = (n - filled) * 2 + 16
        cand = rng.integers(0, 2**64, size=(m, 4), dtype=np.uint64, endpoint=False)
        cand[:, 3] &= np.uint64((1 << 63) - 1)
        # lexicographic compare with r (most significant limb first)
        lt = np.zeros(m, dtype=bool)
        eq = np.ones(m, dtype=bool)
        for i in (3, 2, 1, 0):
            lt |= eq & (cand[:, i] < r_limbs[i])
            eq &= cand[:, i] == r_limbs[i]
        good = cand[lt]
        take = min(good.shape[0], n - filled)
        out[filled:filled + take] = good[:take]
        filled += take
    return out
