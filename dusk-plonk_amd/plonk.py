"""Host-side mirror of the reference's hot-path interface, over the C ABI (include/plk.h).

The reference exposes the path through Rust structs of un-vendored crates:
``poly_commit::Fft`` (new / dft / idft / coset_dft / coset_idft / size / size_inv /
generator / generator_inv / elements / compute_vanishing_poly_over_coset),
``Coefficients`` / ``PointsValue`` (``pub Vec<F>`` newtypes), and
``zksnarks::plonk::PlonkParams`` (setup / trim / commit). This module keeps those names,
argument meanings and error behaviour:

* NTT calls are infallible for valid lengths and take their input "by value" (a new
  array is returned, the argument is not modified), as the Rust API moves its ``Vec``.
* ``PlonkParams.commit`` raises :class:`PlonkError` with ``status == PLK_E_DEGREE`` when
  the polynomial (trailing zeros ignored) is longer than the trimmed SRS — the only way
  the reference's ``create_proof`` fails on an unsatisfied circuit (prover.rs:262-265).

Field elements are ``numpy.uint64`` arrays of shape ``[n, 4]`` holding Montgomery-form
limbs (R = 2^256, exactly the reference's in-memory ``BlsScalar``); G1 points are
``[n, 13]`` (Montgomery Fp x, y, infinity flag). There is no CPU fallback: without the
HIP library or a GPU every call raises.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

import numpy as np

_PKG = Path(__file__).resolve().parent
# PLK_LIB: an alternative build of the same library (tools/ A/B experiments)
_LIB_PATH = Path(os.environ["PLK_LIB"]) if os.environ.get("PLK_LIB") else _PKG / "libplk.so"

PLK_OK, PLK_E_DEGREE, PLK_E_ARG, PLK_E_DEVICE, PLK_E_OOM, PLK_E_NODEV = range(6)

# Symbols declared in include/plk.h (checked by tests/test_abi.py)
ABI_SYMBOLS = (
    "plk_abi_version", "plk_status_str", "plk_build_info", "plk_device_count", "plk_ctx_create",
    "plk_ctx_destroy", "plk_ctx_stream", "plk_ctx_synchronize", "plk_domain_get",
    "plk_domain_info", "plk_domain_elements", "plk_domain_vanishing_over_coset", "plk_ntt",
    "plk_ntt_dev", "plk_ntt_batch_dev", "plk_srs_setup", "plk_srs_load", "plk_srs_destroy",
    "plk_srs_len", "plk_srs_points", "plk_msm", "plk_commit", "plk_commit_dev",
    "plk_srs_last_msm_stats", "plk_debug_field_op", "plk_commit_batch_dev",
    "plk_commit_batch_dev_part",
    "plk_srs_setup_range", "plk_g1_sum", "plk_msm_sharded", "plk_srs_msm_stats_reset",
    "plk_srs_cum_msm_stats", "plk_ntt_stream", "plk_aggregate_witness",
    "plk_aggregate_witness_dev",
    # prover (dusk-plonk_amd/prover.py binds these)
    "plk_composer_create", "plk_composer_destroy", "plk_composer_size",
    "plk_composer_append_witness", "plk_composer_witness_value", "plk_composer_set_witness",
    "plk_composer_append_public", "plk_composer_append_gate", "plk_composer_append_custom_gate",
    "plk_composer_gate_eval", "plk_composer_assert_equal", "plk_composer_assert_equal_constant",
    "plk_composer_component_boolean", "plk_composer_component_range",
    "plk_composer_synthetic_chain",
    "plk_composer_public_inputs", "plk_composer_export", "plk_key_compile", "plk_key_destroy",
    "plk_key_info",
    "plk_prove", "plk_prover_create", "plk_prover_destroy", "plk_prover_stream",
    "plk_prover_prove", "plk_prover_msm_stats", "plk_prover_shard", "plk_prover_shard_buckets",
    "plk_proof_encode", "plk_proof_decode",
)


class PlonkError(RuntimeError):
    def __init__(self, status: int, what: str = ""):
        self.status = status
        msg = _lib().plk_status_str(status).decode() if _LIB is not None else str(status)
        super().__init__(f"{what}: {msg} (status {status})" if what else msg)


_LIB = None


def _lib():
    """Load libplk.so (built in-tree by build_ext.py). Fails loudly when absent."""
    global _LIB
    if _LIB is None:
        if not _LIB_PATH.exists():
            raise ImportError(f"{_LIB_PATH} not built — run __graft_entry__.build() first")
        # One HIP runtime per process: torch ships its own libamdhip64 (same SONAME as
        # /opt/rocm's). Loading torch first makes libplk bind to that copy, so device
        # pointers and hipStream_t handles from torch are valid in our calls.
        try:
            import torch  # noqa: F401
        except Exception:
            pass
        lib = C.CDLL(str(_LIB_PATH))
        vp, u32, u64, sz, i32 = C.c_void_p, C.c_uint32, C.c_uint64, C.c_size_t, C.c_int
        pp = C.POINTER(C.c_void_p)
        sig = {
            "plk_abi_version": (i32, []),
            "plk_status_str": (C.c_char_p, [i32]),
            "plk_build_info": (C.c_char_p, []),
            "plk_device_count": (i32, [C.POINTER(i32)]),
            "plk_ctx_create": (i32, [i32, pp]),
            "plk_ctx_destroy": (i32, [vp]),
            "plk_ctx_stream": (i32, [vp, pp]),
            "plk_ctx_synchronize": (i32, [vp]),
            "plk_domain_get": (i32, [vp, u32, pp]),
            "plk_domain_info": (i32, [vp, C.POINTER(u64), vp, vp, vp, vp, vp]),
            "plk_domain_elements": (i32, [vp, vp]),
            "plk_domain_vanishing_over_coset": (i32, [vp, u64, vp]),
            "plk_ntt": (i32, [vp, vp, sz, i32, i32]),
            "plk_ntt_dev": (i32, [vp, vp, vp, sz, i32, i32, vp, vp]),
            "plk_ntt_stream": (i32, [vp, vp, sz, i32, i32, vp]),
            "plk_aggregate_witness": (i32, [vp, vp, vp, sz, vp, vp, vp, C.POINTER(sz)]),
            "plk_aggregate_witness_dev": (i32, [vp, vp, vp, sz, vp, vp, vp, C.POINTER(sz), vp]),
            "plk_ntt_batch_dev": (i32, [vp, vp, sz, i32, i32, vp]),
            "plk_srs_setup": (i32, [vp, vp, sz, vp, pp]),
            "plk_srs_load": (i32, [vp, vp, sz, pp]),
            "plk_srs_destroy": (i32, [vp]),
            "plk_srs_len": (i32, [vp, C.POINTER(sz)]),
            "plk_srs_points": (i32, [vp, sz, sz, vp]),
            "plk_msm": (i32, [vp, vp, sz, vp]),
            "plk_commit": (i32, [vp, vp, sz, vp]),
            "plk_commit_dev": (i32, [vp, vp, sz, vp, vp]),
            "plk_srs_last_msm_stats": (i32, [vp, C.POINTER(C.c_float), C.POINTER(u64),
                                             C.POINTER(u32)]),
            "plk_debug_field_op": (i32, [vp, i32, i32, vp, vp, vp, sz]),
            "plk_commit_batch_dev": (i32, [vp, vp, vp, sz, vp, vp, vp]),
            "plk_commit_batch_dev_part": (i32, [vp, vp, vp, sz, u32, u32, vp, vp, vp]),
            "plk_srs_setup_range": (i32, [vp, vp, u64, sz, vp, pp]),
            "plk_g1_sum": (i32, [vp, sz, vp]),
            "plk_msm_sharded": (i32, [vp, i32, vp, sz, vp]),
            "plk_srs_msm_stats_reset": (i32, [vp]),
            "plk_srs_cum_msm_stats": (i32, [vp, C.POINTER(C.c_double), C.POINTER(u64),
                                            C.POINTER(u64), C.POINTER(u64)]),
        }
        for name, (res, args) in sig.items():
            f = getattr(lib, name)
            f.restype, f.argtypes = res, args
        _LIB = lib
    return _LIB


def build_info() -> dict:
    """plk_build_info of the loaded library: {'src', 'flags', 'variant', 'lib'}."""
    raw = _lib().plk_build_info().decode()
    d = dict(kv.split("=", 1) for kv in raw.split())
    d["lib"] = str(_LIB_PATH)
    return d


def check_build(root: Path | None = None) -> dict:
    """Refuse a library built from other sources than the tree it is loaded from (round-5
    verdict: a pushed prebuilt libplk.so was not tied to its sources). The default library
    must also carry the default flags; a PLK_LIB variant (tools/ab.py) may differ in flags.
    Returns build_info() with the tree's ids; raises ImportError on a mismatch."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("_plk_build_ext", _PKG / "build_ext.py")
    be = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(be)
    info = build_info()
    tree_src = be.source_id(root or be.ROOT)
    info["tree_src"] = tree_src
    if os.environ.get("PLK_LIB") and os.environ.get("PLK_LIB_ANY_SRC") == "1":
        info["src_check"] = "skipped (PLK_LIB variant with PLK_LIB_ANY_SRC=1: an A/B against another tree)"
        return info
    if info.get("src") != tree_src:
        raise ImportError(f"{_LIB_PATH} was built from other sources (library src={info.get('src')}, "
                          f"tree src={tree_src}): rebuild with __graft_entry__.build()")
    if not os.environ.get("PLK_LIB") and info.get("flags") != be.flags_id():
        raise ImportError(f"{_LIB_PATH} was built with other flags (library flags={info.get('flags')}, "
                          f"default flags={be.flags_id()}): rebuild with __graft_entry__.build()")
    return info


def _check(status: int, what: str):
    if status != PLK_OK:
        raise PlonkError(status, what)


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


def device_count() -> int:
    n = C.c_int(0)
    _check(_lib().plk_device_count(C.byref(n)), "plk_device_count")
    return n.value


# ------------------------------------------------------------------------------ context
class Context:
    """One plk_ctx per GPU (device memory, stream, cached Fft domains)."""

    _default: dict[int, "Context"] = {}

    def __init__(self, device: int = 0):
        h = C.c_void_p()
        _check(_lib().plk_ctx_create(device, C.byref(h)), "plk_ctx_create")
        self.handle = h
        self.device = device
        self._domains: dict[int, C.c_void_p] = {}

    @classmethod
    def default(cls, device: int | None = None) -> "Context":
        if device is None:
            device = int(os.environ.get("LOCAL_RANK", "0")) if "LOCAL_RANK" in os.environ else 0
            try:
                import torch  # noqa: F401 — only to follow torch's current device when present
                if torch.cuda.is_available():
                    device = torch.cuda.current_device()
            except Exception:
                pass
        if device not in cls._default:
            cls._default[device] = Context(device)
        return cls._default[device]

    def stream(self) -> int:
        s = C.c_void_p()
        _check(_lib().plk_ctx_stream(self.handle, C.byref(s)), "plk_ctx_stream")
        return s.value or 0

    def synchronize(self):
        _check(_lib().plk_ctx_synchronize(self.handle), "plk_ctx_synchronize")

    def field_op(self, field: str, op: str, a: np.ndarray, b: np.ndarray | None = None):
        """Elementwise device field arithmetic (test support): field 'fr'|'fp',
        op 'mul'|'add'|'sub'|'sqr'|'inv'; Montgomery limbs in and out."""
        w = 4 if field == "fr" else 6
        a = np.ascontiguousarray(np.asarray(a, dtype=np.uint64).reshape(-1, w))
        bb = None if b is None else np.ascontiguousarray(np.asarray(b, dtype=np.uint64).reshape(-1, w))
        out = np.zeros_like(a)
        code = {"mul": 0, "add": 1, "sub": 2, "sqr": 3, "inv": 4}[op]
        _check(_lib().plk_debug_field_op(self.handle, 0 if field == "fr" else 1, code, _ptr(a),
                                         None if bb is None else _ptr(bb), _ptr(out), a.shape[0]),
               "plk_debug_field_op")
        return out

    def domain(self, k: int) -> C.c_void_p:
        if k not in self._domains:
            d = C.c_void_p()
            _check(_lib().plk_domain_get(self.handle, k, C.byref(d)), "plk_domain_get")
            self._domains[k] = d
        return self._domains[k]


# ------------------------------------------------------------------------ value types
def _as_fr_array(values) -> np.ndarray:
    a = np.ascontiguousarray(np.asarray(values, dtype=np.uint64))
    if a.ndim == 1 and a.size % 4 == 0:
        a = a.reshape(-1, 4)
    if a.ndim != 2 or a.shape[1] != 4:
        raise ValueError("expected uint64[n, 4] Montgomery Fr limbs")
    return a


class Coefficients:
    """poly_commit::Coefficients<Fr> — ``pub Vec<F>`` of coefficients (``.0`` is ``.values``)."""

    def __init__(self, values):
        self.values = _as_fr_array(values)

    def __len__(self):
        return self.values.shape[0]

    def clone(self):
        return type(self)(self.values.copy())

    def degree(self) -> int:
        """Index of the last non-zero coefficient (0 for the zero polynomial)."""
        nz = np.nonzero(self.values.any(axis=1))[0]
        return int(nz[-1]) if nz.size else 0


class PointsValue(Coefficients):
    """poly_commit::PointsValue<Fr> — evaluations over a domain."""


# ------------------------------------------------------------------------------- Fft
class Fft:
    """poly_commit::Fft<Fr> on the GPU: ``Fft(k)`` = ``Fft::new(k)`` (n = 2^k).

    w = ROOT_OF_UNITY^(2^(32-k)); cosets use g = 7; tables live in HBM per context.
    """

    def __init__(self, k: int, ctx: Context | None = None):
        self.ctx = ctx or Context.default()
        self.k = k
        self._d = self.ctx.domain(k)
        n = C.c_uint64()
        self._consts = [np.zeros(4, dtype=np.uint64) for _ in range(5)]
        _check(_lib().plk_domain_info(self._d, C.byref(n), *[_ptr(c) for c in self._consts]),
               "plk_domain_info")
        self._n = n.value
        self._elements = None

    # -- accessors (key.rs:205-207, prover.rs:252,446)
    def size(self) -> int:
        return self._n

    def generator(self) -> np.ndarray:
        return self._consts[0].copy()

    def generator_inv(self) -> np.ndarray:
        return self._consts[1].copy()

    def size_inv(self) -> np.ndarray:
        return self._consts[2].copy()

    def coset_generator(self) -> np.ndarray:
        return self._consts[3].copy()

    @property
    def elements(self) -> np.ndarray:
        """elements[i] = w^i (permutation.rs:148)."""
        if self._elements is None:
            out = np.zeros((self._n, 4), dtype=np.uint64)
            _check(_lib().plk_domain_elements(self._d, _ptr(out)), "plk_domain_elements")
            self._elements = out
        return self._elements

    def compute_vanishing_poly_over_coset(self, poly_degree: int) -> PointsValue:
        out = np.zeros((self._n, 4), dtype=np.uint64)
        _check(_lib().plk_domain_vanishing_over_coset(self._d, poly_degree, _ptr(out)),
               "plk_domain_vanishing_over_coset")
        return PointsValue(out)

    # -- transforms
    def _run(self, vals: np.ndarray, direction: int, coset: int, stream: int = 0) -> np.ndarray:
        """stream != 0: plk_ntt_stream on that hipStream_t (own staging, so threads with
        their own streams may share this Fft); else plk_ntt on the context's stream."""
        vals = _as_fr_array(vals)
        if vals.shape[0] > self._n:
            raise ValueError(f"input of length {vals.shape[0]} exceeds the domain size {self._n}")
        buf = np.zeros((self._n, 4), dtype=np.uint64)
        buf[: vals.shape[0]] = vals
        if stream:
            _check(_lib().plk_ntt_stream(self._d, _ptr(buf), vals.shape[0], direction, coset,
                                         C.c_void_p(stream)), "plk_ntt_stream")
        else:
            _check(_lib().plk_ntt(self._d, _ptr(buf), vals.shape[0], direction, coset), "plk_ntt")
        return buf

    def dft(self, coeffs: Coefficients, stream: int = 0) -> PointsValue:
        return PointsValue(self._run(coeffs.values, 1, 0, stream))

    def idft(self, points: PointsValue, stream: int = 0) -> Coefficients:
        return Coefficients(self._run(points.values, -1, 0, stream))

    def coset_dft(self, coeffs: Coefficients, stream: int = 0) -> PointsValue:
        return PointsValue(self._run(coeffs.values, 1, 1, stream))

    def coset_idft(self, points: PointsValue, stream: int = 0) -> Coefficients:
        return Coefficients(self._run(points.values, -1, 1, stream))

    # -- device-resident variants (torch tensors of dtype int64, shape [n, 4], on cuda)
    def ntt_dev(self, d_in_ptr: int, d_out_ptr: int, len_in: int, direction: int, coset: bool,
                stream: int = 0, d_scratch_ptr: int = 0):
        _check(_lib().plk_ntt_dev(self._d, C.c_void_p(d_in_ptr), C.c_void_p(d_out_ptr), len_in,
                                  direction, int(coset), C.c_void_p(d_scratch_ptr or None),
                                  C.c_void_p(stream or None)), "plk_ntt_dev")


# ------------------------------------------------------------------------------ KZG
class Commitment:
    """Commitment<G1Affine>: one canonical affine point (uint64[13])."""

    def __init__(self, words: np.ndarray):
        self.words = np.asarray(words, dtype=np.uint64).reshape(13)

    @property
    def is_identity(self) -> bool:
        return bool(self.words[12])

    def __eq__(self, other):
        return isinstance(other, Commitment) and np.array_equal(self.words, other.words)

    def __repr__(self):
        return "Commitment(identity)" if self.is_identity else \
            f"Commitment(x0={int(self.words[0]):#x}...)"


def g1_sum(points: np.ndarray) -> Commitment:
    """Host-side sum of affine points uint64[n, 13] (no GPU needed)."""
    pts = np.ascontiguousarray(np.asarray(points, dtype=np.uint64).reshape(-1, 13))
    out = np.zeros(13, dtype=np.uint64)
    _check(_lib().plk_g1_sum(_ptr(pts), pts.shape[0], _ptr(out)), "plk_g1_sum")
    return Commitment(out)


def msm_sharded(shards, scalars) -> Commitment:
    """One MSM over consecutive SRS slices held by different GPUs of this process
    (PlonkParams.setup_range per device, in order): plk_msm_sharded."""
    vals = _as_fr_array(scalars)
    hs = (C.c_void_p * len(shards))(*[s._h.value for s in shards])
    out = np.zeros(13, dtype=np.uint64)
    _check(_lib().plk_msm_sharded(hs, len(shards), _ptr(vals), vals.shape[0], _ptr(out)),
           "plk_msm_sharded")
    return Commitment(out)


class PlonkParams:
    """zksnarks::plonk::PlonkParams<TatePairing> (the G1 side used by the prover).

    ``setup(k, tau)`` restates ``PlonkParams::setup(k, rng)`` with an explicit secret tau
    (Montgomery Fr limbs) so the CPU and GPU paths see identical randomness; it emits
    2^k + 8 powers because the blinded z (n+3) and t_4 (up to n+7) overrun 2^k.
    """

    SLACK = 8

    def __init__(self, handle: C.c_void_p, n_points: int, ctx: Context):
        self._h = handle
        self.n = n_points
        self.ctx = ctx

    @classmethod
    def setup(cls, k: int, tau, ctx: Context | None = None, n_points: int | None = None):
        ctx = ctx or Context.default()
        n = n_points if n_points is not None else (1 << k) + cls.SLACK
        tau = _as_fr_array(tau).reshape(4)
        h = C.c_void_p()
        _check(_lib().plk_srs_setup(ctx.handle, _ptr(tau), n, None, C.byref(h)), "plk_srs_setup")
        return cls(h, n, ctx)

    @classmethod
    def setup_range(cls, tau, start: int, count: int, ctx: Context | None = None):
        """The slice [start, start + count) of the SRS of `tau` (a sharded MSM's shard)."""
        ctx = ctx or Context.default()
        tau = _as_fr_array(tau).reshape(4)
        h = C.c_void_p()
        _check(_lib().plk_srs_setup_range(ctx.handle, _ptr(tau), start, count, None, C.byref(h)),
               "plk_srs_setup_range")
        return cls(h, count, ctx)

    @classmethod
    def load(cls, points: np.ndarray, ctx: Context | None = None):
        ctx = ctx or Context.default()
        pts = np.ascontiguousarray(np.asarray(points, dtype=np.uint64).reshape(-1, 13))
        h = C.c_void_p()
        _check(_lib().plk_srs_load(ctx.handle, _ptr(pts), pts.shape[0], C.byref(h)), "plk_srs_load")
        return cls(h, pts.shape[0], ctx)

    def trim(self, n: int) -> "PlonkParams":
        """Keep the first n + SLACK powers (key.rs:81-82)."""
        keep = min(self.n, n + self.SLACK)
        if keep == self.n:
            return self
        return PlonkParams.load(self.points(0, keep), self.ctx)

    def points(self, start: int = 0, count: int | None = None) -> np.ndarray:
        count = self.n - start if count is None else count
        out = np.zeros((count, 13), dtype=np.uint64)
        _check(_lib().plk_srs_points(self._h, start, count, _ptr(out)), "plk_srs_points")
        return out

    def commit(self, poly: Coefficients) -> Commitment:
        vals = _as_fr_array(poly.values if isinstance(poly, Coefficients) else poly)
        out = np.zeros(13, dtype=np.uint64)
        _check(_lib().plk_commit(self._h, _ptr(vals), vals.shape[0], _ptr(out)), "commit")
        return Commitment(out)

    def msm(self, scalars) -> Commitment:
        vals = _as_fr_array(scalars)
        out = np.zeros(13, dtype=np.uint64)
        _check(_lib().plk_msm(self._h, _ptr(vals), vals.shape[0], _ptr(out)), "msm")
        return Commitment(out)

    def commit_dev(self, d_ptr: int, length: int, stream: int = 0) -> Commitment:
        out = np.zeros(13, dtype=np.uint64)
        _check(_lib().plk_commit_dev(self._h, C.c_void_p(d_ptr), length, _ptr(out),
                                     C.c_void_p(stream or None)), "commit_dev")
        return Commitment(out)

    def commit_batch_dev(self, ptrs_lens, stream: int = 0, raise_on_error: bool = True,
                         part: int = 0, parts: int = 1):
        """Commit several device-resident polynomials [(ptr, len), ...] as one batch.
        Returns a list of Commitment (or PlonkError per failed slot when not raising).
        parts > 1: only bucket range `part` of `parts` (plk_commit_batch_dev_part): the
        returned points are that range's shares, which sum over the parts to the commits."""
        k = len(ptrs_lens)
        ptrs = (C.c_void_p * k)(*[C.c_void_p(p) for p, _ in ptrs_lens])
        lens = (C.c_size_t * k)(*[n for _, n in ptrs_lens])
        outs = np.zeros((k, 13), dtype=np.uint64)
        sts = (C.c_int * k)()
        if parts == 1:
            st = _lib().plk_commit_batch_dev(self._h, ptrs, lens, k, _ptr(outs), sts,
                                             C.c_void_p(stream or None))
        else:
            st = _lib().plk_commit_batch_dev_part(self._h, ptrs, lens, k, part, parts, _ptr(outs),
                                                  sts, C.c_void_p(stream or None))
        if st not in (PLK_OK, PLK_E_DEGREE) or (raise_on_error and st != PLK_OK):
            raise PlonkError(st, "commit_batch_dev")
        return [Commitment(outs[i]) if sts[i] == PLK_OK else PlonkError(sts[i], "commit")
                for i in range(k)]

    def compute_aggregate_witness(self, polys, point, challenge) -> Coefficients:
        """PlonkParams::compute_aggregate_witness (prover.rs:422-450):
        (sum_i challenge^i polys[i]) / (X - point), remainder dropped (plk_aggregate_witness)."""
        arrs = [_as_fr_array(p.values if isinstance(p, Coefficients) else p) for p in polys]
        k = len(arrs)
        ptrs = (C.c_void_p * max(k, 1))(*[C.c_void_p(a.ctypes.data) for a in arrs])
        lens = (C.c_size_t * max(k, 1))(*[a.shape[0] for a in arrs])
        pt = _as_fr_array(point).reshape(4)
        ch = _as_fr_array(challenge).reshape(4)
        m = max((a.shape[0] for a in arrs), default=0)
        out = np.zeros((max(m - 1, 1), 4), dtype=np.uint64)
        n_out = C.c_size_t()
        _check(_lib().plk_aggregate_witness(self.ctx.handle, ptrs, lens, k, _ptr(pt), _ptr(ch),
                                            _ptr(out), C.byref(n_out)), "compute_aggregate_witness")
        return Coefficients(out[: n_out.value])

    def compute_aggregate_witness_dev(self, ptrs_lens, point, challenge, d_out: int,
                                      stream: int = 0) -> int:
        """Device form (plk_aggregate_witness_dev): [(ptr, len)] -> d_out; returns its length."""
        k = len(ptrs_lens)
        ptrs = (C.c_void_p * max(k, 1))(*[C.c_void_p(p) for p, _ in ptrs_lens])
        lens = (C.c_size_t * max(k, 1))(*[n for _, n in ptrs_lens])
        pt = _as_fr_array(point).reshape(4)
        ch = _as_fr_array(challenge).reshape(4)
        n_out = C.c_size_t()
        _check(_lib().plk_aggregate_witness_dev(self.ctx.handle, ptrs, lens, k, _ptr(pt), _ptr(ch),
                                                C.c_void_p(d_out or None), C.byref(n_out),
                                                C.c_void_p(stream or None)),
               "compute_aggregate_witness_dev")
        return n_out.value

    def msm_stats_reset(self):
        _check(_lib().plk_srs_msm_stats_reset(self._h), "plk_srs_msm_stats_reset")

    def cum_msm_stats(self):
        """(accumulate ms, launches, point adds, MSM points) since msm_stats_reset."""
        ms, ln, adds, pts = C.c_double(), C.c_uint64(), C.c_uint64(), C.c_uint64()
        _check(_lib().plk_srs_cum_msm_stats(self._h, C.byref(ms), C.byref(ln), C.byref(adds),
                                            C.byref(pts)), "plk_srs_cum_msm_stats")
        return ms.value, ln.value, adds.value, pts.value

    def last_msm_stats(self):
        ms, adds, c = C.c_float(), C.c_uint64(), C.c_uint32()
        _check(_lib().plk_srs_last_msm_stats(self._h, C.byref(ms), C.byref(adds), C.byref(c)),
               "plk_srs_last_msm_stats")
        return ms.value, adds.value, c.value

    def __del__(self):
        try:
            if self._h and _LIB is not None:
                _LIB.plk_srs_destroy(self._h)
        except Exception:
            pass
        self._h = None
