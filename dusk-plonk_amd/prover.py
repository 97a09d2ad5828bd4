"""Host-side mirror of the reference's prover API over the C ABI (include/plk.h):

* ``Constraint`` — zksnarks::Constraint builder (``mult/left/right/output/fourth/constant/
  public/a/b/o/d``), values as Python ints (canonical Fr) or Montgomery limb arrays.
* ``Plonk`` — the composer (``src/lib.rs``: ``append_witness``, ``append_public``,
  ``append_gate``, ``gate_add``, ``gate_mul``, ``assert_equal``, ``assert_equal_constant``,
  ``component_boolean``); ``Plonk()`` is ``Plonk::initialize()``.
* ``PlonkKey.compile_with_circuit(pp, label, circuit)`` — ``src/key.rs:63-327``, returning
  ``(Prover, VerifierData)``; ``Prover.create_proof(seed, circuit)`` — ``src/prover.rs:67``,
  returning ``(Proof, public_inputs)``. A circuit is any object with
  ``synthesize(composer)`` (the reference's ``Circuit`` trait).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from .plonk import (PLK_OK, PlonkError, PlonkParams, _check, _lib, _ptr)

R_MOD = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
_R = 1 << 256


class PlkFr(C.Structure):
    _fields_ = [("l", C.c_uint64 * 4)]


class PlkG1(C.Structure):
    _fields_ = [("x", C.c_uint64 * 6), ("y", C.c_uint64 * 6), ("infinity", C.c_uint64)]


_SEL = ["q_m", "q_l", "q_r", "q_o", "q_4", "q_c", "q_arith", "q_range", "q_logic",
        "q_fixed_group_add", "q_variable_group_add"]


class PlkConstraint(C.Structure):
    _fields_ = [(s, PlkFr) for s in _SEL] + [
        ("a", C.c_uint32), ("b", C.c_uint32), ("o", C.c_uint32), ("d", C.c_uint32),
        ("has_public", C.c_uint32), ("_pad", C.c_uint32), ("public_input", PlkFr)]


_COMMS = ["a_comm", "b_comm", "c_comm", "d_comm", "z_comm", "t_low_comm", "t_mid_comm",
          "t_high_comm", "t_4_comm", "w_z_chall_comm", "w_z_chall_w_comm"]
_EVALS = ["a_eval", "b_eval", "c_eval", "d_eval", "a_next_eval", "b_next_eval", "d_next_eval",
          "q_arith_eval", "q_c_eval", "q_l_eval", "q_r_eval", "s_sigma_1_eval",
          "s_sigma_2_eval", "s_sigma_3_eval", "r_poly_eval", "perm_eval"]


class PlkProof(C.Structure):
    _fields_ = [(c, PlkG1) for c in _COMMS] + [(e, PlkFr) for e in _EVALS]


# plk_allgather_fn (include/plk.h): (user, send, bytes, recv) -> 0 on success
ALLGATHER_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p)
PROOF_SCALE_BYTES = 11 * 97 + 16 * 32  # PLK_PROOF_SCALE_BYTES


def _bind():
    lib = _lib()
    if getattr(lib, "_prover_bound", False):
        return lib
    vp, u32, u64, sz, i32 = C.c_void_p, C.c_uint32, C.c_uint64, C.c_size_t, C.c_int
    pp = C.POINTER(C.c_void_p)
    sig = {
        "plk_composer_create": [pp], "plk_composer_destroy": [vp],
        "plk_composer_size": [vp, C.POINTER(sz), C.POINTER(sz)],
        "plk_composer_append_witness": [vp, vp, C.POINTER(u32)],
        "plk_composer_witness_value": [vp, u32, vp],
        "plk_composer_set_witness": [vp, u32, vp],
        "plk_composer_append_public": [vp, vp, C.POINTER(u32)],
        "plk_composer_append_gate": [vp, vp], "plk_composer_append_custom_gate": [vp, vp],
        "plk_composer_gate_eval": [vp, vp, C.POINTER(u32)],
        "plk_composer_assert_equal": [vp, u32, u32],
        "plk_composer_assert_equal_constant": [vp, u32, vp, vp],
        "plk_composer_component_boolean": [vp, u32],
        "plk_composer_component_range": [vp, u32, sz],
        "plk_composer_synthetic_chain": [vp, sz, u64],
        "plk_composer_public_inputs": [vp, vp, vp, sz, C.POINTER(sz)],
        "plk_composer_export": [vp, vp, sz, vp, sz, C.POINTER(sz), C.POINTER(sz)],
        "plk_key_compile": [vp, vp, C.c_char_p, pp], "plk_key_destroy": [vp],
        "plk_key_info": [vp, C.POINTER(u64), C.POINTER(u64), vp],
        "plk_prove": [vp, vp, u64, vp, vp, sz, C.POINTER(sz)],
        "plk_prover_create": [vp, pp], "plk_prover_destroy": [vp],
        "plk_prover_stream": [vp, pp],
        "plk_prover_prove": [vp, vp, u64, vp, vp, sz, C.POINTER(sz)],
        "plk_prover_msm_stats": [vp, i32, C.POINTER(C.c_double), C.POINTER(u64),
                                 C.POINTER(u64), C.POINTER(u64)],
        "plk_prover_shard": [vp, vp, u64, i32, i32, vp, vp],  # fn: ALLGATHER_FN cast
        "plk_prover_shard_buckets": [vp, i32, i32, vp, vp],
        "plk_proof_encode": [vp, vp, sz, C.POINTER(sz)],
        "plk_proof_decode": [vp, sz, vp],
    }
    for name, args in sig.items():
        f = getattr(lib, name)
        f.restype, f.argtypes = i32, args
    lib._prover_bound = True
    return lib


def _fr(v) -> PlkFr:
    """Python int (canonical) or Montgomery limb array -> PlkFr (Montgomery)."""
    out = PlkFr()
    if isinstance(v, (int, np.integer)):
        m = (int(v) % R_MOD) * _R % R_MOD
        for i in range(4):
            out.l[i] = (m >> (64 * i)) & 0xFFFFFFFFFFFFFFFF
    else:
        a = np.asarray(v, dtype=np.uint64).reshape(4)
        for i in range(4):
            out.l[i] = int(a[i])
    return out


def fr_limbs(p: PlkFr) -> np.ndarray:
    return np.array([p.l[i] for i in range(4)], dtype=np.uint64)


def fr_int(p) -> int:
    """Montgomery limbs (PlkFr or array) -> canonical int."""
    a = fr_limbs(p) if isinstance(p, PlkFr) else np.asarray(p, dtype=np.uint64)
    v = sum(int(a[i]) << (64 * i) for i in range(4))
    return v * pow(_R, -1, R_MOD) % R_MOD


class Constraint:
    """zksnarks::Constraint builder (selectors default 0, wires default Plonk::ZERO)."""

    def __init__(self):
        self.c = PlkConstraint()

    def _set(self, name, v):
        setattr(self.c, name, _fr(v))
        return self

    def mult(self, v):
        return self._set("q_m", v)

    def left(self, v):
        return self._set("q_l", v)

    def right(self, v):
        return self._set("q_r", v)

    def output(self, v):
        return self._set("q_o", v)

    def fourth(self, v):
        return self._set("q_4", v)

    def constant(self, v):
        return self._set("q_c", v)

    def range(self, v):
        return self._set("q_range", v)

    def logic(self, v):
        return self._set("q_logic", v)

    def public(self, v):
        self.c.has_public = 1
        self.c.public_input = _fr(v)
        return self

    def a(self, w):
        self.c.a = w
        return self

    def b(self, w):
        self.c.b = w
        return self

    def o(self, w):
        self.c.o = w
        return self

    def d(self, w):
        self.c.d = w
        return self


# ---- JubJub (twisted Edwards -x^2 + y^2 = 1 + d x^2 y^2 over Fr), the composer's curve C ----
EDWARDS_D = (-10240 * pow(10241, -1, R_MOD)) % R_MOD
JUBJUB_IDENTITY = (0, 1)
# dusk-jubjub / jub_jub GENERATOR (on the curve, prime-order subgroup; tests/test_ecc)
JUBJUB_GENERATOR = (0x3FD2814C43AC65A6F1FBF02D0FD6CCE62E3EBB21FD6C54ED4DF7B7FFEC7BEACA, 0x12)
JUBJUB_ORDER = 0x0E7DB4EA6533AFA906673B0101343B00A6682093CCC81082D0970E5ED6F72CB7


def jubjub_add(p, q):
    (x1, y1), (x2, y2) = p, q
    t = EDWARDS_D * x1 * x2 * y1 * y2 % R_MOD
    x3 = (x1 * y2 + y1 * x2) * pow(1 + t, -1, R_MOD) % R_MOD
    y3 = (y1 * y2 + x1 * x2) * pow(1 - t, -1, R_MOD) % R_MOD
    return (x3, y3)


def jubjub_neg(p):
    return ((-p[0]) % R_MOD, p[1])


def jubjub_mul(p, k: int):
    acc = JUBJUB_IDENTITY
    for b in bin(k)[2:] if k > 0 else "":
        acc = jubjub_add(acc, acc)
        if b == "1":
            acc = jubjub_add(acc, p)
    return acc


def windowed_naf(k: int, width: int = 2):
    """compute_windowed_naf(scalar, width) (zkstd, un-vendored): signed digits, least
    significant first, 256 entries; width 2 gives the NAF with digits in {-1, 0, 1}."""
    out = [0] * 256
    i = 0
    while k >= 1:
        if k & 1:
            d = k % (1 << width)
            if d >= 1 << (width - 1):
                d -= 1 << width
            out[i] = d
            k -= d
        k >>= 1
        i += 1
    return out


class WitnessPoint:
    def __init__(self, x: int, y: int):
        self.x, self.y = x, y


class Plonk:
    """The composer, Plonk<JubjubAffine> (src/lib.rs:103-115); construction = initialize()."""

    ZERO = 0
    ONE = 1

    def __init__(self):
        lib = _bind()
        h = C.c_void_p()
        _check(lib.plk_composer_create(C.byref(h)), "plk_composer_create")
        self._h = h

    def __del__(self):
        try:
            if self._h:
                _bind().plk_composer_destroy(self._h)
        except Exception:
            pass

    def m(self) -> int:
        g = C.c_size_t()
        _check(_bind().plk_composer_size(self._h, C.byref(g), None), "size")
        return g.value

    def set_witness(self, w: int, v):
        """Overwrite witness `w` (plk_composer_set_witness): a new instance of the same
        circuit structure."""
        f = _fr(v)
        _check(_bind().plk_composer_set_witness(self._h, w, C.byref(f)), "set_witness")

    def append_witness(self, v) -> int:
        w = C.c_uint32()
        f = _fr(v)
        _check(_bind().plk_composer_append_witness(self._h, C.byref(f), C.byref(w)), "witness")
        return w.value

    def __getitem__(self, w) -> int:
        f = PlkFr()
        _check(_bind().plk_composer_witness_value(self._h, w, C.byref(f)), "witness_value")
        return fr_int(f)

    def append_public(self, v) -> int:
        w = C.c_uint32()
        f = _fr(v)
        _check(_bind().plk_composer_append_public(self._h, C.byref(f), C.byref(w)), "public")
        return w.value

    def append_gate(self, c: Constraint):
        _check(_bind().plk_composer_append_gate(self._h, C.byref(c.c)), "append_gate")

    def append_custom_gate(self, c: Constraint):
        _check(_bind().plk_composer_append_custom_gate(self._h, C.byref(c.c)), "custom_gate")

    def gate_add(self, c: Constraint) -> int:
        w = C.c_uint32()
        _check(_bind().plk_composer_gate_eval(self._h, C.byref(c.c), C.byref(w)), "gate_add")
        return w.value

    gate_mul = gate_add  # both evaluate o with q_o = -1 (lib.rs:1169-1197)

    def assert_equal(self, a: int, b: int):
        _check(_bind().plk_composer_assert_equal(self._h, a, b), "assert_equal")

    def assert_equal_constant(self, a: int, constant, public=None):
        c = _fr(constant)
        p = None if public is None else C.byref(_fr(public))
        _check(_bind().plk_composer_assert_equal_constant(self._h, a, C.byref(c), p),
               "assert_equal_constant")

    def component_boolean(self, a: int):
        _check(_bind().plk_composer_component_boolean(self._h, a), "component_boolean")

    # ---- arithmetic-gate gadgets, restating src/lib.rs on top of the gate calls ----------
    def component_decomposition(self, scalar: int, n: int):
        """lib.rs:877-909: bits of `scalar` (LSB first, N of them), each boolean-constrained,
        recombined with gate_add and asserted equal to the scalar (2N + 1 gates)."""
        assert 0 < n <= 256
        value = self[scalar]
        acc = self.ZERO
        bits = []
        for i in range(n):
            d = self.append_witness((value >> i) & 1)
            self.component_boolean(d)
            acc = self.gate_add(Constraint().left(pow(2, i, R_MOD)).right(1).a(d).b(acc))
            bits.append(d)
        self.assert_equal(acc, scalar)
        return bits

    def component_select(self, bit: int, a: int, b: int) -> int:
        """lib.rs:959-990: bit ? a : b."""
        bit_times_a = self.gate_mul(Constraint().mult(1).a(bit).b(a))
        one_min_bit = self.gate_add(Constraint().left(-1).constant(1).a(bit))
        one_min_bit_b = self.gate_mul(Constraint().mult(1).a(one_min_bit).b(b))
        return self.gate_add(Constraint().left(1).right(1).a(one_min_bit_b).b(bit_times_a))

    def component_select_one(self, bit: int, value: int) -> int:
        """lib.rs:996-1020: bit ? value : 1."""
        b, v = self[bit], self[value]
        f_x = self.append_witness((1 - b + b * v) % R_MOD)
        self.append_gate(Constraint().mult(1).left(-1).output(-1).constant(1)
                         .a(bit).b(value).o(f_x))
        return f_x

    def component_select_zero(self, bit: int, value: int) -> int:
        """lib.rs:1047-1057: bit ? value : 0."""
        return self.gate_mul(Constraint().mult(1).a(bit).b(value))

    def append_logic_and(self, a: int, b: int, num_bits: int) -> int:
        """lib.rs:738-745"""
        return self._append_logic_component(a, b, num_bits, False)

    def append_logic_xor(self, a: int, b: int, num_bits: int) -> int:
        """lib.rs:754-761"""
        return self._append_logic_component(a, b, num_bits, True)

    def _append_logic_component(self, a: int, b: int, num_bits: int, xor: bool) -> int:
        """lib.rs:284-391: 2-bit quads of the low num_bits of a and b, most significant
        first, accumulated 4x per gate (a, b, d wires: left, right, output accumulators; c:
        the quad product), q_logic = q_c = 1 (AND) or -1 (XOR), closed by a zero gate."""
        num_bits = min(num_bits, 256)
        num_quads = num_bits >> 1
        av, bv = self[a], self[b]
        a_bits = [(av >> (num_bits - 1 - j)) & 1 for j in range(num_bits)]
        b_bits = [(bv >> (num_bits - 1 - j)) & 1 for j in range(num_bits)]
        sel = -1 if xor else 1
        con = Constraint().logic(sel).constant(sel)
        left = right = out = 0
        for i in range(num_quads):
            lq = (a_bits[2 * i] << 1) + a_bits[2 * i + 1]
            rq = (b_bits[2 * i] << 1) + b_bits[2 * i + 1]
            oq = (lq ^ rq) if xor else (lq & rq)
            left, right, out = left * 4 + lq, right * 4 + rq, out * 4 + oq
            wa, wb = self.append_witness(left), self.append_witness(right)
            wc, wd = self.append_witness(lq * rq), self.append_witness(out)
            con.o(wc)
            self.append_custom_gate(con)
            con.a(wa).b(wb).d(wd)
        d = con.c.d
        self.append_custom_gate(Constraint().a(con.c.a).b(con.c.b).d(d))
        return d

    # ---- curve gadgets (lib.rs), JubJub points as pairs of witnesses ------------------
    IDENTITY = WitnessPoint(0, 1)

    def append_constant(self, v) -> int:
        w = self.append_witness(v)
        self.assert_equal_constant(w, v)
        return w

    def append_point(self, p) -> WitnessPoint:
        """lib.rs:657-664"""
        return WitnessPoint(self.append_witness(p[0]), self.append_witness(p[1]))

    def append_constant_point(self, p) -> WitnessPoint:
        """lib.rs:668-678"""
        return WitnessPoint(self.append_constant(p[0]), self.append_constant(p[1]))

    def append_public_point(self, p) -> WitnessPoint:
        """lib.rs:683-700"""
        pt = self.append_point(p)
        self.assert_equal_constant(pt.x, 0, -p[0])
        self.assert_equal_constant(pt.y, 0, -p[1])
        return pt

    def assert_equal_point(self, a: WitnessPoint, b: WitnessPoint):
        """lib.rs:781-784"""
        self.assert_equal(a.x, b.x)
        self.assert_equal(a.y, b.y)

    def assert_equal_public_point(self, point: WitnessPoint, p):
        """lib.rs:789-805"""
        self.assert_equal_constant(point.x, 0, -p[0])
        self.assert_equal_constant(point.y, 0, -p[1])

    def component_add_point(self, a: WitnessPoint, b: WitnessPoint) -> WitnessPoint:
        """lib.rs:810-852: two gates, (x1, y1, x2, y2) with q_variable_group_add = 1 and
        (x3, y3, ., x1 y2)."""
        x1, y1, x2, y2 = self[a.x], self[a.y], self[b.x], self[b.y]
        x3, y3 = jubjub_add((x1, y1), (x2, y2))
        w_x1y2 = self.append_witness(x1 * y2 % R_MOD)
        w_x3, w_y3 = self.append_witness(x3), self.append_witness(y3)
        con = Constraint().a(a.x).b(a.y).o(b.x).d(b.y)
        con._set("q_variable_group_add", 1)
        self.append_custom_gate(con)
        self.append_custom_gate(Constraint().a(w_x3).b(w_y3).d(w_x1y2))
        return WitnessPoint(w_x3, w_y3)

    def component_select_identity(self, bit: int, a: WitnessPoint) -> WitnessPoint:
        """lib.rs:920-929: bit ? a : identity"""
        return WitnessPoint(self.component_select_zero(bit, a.x),
                            self.component_select_one(bit, a.y))

    def component_select_point(self, bit: int, a: WitnessPoint, b: WitnessPoint):
        """lib.rs:1028-1040"""
        return WitnessPoint(self.component_select(bit, a.x, b.x),
                            self.component_select(bit, a.y, b.y))

    def component_mul_point(self, jubjub: int, point: WitnessPoint) -> WitnessPoint:
        """lib.rs:932-954: double-and-add over the 252-bit decomposition."""
        bits = self.component_decomposition(jubjub, 252)
        result = self.IDENTITY
        for bit in reversed(bits):
            result = self.component_add_point(result, result)
            result = self.component_add_point(result, self.component_select_identity(bit, point))
        return result

    def component_mul_generator(self, jubjub: int, generator=JUBJUB_GENERATOR) -> WitnessPoint:
        """lib.rs:395-548: fixed-base multiplication by a width-2 wNAF over the 256
        precomputed multiples 2^i G (constants in q_l, q_r, q_c), one gate per digit with
        q_fixed_group_add = 1, point / scalar accumulators chained to the next gate."""
        bits = 256
        multiples = [generator]
        for _ in range(1, bits):
            multiples.append(jubjub_add(multiples[-1], multiples[-1]))
        multiples.reverse()
        scalar = self[jubjub]
        wnaf = windowed_naf(scalar, 2)
        scalar_acc, point_acc, xy_alphas = [0], [JUBJUB_IDENTITY], []
        for i, entry in enumerate(reversed(wnaf)):
            if entry == 0:
                s_add, p_add = 0, JUBJUB_IDENTITY
            elif entry == -1:
                s_add, p_add = R_MOD - 1, jubjub_neg(multiples[i])
            else:
                s_add, p_add = 1, multiples[i]
            scalar_acc.append((2 * scalar_acc[i] + s_add) % R_MOD)
            point_acc.append(jubjub_add(point_acc[i], p_add))
            xy_alphas.append(p_add[0] * p_add[1] % R_MOD)
        for i in range(bits):
            acc_x = self.append_witness(point_acc[i][0])
            acc_y = self.append_witness(point_acc[i][1])
            acc_bit = self.append_witness(scalar_acc[i])
            if i == 0:
                self.assert_equal_constant(acc_x, 0)
                self.assert_equal_constant(acc_y, 1)
                self.assert_equal_constant(acc_bit, 0)
            x_beta, y_beta = multiples[i]
            xy_alpha = self.append_witness(xy_alphas[i])
            con = (Constraint().left(x_beta).right(y_beta).constant(x_beta * y_beta % R_MOD)
                   .a(acc_x).b(acc_y).o(xy_alpha).d(acc_bit))
            con._set("q_fixed_group_add", 1)
            self.append_custom_gate(con)
        acc_x = self.append_witness(point_acc[bits][0])
        acc_y = self.append_witness(point_acc[bits][1])
        last = self.append_witness(scalar_acc[bits])
        self.append_gate(Constraint().a(acc_x).b(acc_y).d(last))
        self.assert_equal(last, jubjub)
        return WitnessPoint(acc_x, acc_y)

    def component_range(self, a: int, num_bits: int):
        _check(_bind().plk_composer_component_range(self._h, a, num_bits), "component_range")

    def synthetic_chain(self, gates: int, seed: int):
        _check(_bind().plk_composer_synthetic_chain(self._h, gates, seed), "synthetic_chain")

    def export(self):
        """(gates, witness): the circuit as uint64 arrays — gates (m, 51) in plk_constraint
        layout, witness (nw, 4) Montgomery Fr (plk_composer_export)."""
        lib = _bind()
        m, nw = C.c_size_t(), C.c_size_t()
        _check(lib.plk_composer_export(self._h, None, 0, None, 0, C.byref(m), C.byref(nw)),
               "export")
        gates = np.zeros((max(1, m.value), C.sizeof(PlkConstraint) // 8), dtype=np.uint64)
        wit = np.zeros((max(1, nw.value), 4), dtype=np.uint64)
        _check(lib.plk_composer_export(self._h, _ptr(gates), m.value, _ptr(wit), nw.value,
                                       C.byref(m), C.byref(nw)), "export")
        return gates[: m.value], wit[: nw.value]

    def public_inputs(self):
        cnt = C.c_size_t()
        lib = _bind()
        _check(lib.plk_composer_public_inputs(self._h, None, None, 0, C.byref(cnt)), "pi")
        vals = (PlkFr * max(1, cnt.value))()
        idx = (C.c_uint64 * max(1, cnt.value))()
        _check(lib.plk_composer_public_inputs(self._h, vals, idx, cnt.value, C.byref(cnt)), "pi")
        return [fr_int(vals[i]) for i in range(cnt.value)], [idx[i] for i in range(cnt.value)]


class Proof:
    """zksnarks Proof: 11 commitments (uint64[13] each) and 16 evaluations (canonical ints)."""

    def __init__(self, raw: PlkProof):
        self.raw = raw
        for c in _COMMS:
            g = getattr(raw, c)
            setattr(self, c, np.array(list(g.x) + list(g.y) + [g.infinity], dtype=np.uint64))
        for e in _EVALS:
            setattr(self, e, fr_int(getattr(raw, e)))

    def to_bytes(self) -> bytes:
        """The SCALE encoding of the reference's ``Proof`` (``#[derive(Encode)]``,
        src/prover/proof.rs:11,36): 11 commitments then the 16 evaluations, with the
        element encodings ASSUMED as documented at plk_proof_encode (include/plk.h)."""
        out = (C.c_uint8 * PROOF_SCALE_BYTES)()
        n = C.c_size_t()
        _check(_bind().plk_proof_encode(C.byref(self.raw), out, PROOF_SCALE_BYTES, C.byref(n)),
               "Proof::encode")
        return bytes(out[: n.value])

    @staticmethod
    def from_bytes(data: bytes) -> "Proof":
        """``Proof::decode`` of :meth:`to_bytes` output; raises PlonkError(PLK_E_ARG) on a
        wrong length, a non-boolean infinity byte, non-canonical limbs or an off-curve point."""
        raw = PlkProof()
        buf = (C.c_uint8 * len(data)).from_buffer_copy(data) if data else None
        _check(_bind().plk_proof_decode(buf, len(data), C.byref(raw)), "Proof::decode")
        return Proof(raw)

    @staticmethod
    def from_words(comms, evals) -> "Proof":
        """A Proof from uint64 arrays: comms (11, 13) ABI points, evals (16, 4) Montgomery."""
        c = np.ascontiguousarray(comms, dtype=np.uint64).reshape(11, 13)
        e = np.ascontiguousarray(evals, dtype=np.uint64).reshape(16, 4)
        raw = PlkProof.from_buffer_copy(c.tobytes() + e.tobytes())
        return Proof(raw)

    def raw_bytes(self) -> bytes:
        """The in-memory plk_proof struct (104-byte ABI points, Montgomery limbs)."""
        return bytes(self.raw)

    def __eq__(self, other) -> bool:
        return isinstance(other, Proof) and self.raw_bytes() == other.raw_bytes()


class VerifierData:
    """What Verifier::new receives (verifier.rs:24-44): label, m, the 15 commitments in
    transcript order, public input indexes."""

    def __init__(self, label: bytes, n: int, m: int, comms: np.ndarray, pi_indexes):
        self.label, self.n, self.m, self.comms, self.pi_indexes = label, n, m, comms, pi_indexes


class Prover:
    def __init__(self, key_handle, n, m, label, pp):
        self._key, self.n, self.m, self.label, self.pp = key_handle, n, m, label, pp

    def create_proof(self, seed: int, circuit):
        cs = Plonk()
        circuit.synthesize(cs)
        return self.prove_composer(cs, seed)

    def prove_composer(self, cs: Plonk, seed: int):
        proof = PlkProof()
        pis = (PlkFr * 4096)()
        cnt = C.c_size_t()
        st = _bind().plk_prove(self._key, cs._h, seed, C.byref(proof), pis, 4096, C.byref(cnt))
        if st != PLK_OK:
            raise PlonkError(st, "create_proof")
        return Proof(proof), [fr_int(pis[i]) for i in range(cnt.value)]

    def lane(self) -> "ProverLane":
        """A concurrent prover over this key (plk_prover_create): own stream, MSM workspace
        and scratch; the key and the SRS window table are shared, not copied. Lanes may
        prove from different threads at once (``Prover: Clone`` in the reference)."""
        return ProverLane(self)

    def __del__(self):
        try:
            for ln in list(getattr(self, "_lanes", [])):
                ln.close()
            if self._key:
                _bind().plk_key_destroy(self._key)
        except Exception:
            pass


class ProverLane:
    """One plk_prover: create_proof on its own stream, sharing the key of `prover`."""

    def __init__(self, prover: Prover):
        self.prover = prover
        self._h = C.c_void_p()
        _check(_bind().plk_prover_create(prover._key, C.byref(self._h)), "plk_prover_create")
        if not hasattr(prover, "_lanes"):
            prover._lanes = []
        prover._lanes.append(self)
        self._shard_keep = None

    @property
    def stream(self) -> int:
        s = C.c_void_p()
        _check(_bind().plk_prover_stream(self._h, C.byref(s)), "plk_prover_stream")
        return s.value or 0

    def shard(self, slice_params, slice_start: int, rank: int, world: int, allgather,
              buckets: bool = False):
        """Split every commit of this lane's proofs over `world` ranks: by SRS slice
        (plk_prover_shard: `slice_params` is this rank's PlonkParams slice, PlonkParams.setup_range,
        starting at SRS index `slice_start`) or, with buckets=True, by bucket range on the key's
        own SRS (plk_prover_shard_buckets; slice_params / slice_start unused; PlonkError
        PLK_E_ARG where the key's SRS cannot be split `world` ways). `allgather(send: bytes) ->
        bytes` returns the concatenation of every rank's `send` in rank order."""
        def cb(_user, send, nbytes, recv):
            try:
                data = allgather(C.string_at(send, nbytes))
                if len(data) != world * nbytes:
                    return 1
                C.memmove(recv, data, len(data))
                return 0
            except Exception:  # noqa: BLE001 — reported to the prover as PLK_E_DEVICE
                import traceback
                traceback.print_exc()
                return 1
        fn = ALLGATHER_FN(cb)
        if buckets:
            _check(_bind().plk_prover_shard_buckets(self._h, rank, world, C.cast(fn, C.c_void_p),
                                                    None), "plk_prover_shard_buckets")
            self._shard_keep = (fn, None)  # keep the callback alive
            return
        self._shard_keep = (fn, slice_params)  # keep the callback and the slice alive
        _check(_bind().plk_prover_shard(self._h, slice_params._h if slice_params else None,
                                        slice_start, rank, world, C.cast(fn, C.c_void_p), None),
               "plk_prover_shard")

    def prove_composer(self, cs: Plonk, seed: int):
        proof = PlkProof()
        pis = (PlkFr * 4096)()
        cnt = C.c_size_t()
        st = _bind().plk_prover_prove(self._h, cs._h, seed, C.byref(proof), pis, 4096,
                                      C.byref(cnt))
        if st != PLK_OK:
            raise PlonkError(st, "create_proof")
        return Proof(proof), [fr_int(pis[i]) for i in range(cnt.value)]

    def create_proof(self, seed: int, circuit):
        cs = Plonk()
        circuit.synthesize(cs)
        return self.prove_composer(cs, seed)

    def msm_stats(self, reset: bool = False):
        """(k_accumulate ms, launches, point additions, MSM points) since the last reset."""
        ms, la, ad, pt = C.c_double(), C.c_uint64(), C.c_uint64(), C.c_uint64()
        _check(_bind().plk_prover_msm_stats(self._h, 1 if reset else 0, C.byref(ms),
                                            C.byref(la), C.byref(ad), C.byref(pt)),
               "plk_prover_msm_stats")
        return ms.value, la.value, ad.value, pt.value

    def close(self):
        if self._h:
            _bind().plk_prover_destroy(self._h)
            self._h = C.c_void_p()
            try:
                self.prover._lanes.remove(self)
            except (AttributeError, ValueError):
                pass

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class PlonkKey:
    @staticmethod
    def compile_with_circuit(pp: PlonkParams, label: bytes, circuit):
        cs = Plonk()
        circuit.synthesize(cs)
        return PlonkKey.compile_composer(pp, label, cs)

    @staticmethod
    def compile_composer(pp: PlonkParams, label: bytes, cs: Plonk):
        lib = _bind()
        h = C.c_void_p()
        _check(lib.plk_key_compile(pp._h, cs._h, label, C.byref(h)), "PlonkKey::compile")
        n, m = C.c_uint64(), C.c_uint64()
        comms = np.zeros((15, 13), dtype=np.uint64)
        _check(lib.plk_key_info(h, C.byref(n), C.byref(m), _ptr(comms)), "plk_key_info")
        _, idx = cs.public_inputs()
        prover = Prover(h, n.value, m.value, label, pp)
        return prover, VerifierData(label, n.value, m.value, comms, idx)
