"""PLONK verifier restated in Python — TEST INFRASTRUCTURE (the acceptance check for proofs
produced on the GPU; the verifier is out of scope for the device).

Follows /root/reference/src/verifier.rs:46-81 and src/prover/proof.rs:70-591: transcript
replay, Z_H(z), L1(z), barycentric PI(z), t_eval, [t] and [r] commitments, the two
aggregate proofs flattened with the v challenges, and commitment_scheme.rs:24-66's batch
check. The only deviation: the final pairing equation
    e(-W, [tau]H) * e(C, H) == 1
is checked as C == tau * W in G1 with the SRS trapdoor tau, which the tests know (by
bilinearity the two are equivalent); no pairing code is needed.
"""
from __future__ import annotations

import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "oracle"))
import pyref as P  # noqa: E402
from transcript import Transcript  # noqa: E402

r = P.R_MOD
K1, K2, K3 = 7, 13, 17


class VerificationError(Exception):
    pass


def pt(words):
    """uint64[13] ABI point -> affine (x, y) ints or None."""
    return P.g1_vec_from_np(words)[0]


def compress(p) -> bytes:
    """zkcrypto compressed G1 (48 B): BE x with compression/infinity/sort flags."""
    if p is None:
        return bytes([0xC0]) + bytes(47)
    x, y = p
    b = bytearray(x.to_bytes(48, "big"))
    b[0] |= 0x80
    if y > (P.P_MOD - 1) // 2:
        b[0] |= 0x20
    return bytes(b)


def append_scalar(t, label, s):
    t.append_message(label, (s % r).to_bytes(32, "little"))


def append_commitment(t, label, p):
    t.append_message(label, compress(p))


def challenge_scalar(t, label) -> int:
    return int.from_bytes(t.challenge_bytes(label, 64), "little") % r


SEED_LABELS = [b"q_m", b"q_l", b"q_r", b"q_o", b"q_c", b"q_4", b"q_arith", b"q_range",
               b"q_logic", b"q_fixed_group_add", b"q_variable_group_add",
               b"s_sigma_1", b"s_sigma_2", b"s_sigma_3", b"s_sigma_4"]


def base_transcript(vd):
    """Transcript::base(label, vk, constraints) (prover.rs:54-55, verifier.rs:33-34)."""
    t = Transcript(vd.label)
    t.append_message(b"dom-sep", b"circuit_size")
    t.append_u64(b"n", vd.m)
    for lab, c in zip(SEED_LABELS, vd.comms):
        append_commitment(t, lab, pt(c))
    return t


def gmul(p, s):
    return P.g1_mul(p, s % r)


def gsum(terms):
    acc = None
    for p, s in terms:
        acc = P.g1_add(acc, gmul(p, s))
    return acc


def verify(vd, proof, public_inputs, tau: int) -> None:
    if len(public_inputs) != len(vd.pi_indexes):
        raise VerificationError("InconsistentPublicInputsLen")  # verifier.rs:51-56
    t = base_transcript(vd)
    for v in public_inputs:
        append_scalar(t, b"pi", v)
    n = vd.n
    dense = [0] * n
    for idx, v in zip(vd.pi_indexes, public_inputs):
        dense[idx] = v
    C = {c: pt(getattr(proof, c)) for c in
         ("a_comm", "b_comm", "c_comm", "d_comm", "z_comm", "t_low_comm", "t_mid_comm",
          "t_high_comm", "t_4_comm", "w_z_chall_comm", "w_z_chall_w_comm")}
    append_commitment(t, b"a_w", C["a_comm"])
    append_commitment(t, b"b_w", C["b_comm"])
    append_commitment(t, b"c_w", C["c_comm"])
    append_commitment(t, b"d_w", C["d_comm"])
    beta = challenge_scalar(t, b"beta")
    append_scalar(t, b"beta", beta)
    gamma = challenge_scalar(t, b"gamma")
    append_commitment(t, b"z", C["z_comm"])
    alpha = challenge_scalar(t, b"alpha")
    range_sep = challenge_scalar(t, b"range separation challenge")
    logic_sep = challenge_scalar(t, b"logic separation challenge")
    fixed_sep = challenge_scalar(t, b"fixed base separation challenge")
    var_sep = challenge_scalar(t, b"variable base separation challenge")
    for lab, c in ((b"t_low", "t_low_comm"), (b"t_mid", "t_mid_comm"), (b"t_high", "t_high_comm"),
                   (b"t_4", "t_4_comm")):
        append_commitment(t, lab, C[c])
    z = challenge_scalar(t, b"z_challenge")

    e = proof
    omega = P.omega(n.bit_length() - 1)
    z_h = (pow(z, n, r) - 1) % r
    l1 = z_h * pow(n * (z - 1) % r, -1, r) % r
    # barycentric PI(z) (proof.rs:540-591)
    winv = pow(omega, -1, r)
    pi_eval = 0
    for i, v in enumerate(dense):
        if v:
            pi_eval += v * pow((pow(winv, i, r) * z - 1) % r, -1, r)
    pi_eval = pi_eval * z_h * pow(n, -1, r) % r
    # t_eval (proof.rs:386-440)
    a_term = (e.r_poly_eval + pi_eval) % r
    b0 = (e.a_eval + beta * e.s_sigma_1_eval + gamma) % r
    b1 = (e.b_eval + beta * e.s_sigma_2_eval + gamma) % r
    b2 = (e.c_eval + beta * e.s_sigma_3_eval + gamma) % r
    b3 = (e.d_eval + gamma) * e.perm_eval * alpha % r
    b_term = b0 * b1 * b2 * b3 % r
    c_term = l1 * alpha * alpha % r
    t_eval = (a_term - b_term - c_term) * pow(z_h, -1, r) % r
    # [t] = t_low + z^n t_mid + z^2n t_high + z^3n t_4 (proof.rs:442-455)
    zn = pow(z, n, r)
    t_comm = gsum([(C["t_low_comm"], 1), (C["t_mid_comm"], zn), (C["t_high_comm"], zn * zn),
                   (C["t_4_comm"], zn * zn * zn)])
    for lab, v in ((b"a_eval", e.a_eval), (b"b_eval", e.b_eval), (b"c_eval", e.c_eval),
                   (b"d_eval", e.d_eval), (b"a_next_eval", e.a_next_eval),
                   (b"b_next_eval", e.b_next_eval), (b"d_next_eval", e.d_next_eval),
                   (b"s_sigma_1_eval", e.s_sigma_1_eval), (b"s_sigma_2_eval", e.s_sigma_2_eval),
                   (b"s_sigma_3_eval", e.s_sigma_3_eval), (b"q_arith_eval", e.q_arith_eval),
                   (b"q_c_eval", e.q_c_eval), (b"q_l_eval", e.q_l_eval),
                   (b"q_r_eval", e.q_r_eval), (b"perm_eval", e.perm_eval),
                   (b"t_eval", t_eval), (b"r_eval", e.r_poly_eval)):
        append_scalar(t, lab, v)
    # [r] (proof.rs:459-527): arithmetic, range, permutation widgets (logic / curve selector
    # commitments are the identity for the circuits this backend accepts)
    vk = {lab.decode(): pt(c) for lab, c in zip(SEED_LABELS, vd.comms)}
    qa = e.q_arith_eval
    terms = [(vk["q_m"], e.a_eval * e.b_eval * qa), (vk["q_l"], e.a_eval * qa),
             (vk["q_r"], e.b_eval * qa), (vk["q_o"], e.c_eval * qa), (vk["q_4"], e.d_eval * qa),
             (vk["q_c"], qa)]
    if vk["q_range"] is not None:
        def delta(f):
            return f * (f - 1) * (f - 2) * (f - 3) % r
        kap = range_sep * range_sep % r
        rr = (delta(e.c_eval - 4 * e.d_eval) + delta(e.b_eval - 4 * e.c_eval) * kap
              + delta(e.a_eval - 4 * e.b_eval) * kap * kap
              + delta(e.d_next_eval - 4 * e.a_eval) * kap * kap * kap) % r
        terms.append((vk["q_range"], rr * range_sep))
    if vk["q_logic"] is not None:  # logic::linearize (dusk-plonk LogicGate; zksnarks)
        def delta(f):
            return f * (f - 1) * (f - 2) * (f - 3) % r
        k = logic_sep * logic_sep % r
        qa = (e.a_next_eval - 4 * e.a_eval) % r
        qb = (e.b_next_eval - 4 * e.b_eval) % r
        qd = (e.d_next_eval - 4 * e.d_eval) % r
        w = e.c_eval
        f = w * (w * (4 * w - 18 * (qa + qb) + 81) + 18 * (qa * qa + qb * qb)
                 - 81 * (qa + qb) + 83) % r
        xor_and = (3 * (qa + qb + qd) - 2 * f + e.q_c_eval * (9 * qd - 3 * (qa + qb))) % r
        lt = (delta(qa) + delta(qb) * k + delta(qd) * k ** 2 + (w - qa * qb) * k ** 3
              + xor_and * k ** 4) % r
        terms.append((vk["q_logic"], lt * logic_sep))
    ed = (-10240 * pow(10241, -1, r)) % r
    if vk["q_fixed_group_add"] is not None:  # curve_scalar::linearize (fixed base)
        k = fixed_sep * fixed_sep % r
        ax, axn, ay, ayn = e.a_eval, e.a_next_eval, e.b_eval, e.b_next_eval
        xya, acc, accn = e.c_eval, e.d_eval, e.d_next_eval
        xb, yb, xyb = e.q_l_eval, e.q_r_eval, e.q_c_eval
        bit = (accn - 2 * acc) % r
        ya = (bit * bit * (yb - 1) + 1) % r
        xa = xb * bit % r
        prod = xya * ax * ay * ed % r
        w = (bit * (bit - 1) * (bit + 1) + (bit * xyb - xya) * k
             + (axn + axn * prod - (ax * ya + ay * xa)) * k ** 2
             + (ayn - ayn * prod - (ay * ya + ax * xa)) * k ** 3) % r
        terms.append((vk["q_fixed_group_add"], w * fixed_sep))
    if vk["q_variable_group_add"] is not None:  # curve_addtion::linearize (variable base)
        k = var_sep * var_sep % r
        x1, x3, y1, y3 = e.a_eval, e.a_next_eval, e.b_eval, e.b_next_eval
        x2, y2, x1y2 = e.c_eval, e.d_eval, e.d_next_eval
        dp = ed * x1y2 * y1 * x2 % r
        w = ((x1 * y2 - x1y2) + (x1y2 + y1 * x2 - (x3 + x3 * dp)) * k
             + (y1 * y2 + x1 * x2 - (y3 - y3 * dp)) * k * k) % r
        terms.append((vk["q_variable_group_add"], w * var_sep))
    bz = beta * z % r
    x = ((e.a_eval + bz + gamma) * (e.b_eval + K1 * bz + gamma) * (e.c_eval + K2 * bz + gamma)
         * (e.d_eval + K3 * bz + gamma) * alpha) % r
    terms.append((C["z_comm"], x + l1 * alpha * alpha))
    y = -(b0 * b1 * b2 * beta * e.perm_eval * alpha) % r
    terms.append((vk["s_sigma_4"], y))
    r_comm = gsum(terms)
    # aggregate proofs flattened with v (commitment_scheme.rs:107-152)
    va = challenge_scalar(t, b"v_challenge")
    parts_a = [(t_eval, t_comm), (e.r_poly_eval, r_comm), (e.a_eval, C["a_comm"]),
               (e.b_eval, C["b_comm"]), (e.c_eval, C["c_comm"]), (e.d_eval, C["d_comm"]),
               (e.s_sigma_1_eval, vk["s_sigma_1"]), (e.s_sigma_2_eval, vk["s_sigma_2"]),
               (e.s_sigma_3_eval, vk["s_sigma_3"])]
    vb = challenge_scalar(t, b"v_challenge")
    parts_b = [(e.perm_eval, C["z_comm"]), (e.a_next_eval, C["a_comm"]),
               (e.b_next_eval, C["b_comm"]), (e.d_next_eval, C["d_comm"])]

    def flatten(parts, v):
        comm = gsum([(c, pow(v, i, r)) for i, (_, c) in enumerate(parts)])
        ev = sum(val * pow(v, i, r) for i, (val, _) in enumerate(parts)) % r
        return comm, ev

    fa = flatten(parts_a, va)
    fb = flatten(parts_b, vb)
    append_commitment(t, b"w_z", C["w_z_chall_comm"])
    append_commitment(t, b"w_z_w", C["w_z_chall_w_comm"])
    u = challenge_scalar(t, b"batch")
    points = [z, z * omega % r]
    total_c, total_w, g_mult = None, None, 0
    for k, ((comm, ev), w, point) in enumerate(zip((fa, fb), (C["w_z_chall_comm"],
                                                              C["w_z_chall_w_comm"]), points)):
        uk = pow(u, k, r)
        c = P.g1_add(comm, gmul(w, point))
        g_mult = (g_mult + uk * ev) % r
        total_c = P.g1_add(total_c, gmul(c, uk))
        total_w = P.g1_add(total_w, gmul(w, uk))
    total_c = P.g1_add(total_c, gmul(P.G1_GEN, -g_mult))
    # e(-total_w, [tau]H) e(total_c, H) == 1  <=>  total_c == tau * total_w
    if total_c != gmul(total_w, tau):
        raise VerificationError("ProofVerificationError (pairing check)")
