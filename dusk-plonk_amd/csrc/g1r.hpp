// g1r.hpp — the XYZZ group law of g1.hpp over the redundant-limb field (ffr.hpp), for the
// MSM's device stages. Same formulas (EFD g1p/shortw/xyzz madd-2008-s, add-2008-s,
// dbl-2008-s-1, mdbl-2008-s-1, a = 0) and the same exceptional-case handling; coordinates
// are R'-domain values in [0, 2p). Points travel through memory in the packed G1Affine /
// G1xyzz layouts of g1.hpp (R'-domain contents).
#pragma once
#include "ffr.hpp"
#include "g1.hpp"

namespace plk {

using RFp = Rx<FpCfg>;

struct G1R {
  RFp X, Y, ZZ, ZZZ;  // ZZ == 0 <=> infinity
};

__device__ __forceinline__ G1R g1r_infinity() {
  G1R r;
  r.X = rx_one<FpCfg>();
  r.Y = rx_one<FpCfg>();
  r.ZZ = rx_zero<FpCfg>();
  r.ZZZ = rx_zero<FpCfg>();
  return r;
}

__device__ __forceinline__ bool g1r_is_inf(const G1R& p) { return rx_is_zero(p.ZZ); }

__device__ __forceinline__ G1R g1r_neg(const G1R& p) {
  G1R r = p;
  r.Y = rx_neg(p.Y);
  return r;
}

__device__ __forceinline__ G1R g1r_dbl(const G1R& p) {
  if (g1r_is_inf(p)) return p;
  const RFp U = rx_dbl(p.Y);
  const RFp V = rx_sqr(U);
  const RFp W = rx_mul(U, V);
  const RFp S = rx_mul(p.X, V);
  const RFp X2 = rx_sqr(p.X);
  const RFp M = rx_add(rx_dbl(X2), X2);
  G1R r;
  r.X = rx_sub(rx_sqr(M), rx_dbl(S));
  r.Y = rx_sub(rx_mul(M, rx_sub(S, r.X)), rx_mul(W, p.Y));
  r.ZZ = rx_mul(V, p.ZZ);
  r.ZZZ = rx_mul(W, p.ZZZ);
  return r;
}

__device__ __forceinline__ G1R g1r_dbl_affine(const RFp& x, const RFp& y) {
  const RFp U = rx_dbl(y);
  const RFp V = rx_sqr(U);
  const RFp W = rx_mul(U, V);
  const RFp S = rx_mul(x, V);
  const RFp X2 = rx_sqr(x);
  const RFp M = rx_add(rx_dbl(X2), X2);
  G1R r;
  r.X = rx_sub(rx_sqr(M), rx_dbl(S));
  r.Y = rx_sub(rx_mul(M, rx_sub(S, r.X)), rx_mul(W, y));
  r.ZZ = V;
  r.ZZZ = W;
  return r;
}

// p + (x2, y2), the affine operand never infinity
__device__ __forceinline__ G1R g1r_add_affine(const G1R& p, const RFp& x2, const RFp& y2) {
  if (g1r_is_inf(p)) {
    G1R r;
    r.X = x2;
    r.Y = y2;
    r.ZZ = rx_one<FpCfg>();
    r.ZZZ = rx_one<FpCfg>();
    return r;
  }
  const RFp U2 = rx_mul(x2, p.ZZ);
  const RFp S2 = rx_mul(y2, p.ZZZ);
  const RFp P = rx_sub(U2, p.X);
  const RFp R = rx_sub(S2, p.Y);
  if (rx_is_zero(P)) {
    if (rx_is_zero(R)) return g1r_dbl_affine(x2, y2);
    return g1r_infinity();
  }
  const RFp PP = rx_sqr(P);
  const RFp PPP = rx_mul(P, PP);
  const RFp Q = rx_mul(p.X, PP);
  G1R r;
  r.X = rx_sub(rx_sub(rx_sqr(R), PPP), rx_dbl(Q));
  r.Y = rx_sub(rx_mul(R, rx_sub(Q, r.X)), rx_mul(p.Y, PPP));
  r.ZZ = rx_mul(p.ZZ, PP);
  r.ZZZ = rx_mul(p.ZZZ, PPP);
  return r;
}

__device__ __forceinline__ G1R g1r_add(const G1R& p, const G1R& q) {
  if (g1r_is_inf(p)) return q;
  if (g1r_is_inf(q)) return p;
  const RFp U1 = rx_mul(p.X, q.ZZ);
  const RFp U2 = rx_mul(q.X, p.ZZ);
  const RFp S1 = rx_mul(p.Y, q.ZZZ);
  const RFp S2 = rx_mul(q.Y, p.ZZZ);
  const RFp P = rx_sub(U2, U1);
  const RFp R = rx_sub(S2, S1);
  if (rx_is_zero(P)) {
    if (rx_is_zero(R)) return g1r_dbl(p);
    return g1r_infinity();
  }
  const RFp PP = rx_sqr(P);
  const RFp PPP = rx_mul(P, PP);
  const RFp Q = rx_mul(U1, PP);
  G1R r;
  r.X = rx_sub(rx_sub(rx_sqr(R), PPP), rx_dbl(Q));
  r.Y = rx_sub(rx_mul(R, rx_sub(Q, r.X)), rx_mul(S1, PPP));
  r.ZZ = rx_mul(rx_mul(p.ZZ, q.ZZ), PP);
  r.ZZZ = rx_mul(rx_mul(p.ZZZ, q.ZZZ), PPP);
  return r;
}

// ---- lazy mixed addition for the bucket accumulation (k_accumulate) ----------------
// Same formulas as g1r_add_affine with the normalisation deferred. Accumulator invariant:
// X in (0, 8p), Y in (0, 4p), ZZ, ZZZ in [0, 2p), all limbs normalised; g1r_lazy_finish
// brings X, Y back to [0, 2p). The affine y may be an unnormalised value < 4p (a lazy
// negation 4p - y). Of the seven add/sub passes of the plain formula (~125 instructions
// each) the four that feed multiplications are limb-wise (28) and X3 = R^2 - PPP - 2Q is
// one signed-carry pass.
//
// g1r_madd_lazy_sl is straight-line: no exceptional-case branch. A branch in the middle
// of the formula cost ~800 instructions per addition (the backend's per-block lowering
// then treats operands crossing it as 64-bit: +260 mads, +540 v_mov), so the cases are
// repaired AFTER, from the result alone:
//   * accumulator at infinity (ZZ1 = 0): ZZ3 = ZZ1 * PP = 0;
//   * P == 0 (same x): ZZ3 = ZZ1 * P^2 == 0, and then X3 = R^2 + 6p, so R == 0 (same
//     point: the sum is a doubling) <=> X3 == 0 mod p; otherwise the sum is infinity.
// A zero ZZ3 is the single (rare) trigger; g1r_madd_lazy_fix finishes those cases.
// GROUPED: the nine reductions as independent groups whose chains interleave (ffr.hpp
// rx_prod_group): (U2, S2), (PP, R^2), (PPP, Q), (Y3, ZZ3, ZZZ3) — 4 346 VALU + ~440 s_nop per
// addition; at 2 waves per SIMD (prover lanes) 6.83-6.90e9 solo additions/s in the 2^20 proof
// against 6.57-6.60e9 for the plain chains at 3 waves (round 5, profiles/r05_acc_dma_ab.jsonl).
// Otherwise one product at a time (4 536 VALU, no s_nop, ~30 fewer VGPRs): at 3 waves per SIMD
// it is the faster form where the chip is otherwise idle (lone 2^20 MSM 2.84-2.85 against
// 2.92 ms). Measured and dropped in round 5: (PPP, Q, ZZ3) + (Y3, ZZZ3) (round 4's libplk-g2)
// and (PPP, ZZ3) + (Q, ZZZ3) + Y3 alone, both spilling at 3 waves.
// ASM (round 6, k_accumulate's lane form): the groups' columns as single asm statements
// (ffr.hpp RxAsmText): ~4 505 instructions and ~72 s_nop per loop iteration instead of ~4 865 /
// ~430. PAIRS (with ASM): Y3 as a plain product and (ZZ3, ZZZ3) as a pair instead of the
// triple group: 168 VGPRs, so it fits 3 waves per SIMD without spilling (k_accumulate's lone
// form since round 6; the plain chains below are the formula as one product at a time, the
// lone form before).
template <bool GROUPED, bool ASM = false, bool PAIRS = false>
__device__ __forceinline__ G1R g1r_madd_lazy_sl(const G1R& p, const RFp& x2, const RFp& y2) {
  if constexpr (GROUPED && PAIRS) {
    RFp U2, S2, PP, RR, PPP, Q;
    rx_mul2<FpCfg, ASM>(x2, p.ZZ, y2, p.ZZZ, U2, S2);
    const RFp P = rx_sub_u<FpCfg, 10>(U2, p.X);
    const RFp R = rx_sub_u<FpCfg, 6>(S2, p.Y);
    rx_sqr2<FpCfg, ASM>(P, R, PP, RR);
    G1R r;
    rx_mul2<FpCfg, ASM>(P, PP, p.X, PP, PPP, Q);
    r.X = rx_sub2_n<FpCfg, 6>(RR, PPP, Q);
    r.Y = rx_mul_add(R, rx_sub_u<FpCfg, 10>(Q, r.X), rx_sub_u<FpCfg, 5>(rx_zero<FpCfg>(), p.Y), PPP);
    rx_mul2<FpCfg, ASM>(p.ZZ, PP, p.ZZZ, PPP, r.ZZ, r.ZZZ);
    return r;
  } else if constexpr (GROUPED) {
    RFp U2, S2, PP, RR, PPP, Q;
    rx_mul2<FpCfg, ASM>(x2, p.ZZ, y2, p.ZZZ, U2, S2);
    const RFp P = rx_sub_u<FpCfg, 10>(U2, p.X);
    const RFp R = rx_sub_u<FpCfg, 6>(S2, p.Y);
    rx_sqr2<FpCfg, ASM>(P, R, PP, RR);
    G1R r;
    rx_mul2<FpCfg, ASM>(P, PP, p.X, PP, PPP, Q);
    r.X = rx_sub2_n<FpCfg, 6>(RR, PPP, Q);
    rx_mul_add_mul2<FpCfg, ASM>(R, rx_sub_u<FpCfg, 10>(Q, r.X), rx_sub_u<FpCfg, 5>(rx_zero<FpCfg>(), p.Y), PPP,
                    p.ZZ, PP, p.ZZZ, PPP, r.Y, r.ZZ, r.ZZZ);
    return r;
  } else {
    const RFp U2 = rx_mul(x2, p.ZZ);
    const RFp S2 = rx_mul(y2, p.ZZZ);
    const RFp P = rx_sub_u<FpCfg, 10>(U2, p.X);  // (2p, 12p): U2 - X1 in (-8p, 2p)
    const RFp R = rx_sub_u<FpCfg, 6>(S2, p.Y);   // (2p, 8p): S2 - Y1 in (-4p, 2p)
    const RFp PP = rx_sqr(P);
    const RFp PPP = rx_mul(P, PP);
    const RFp Q = rx_mul(p.X, PP);
    G1R r;
    r.X = rx_sub2_n<FpCfg, 6>(rx_sqr(R), PPP, Q);  // R^2 + 6p - PPP - 2Q in (0, 8p)
    // Y3 = R (Q - X3) + (5p - Y1) PPP with one reduction (all operands normalised, the
    // split columns of rx_mul_add keep each accumulator below 2^64); value
    // (8p * 12p + 5p * 2p) / R' + p < 2p at R' = 2^390
    r.Y = rx_mul_add(R, rx_sub_u<FpCfg, 10>(Q, r.X), rx_sub_u<FpCfg, 5>(rx_zero<FpCfg>(), p.Y), PPP);
    r.ZZ = rx_mul(p.ZZ, PP);
    r.ZZZ = rx_mul(p.ZZZ, PPP);
    return r;
  }
}

// The result of p + (x2, y2) when g1r_madd_lazy_sl returned r with r.ZZ == 0; was_inf =
// p was the point at infinity. (x2, y2): the affine point, y2 normalised in [0, 2p).
__device__ __forceinline__ G1R g1r_madd_lazy_fix(bool was_inf, const G1R& r, const RFp& x2,
                                                 const RFp& y2) {
  if (was_inf) {
    G1R q;
    q.X = x2;
    q.Y = y2;
    q.ZZ = rx_one<FpCfg>();
    q.ZZZ = rx_one<FpCfg>();
    return q;
  }
  if (rx_is_zero_u(r.X)) return g1r_dbl_affine(x2, y2);
  return g1r_infinity();
}

// both halves, for callers that keep (x2, y2) live (y2 may be the lazy negation)
__device__ __forceinline__ G1R g1r_madd_lazy(const G1R& p, const RFp& x2, const RFp& y2) {
  const bool was_inf = g1r_is_inf(p);
  G1R r = g1r_madd_lazy_sl<true>(p, x2, y2);
  if (rx_is_zero(r.ZZ)) r = g1r_madd_lazy_fix(was_inf, r, x2, rx_canon(y2));
  return r;
}

// 4p - y (normalised for the split Fp shape, rx_sub_u): the negated affine y for
// g1r_madd_lazy
__device__ __forceinline__ RFp rx_neg_lazy(const RFp& y) { return rx_sub_u<FpCfg, 4>(rx_zero<FpCfg>(), y); }

__device__ __forceinline__ G1R g1r_lazy_finish(const G1R& p) {
  G1R r = p;
  r.X = rx_canon(p.X);
  r.Y = rx_canon(p.Y);
  return r;
}

// ---- lazy full addition (both operands XYZZ), for the run-sum bucket reduction --------
// add-2008-s with the normalisation deferred as in g1r_madd_lazy_sl. Operands: X in [0, 8p),
// Y in [0, 4p), ZZ, ZZZ in [0, 2p), normalised limbs (g1r_lazy_finish outputs, g1r_infinity,
// or results of this function); the result satisfies the same. Straight-line; the
// exceptional cases (either operand at infinity, equal x) all give ZZ3 = ZZ1 ZZ2 P^2 = 0 and
// are repaired after, by g1r_add_lazy.
__device__ __forceinline__ G1R g1r_add_lazy_sl(const G1R& p, const G1R& q) {
  // interleaved groups (ffr.hpp rx_prod_group): (U1, U2, ZZ1 ZZ2), (S1, S2, ZZZ1 ZZZ2),
  // (PP, R^2), (PPP, Q), (Y3, ZZ3, ZZZ3)
  RFp U1, U2, ZZ12, S1, S2, ZZZ12, PP, RR, PPP, Q;
  rx_mul3(p.X, q.ZZ, q.X, p.ZZ, p.ZZ, q.ZZ, U1, U2, ZZ12);
  const RFp P = rx_sub_u<FpCfg, 3>(U2, U1);  // U2 - U1 + 3p in (p, 5p)
  rx_mul3(p.Y, q.ZZZ, q.Y, p.ZZZ, p.ZZZ, q.ZZZ, S1, S2, ZZZ12);
  const RFp R = rx_sub_u<FpCfg, 3>(S2, S1);  // S2 - S1 + 3p in (p, 5p)
  rx_sqr2(P, R, PP, RR);
  rx_mul2(P, PP, U1, PP, PPP, Q);
  G1R r;
  r.X = rx_sub2_n<FpCfg, 6>(RR, PPP, Q);  // R^2 + 6p - PPP - 2Q in (0, 8p)
  rx_mul_add_mul2(R, rx_sub_u<FpCfg, 10>(Q, r.X), rx_sub_u<FpCfg, 5>(rx_zero<FpCfg>(), S1), PPP,
                  ZZ12, PP, ZZZ12, PPP, r.Y, r.ZZ, r.ZZZ);
  return r;
}

// dbl-2008-s-1 on a lazy operand (X < 8p, Y < 4p, ZZ, ZZZ < 2p; normalised limbs) with the
// lazy normalisation of g1r_madd_lazy_sl: result X3 in (2p, 8p), Y3 < 2p. Infinity (ZZ = 0)
// stays infinity (ZZ3 = V ZZ); G1 has no 2-torsion, so Y != 0 otherwise.
__device__ __forceinline__ G1R g1r_dbl_lazy(const G1R& p) {
  const RFp U = rx_small_mul_n<FpCfg, 2>(p.Y);  // 2Y < 8p, normalised
  const RFp V = rx_sqr(U);
  const RFp W = rx_mul(U, V);
  const RFp S = rx_mul(p.X, V);
  const RFp X2 = rx_sqr(p.X);
  const RFp M = rx_small_mul_n<FpCfg, 3>(X2);  // 3X^2 < 6p, normalised
  G1R r;
  r.X = rx_sub2_n<FpCfg, 6>(rx_sqr(M), rx_zero<FpCfg>(), S);  // M^2 + 6p - 2S in (2p, 8p)
  // Y3 = M (S - X3) - W Y = M (S - X3 + 10p) + (5p - Y) W, one reduction (value
  // (6p * 12p + 5p * 2p) / R' + p < 2p)
  r.Y = rx_mul_add(M, rx_sub_u<FpCfg, 10>(S, r.X), rx_sub_u<FpCfg, 5>(rx_zero<FpCfg>(), p.Y), W);
  r.ZZ = rx_mul(V, p.ZZ);
  r.ZZZ = rx_mul(W, p.ZZZ);
  return r;
}

// The rare path's arithmetic is made to depend on an opaque zero defined here: without it
// LLVM speculates the doubling (~3 300 mads) above the branch and selects its result,
// paying it on every addition.
__device__ __forceinline__ G1R g1r_add_lazy_fix(const G1R& p, const G1R& q, const RFp& x3) {
  if (g1r_is_inf(p)) return q;
  if (g1r_is_inf(q)) return p;
  uint32_t z = 0;
  __asm__ volatile(";; plk rare path" : "+v"(z));
  RFp x = x3;
  x.v[0] += z;
  if (rx_is_zero_u(x)) {
    G1R d = p;
    d.X.v[0] += z;
    d.Y.v[0] += z;
    return g1r_dbl_lazy(d);
  }
  return g1r_infinity();
}

__device__ __forceinline__ G1R g1r_add_lazy(const G1R& p, const G1R& q) {
  const G1R r = g1r_add_lazy_sl(p, q);
  return rx_is_zero(r.ZZ) ? g1r_add_lazy_fix(p, q, r.X) : r;  // rare branch
}

// ---- quad-cooperative lazy full addition, for the latency-bound reduction tails -------
// One addition per quad (4 consecutive lanes holding the same p and q; the result comes
// back in all four). A lone wave's addition is issue-bound: g1r_add_lazy_sl issues ~15
// Montgomery products one after another. Here the quad's lanes take one product each in
// the same instruction stream, four levels of the formula's dependency graph:
//   1: U1 = X1 ZZ2, U2 = X2 ZZ1, S1 = Y1 ZZZ2, S2 = Y2 ZZZ1
//   2: PP = P^2, RR = R^2, ZZ1 ZZ2, ZZZ1 ZZZ2       (P = U2 - U1, R = S2 - S1)
//   3: PPP = P PP, Q = U1 PP, ZZ3 = ZZ1 ZZ2 PP
//   4: Y3 = R (Q - X3) + (5p - S1) PPP, ZZZ3 = ZZZ1 ZZZ2 PPP   (one fused form, c d = 0 on
//      the ZZZ3 lane)
// and the lanes swap results through DPP quad broadcasts: ~3.5 products issued instead of ~15.
// Same formulas and bounds as g1r_add_lazy_sl (each lane selects its level's operands from the
// same values); squares run as products. The quad must be active as a whole (control flow
// uniform per quad). Measured (profiles/r04_tail_quad_ab.jsonl): lone MSMs 2^16 0.82 -> 0.68 ms,
// 2^20 3.30 -> 3.01-3.10 ms; 2^12 proofs +8-15 %; proofs at 2^16 / 2^20, where other lanes'
// kernels fill the chip, ~1 % slower (more issue slots per addition): prover lanes above
// 2^13 keep single-lane trees, with quads in k_bitsum2 alone at 2^14 and from 2^19
// (msm_common.hpp tail_quad, prover.hip plk_prover_create).
template <int K>
__device__ __forceinline__ RFp quad_bcast(const RFp& v) {
  RFp r;
#pragma unroll
  for (int i = 0; i < RxShape<FpCfg>::L; ++i)
    r.v[i] = (uint32_t)__builtin_amdgcn_mov_dpp((int)v.v[i], K | (K << 2) | (K << 4) | (K << 6), 0xF,
                                                0xF, false);
  return r;
}

__device__ __forceinline__ RFp quad_sel(uint32_t l, const RFp& a0, const RFp& a1, const RFp& a2,
                                        const RFp& a3) {
  RFp r;
#pragma unroll
  for (int i = 0; i < RxShape<FpCfg>::L; ++i)
    r.v[i] = l < 2 ? (l == 0 ? a0.v[i] : a1.v[i]) : (l == 2 ? a2.v[i] : a3.v[i]);
  return r;
}

// Operands as for g1r_add_lazy. Infinity operands return early (uniform per quad); the
// equal-x case is repaired from (U1, S1, ZZ1 ZZ2, ZZZ1 ZZZ2), which represents p itself
// (p scaled by ZZ2: U1 / ZZ12 = X1 / ZZ1, S1 / ZZZ12 = Y1 / ZZZ1), so neither operand stays
// live past level 2.
__device__ __forceinline__ G1R g1r_add_quad(const G1R& p, const G1R& q, uint32_t l) {
  if (g1r_is_inf(q)) return p;
  if (g1r_is_inf(p)) return q;
  RFp M = rx_mul(quad_sel(l, p.X, q.X, p.Y, q.Y), quad_sel(l, q.ZZ, p.ZZ, q.ZZZ, p.ZZZ));
  const RFp U1 = quad_bcast<0>(M), S1 = quad_bcast<2>(M);
  const RFp P = rx_sub_u<FpCfg, 3>(quad_bcast<1>(M), U1);  // U2 - U1 + 3p in (p, 5p)
  const RFp R = rx_sub_u<FpCfg, 3>(quad_bcast<3>(M), S1);  // S2 - S1 + 3p in (p, 5p)
  M = rx_mul(quad_sel(l, P, R, p.ZZ, p.ZZZ), quad_sel(l, P, R, q.ZZ, q.ZZZ));
  const RFp PP = quad_bcast<0>(M), RR = quad_bcast<1>(M), ZZ12 = quad_bcast<2>(M),
            ZZZ12 = quad_bcast<3>(M);
  M = rx_mul(quad_sel(l, P, U1, ZZ12, ZZ12), PP);
  const RFp PPP = quad_bcast<0>(M), Q = quad_bcast<1>(M);
  G1R r;
  r.ZZ = quad_bcast<2>(M);
  r.X = rx_sub2_n<FpCfg, 6>(RR, PPP, Q);  // R^2 + 6p - PPP - 2Q in (0, 8p)
  if (rx_is_zero(r.ZZ)) {  // P = 0 (rare): the doubling of p if R = 0 (then X3 = R^2 + 6p), else infinity
    uint32_t z = 0;
    __asm__ volatile(";; plk rare path" : "+v"(z));  // as in g1r_add_lazy_fix
    RFp x = r.X;
    x.v[0] += z;
    if (!rx_is_zero_u(x)) return g1r_infinity();
    G1R d;
    d.X = U1;
    d.Y = S1;
    d.ZZ = ZZ12;
    d.ZZZ = ZZZ12;
    d.X.v[0] += z;
    return g1r_dbl_lazy(d);
  }
  const RFp qx = rx_sub_u<FpCfg, 10>(Q, r.X), cd = rx_sub_u<FpCfg, 5>(rx_zero<FpCfg>(), S1);
  const RFp z = rx_zero<FpCfg>();
  M = rx_mul_add(quad_sel(l, R, ZZZ12, R, ZZZ12), quad_sel(l, qx, PPP, qx, PPP),
                 quad_sel(l, cd, z, cd, z), PPP);
  r.Y = quad_bcast<0>(M);
  r.ZZZ = quad_bcast<1>(M);
  return r;
}

// ---- packed memory <-> limbs (16-byte loads/stores of the 48-byte coordinates) -------
__device__ __forceinline__ RFp ld_rfp(const uint32_t* p) {
  const uint4* q = reinterpret_cast<const uint4*>(p);
  Fp x;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const uint4 a = q[i];
    x.v[4 * i] = a.x;
    x.v[4 * i + 1] = a.y;
    x.v[4 * i + 2] = a.z;
    x.v[4 * i + 3] = a.w;
  }
  return rx_unpack(x);
}

__device__ __forceinline__ void st_rfp(uint32_t* p, const RFp& r) {
  const Fp x = rx_pack(r);
  uint4* q = reinterpret_cast<uint4*>(p);
#pragma unroll
  for (int i = 0; i < 3; ++i)
    q[i] = make_uint4(x.v[4 * i], x.v[4 * i + 1], x.v[4 * i + 2], x.v[4 * i + 3]);
}

__device__ __forceinline__ void ld_g1r_aff(const G1Affine* p, RFp& x, RFp& y) {
  x = ld_rfp(reinterpret_cast<const uint32_t*>(p));
  y = ld_rfp(reinterpret_cast<const uint32_t*>(p) + 12);
}

__device__ __forceinline__ G1R ld_g1r(const G1xyzz* p) {
  const uint32_t* q = reinterpret_cast<const uint32_t*>(p);
  G1R r;
  r.X = ld_rfp(q);
  r.Y = ld_rfp(q + 12);
  r.ZZ = ld_rfp(q + 24);
  r.ZZZ = ld_rfp(q + 36);
  return r;
}

__device__ __forceinline__ void st_g1r(G1xyzz* p, const G1R& r) {
  uint32_t* q = reinterpret_cast<uint32_t*>(p);
  st_rfp(q, r.X);
  st_rfp(q + 12, r.Y);
  st_rfp(q + 24, r.ZZ);
  st_rfp(q + 36, r.ZZZ);
}

}  // namespace plk
