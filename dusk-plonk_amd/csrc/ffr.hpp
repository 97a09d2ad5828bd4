// ffr.hpp — redundant-limb Montgomery arithmetic for the gfx950 hot loops (device only).
//
// ff.hpp stores a field element as N packed 32-bit words and multiplies with a 96-bit
// column accumulator: every 32x32 partial product costs v_mad_u64_u32 + v_addc (plus the
// s_nop padding the compiler puts around inline asm). Here an element is L limbs of B < 32
// bits (Fp: 13 x 30, Fr: 9 x 29) so that each partial product is ONE v_mad_u64_u32 into a
// 64-bit column accumulator, no carry chain, plain C the scheduler can interleave.
// Fr (9 x 29): a whole product-scanning column — at most 2L products below 2^(2B) plus the
// incoming carry — fits one accumulator. Fp (round 3: 13 x 30 instead of 14 x 28, 169 + 169
// mads per product instead of 196 + 196): the middle columns' worst-case sums reach 2^64, so
// those columns (RxPlan, computed at compile time from the limb bounds) keep the products and
// the Montgomery reduction terms in separate accumulators and merge their low B bits and
// carries — a few instructions per split column.
// Measured on MI355X (tools/ubench_limbs.hip): Fp 13 x 30 7.86e10 mul/s vs 6.75e10 at
// 14 x 28 and 4.8e10 packed; Fr 1.69e11 vs 1.09e11.
//
// Domain: Montgomery with R' = 2^(B*L) (Fp 2^390, Fr 2^261), values kept in [0, 2p) with
// normalised limbs (4p < R', so the product needs no final subtraction). Memory keeps the
// packed layout of ff.hpp (2p < 2^(32N)): kernels unpack on load and pack on store, and a
// buffer holds either R-domain (ff.hpp) or R'-domain values — each buffer's comment says
// which. Conversion R -> R' is a multiplication by 2^(B*L - 32N) (doublings); R' -> R by
// 2^-(B*L - 32N).
#pragma once
#include <type_traits>
#include <utility>

#include "ff.hpp"

namespace plk {

template <class C>
struct RxShape;
template <>
struct RxShape<FpCfg> {
  static constexpr int L = 13, B = 30;
  static constexpr uint32_t ONE[12] = {0x00d1ff2eu, 0x46760000u, 0x9b4800acu, 0x84b80337u,
                                       0xe882431cu, 0x0dd9a7e0u, 0xb683dcf8u, 0xc26c26d0u,
                                       0x63c4a5eeu, 0x29f14576u, 0x7f3e804bu, 0x015de996u};  // 2^390 mod p
};
template <>
struct RxShape<FrCfg> {
  static constexpr int L = 9, B = 29;
  static constexpr uint32_t ONE[8] = {0xffffffbau, 0x00000045u, 0x0072d846u, 0x1a25272eu,
                                      0x5dbeee8bu, 0xfe2eedcdu, 0x9eefbe41u, 0x4d043f42u};  // 2^261 mod r
};

template <class C>
struct Rx {
  uint32_t v[RxShape<C>::L];
};

template <class C>
struct RxConst {
  static constexpr int L = RxShape<C>::L, B = RxShape<C>::B;
  uint32_t p[L], p2[L], one[L];
  uint32_t inv;  // -p^-1 mod 2^B
};

// limb i (bits [B*i, B*i + B), the last limb takes everything above) of a packed value
constexpr uint32_t rx_limb_of(const uint32_t* w, int nwords, int i, int B, int L) {
  uint32_t x = 0;
  const int width = (i == L - 1) ? 32 : B;
  for (int k = 0; k < width; ++k) {
    const int bit = i * B + k;
    if (bit < 32 * nwords && ((w[bit / 32] >> (bit % 32)) & 1u)) x |= 1u << k;
  }
  return x;
}

template <class C>
constexpr RxConst<C> rx_make() {
  constexpr int L = RxShape<C>::L, B = RxShape<C>::B, N = C::N;
  RxConst<C> k{};
  uint32_t p2w[N] = {};
  uint32_t carry = 0;
  for (int i = 0; i < N; ++i) {
    p2w[i] = (C::P[i] << 1) | carry;
    carry = C::P[i] >> 31;
  }
  for (int i = 0; i < L; ++i) {
    k.p[i] = rx_limb_of(C::P, N, i, B, L);
    k.p2[i] = rx_limb_of(p2w, N, i, B, L);
    k.one[i] = rx_limb_of(RxShape<C>::ONE, N, i, B, L);
  }
  uint32_t y = 1;
  for (int it = 0; it < 6; ++it) y = y * (2u - C::P[0] * y);
  k.inv = (0u - y) & ((1u << B) - 1);
  return k;
}

template <class C>
struct RxK {
  static constexpr RxConst<C> k = rx_make<C>();
};

// Split-column plan of a Montgomery product with NPROD operand products (1: a*b or a^2,
// 2: a*b + c*d) for shapes whose columns can overflow 64 bits (B >= 30). Operand limbs are
// normalised (< 2^B) with a top limb below 2^(TOP_BITS) (values below 2^(B(L-1) + TOP_BITS)
// = 2^386 for Fp): the group-law operands stay below 12p (~2^384.3; rx_sub_u<10> of two
// values < 2p is the largest), checked by the static_assert below the plan; the products'
// output bound a b / R' + p < 2p also needs a b < 630 p^2 at R' = 2^390. split[k]: the worst-case sum
// of column k (incoming carry + products + reduction terms m_i p_j) reaches 2^64, so the
// products and the reduction terms (and for NPROD = 2 each product set) use separate
// accumulators there. Every separate accumulator holds at most L products below 2^60 plus
// the carry: below 2^64.
template <class C>
struct RxSplitOn {
  static constexpr bool value = RxShape<C>::B >= 30;
};

template <class C, int NPROD>
struct RxPlan {
  static constexpr int L = RxShape<C>::L, B = RxShape<C>::B;
  static constexpr int TOP_BITS = 26;
  bool split[2 * L - 1];
  constexpr RxPlan() : split{} {
    constexpr RxConst<C> K = RxK<C>::k;
    long double carry = 0;
    for (int k = 0; k < 2 * L - 1; ++k) {
      long double sum = carry;
      for (int i = 0; i < L; ++i) {
        const int j = k - i;
        if (j < 0 || j >= L) continue;
        const long double ai = (long double)(1ull << (i == L - 1 ? TOP_BITS : B));
        const long double bj = (long double)(1ull << (j == L - 1 ? TOP_BITS : B));
        sum += NPROD * ai * bj + (long double)(1ull << B) * (long double)(K.p[j] + 1);
      }
      // 2^64. The sum is exact in long double on the host and rounded in the device pass
      // (long double is double there): the closest unsplit column sits at 0.993 x 2^64, far
      // outside double's 2^-52 relative error, so both passes give the same plan
      split[k] = sum >= 18446744073709551616.0L;
      carry = sum / (long double)(1ull << B) + 4;
    }
  }
};
template <class C, int NPROD>
struct RxPlanK {
  static constexpr RxPlan<C, NPROD> k{};
};
// (defined below) the limbs of c*p
// c*p as L limbs (c < 16). borrow_free: every limb below the top raised by 2^B - 1 (2^B for
// limb 0) by borrowing from the limb above, so limbs 0..L-2 lie in [2^B - 1, 2^(B+1) - 1):
// a_i + q_i - b_i >= 0 limb by limb for any normalised b whose top limb is below q's.
template <class C>
struct RxMultiple {
  uint32_t v[RxShape<C>::L];
};

template <class C>
constexpr RxMultiple<C> rx_multiple(uint32_t c, bool borrow_free) {
  constexpr int L = RxShape<C>::L, B = RxShape<C>::B, N = C::N;
  uint32_t w[N + 1] = {};
  uint64_t carry = 0;
  for (int i = 0; i < N; ++i) {
    const uint64_t t = (uint64_t)C::P[i] * c + carry;
    w[i] = (uint32_t)t;
    carry = t >> 32;
  }
  w[N] = (uint32_t)carry;
  RxMultiple<C> m{};
  for (int i = 0; i < L; ++i) m.v[i] = rx_limb_of(w, N + 1, i, B, L);
  if (borrow_free) {
    m.v[0] += 1u << B;
    for (int i = 1; i < L - 1; ++i) m.v[i] += (1u << B) - 1;
    m.v[L - 1] -= 1;
  }
  return m;
}

template <class C, uint32_t CP, bool BF>
struct RxMultipleK {
  static constexpr RxMultiple<C> k = rx_multiple<C>(CP, BF);
};
// The split plan's operand bound: the largest group-law multiplicand (below 12p, e.g.
// rx_sub_u<10>(a, b) with a < 2p) must keep its top limb below 2^TOP_BITS, or a column the plan
// leaves unsplit could reach 2^64. A looser operand bound must update TOP_BITS (and the plan).
static_assert(RxMultiple<FpCfg>{rx_multiple<FpCfg>(12, false)}.v[RxShape<FpCfg>::L - 1] <
                  (1u << RxPlan<FpCfg, 1>::TOP_BITS),
              "12p exceeds the split plan's operand bound");

#define PLK_RX __device__ __forceinline__

// acc += x * y as ONE v_mad_u64_u32 on the running column accumulator. (Round 4 measured a
// use-only empty asm after each step, which keeps LLVM from splitting a column: 4 401 instead
// of 4 579 instructions per mixed addition, but one dependent chain per product ran 3-4 %
// SLOWER, profiles/r04_ubench_acc_pins.txt; removed in round 5. The product groups below pin
// with "+v" instead.)
PLK_RX void rx_madd(uint64_t& acc, uint32_t x, uint32_t y) { acc += (uint64_t)x * y; }

// Close column k of a split-capable product: acc holds the products (+ the incoming
// carry), s2 the reduction terms and s3 a second product set (split columns only; both 0
// otherwise). Below L the column's Montgomery digit m[k] is formed and its m_k p_0 added;
// from L on the low B bits are output limb k - L. acc leaves holding the carry.
template <class C>
PLK_RX void rx_column_close(bool split, int k, uint64_t& acc, uint64_t s2, uint64_t s3,
                            uint32_t* m, Rx<C>& r) {
  constexpr int L = RxShape<C>::L, B = RxShape<C>::B;
  constexpr uint32_t MASK = (1u << B) - 1;
  constexpr RxConst<C> K = RxK<C>::k;
  if (!split) {
    if (k < L) {
      m[k] = ((uint32_t)acc * K.inv) & MASK;
      rx_madd(acc, m[k], K.p[0]);
    } else {
      r.v[k - L] = (uint32_t)acc & MASK;
    }
    acc >>= B;
    return;
  }
  // low B bits of each part (< 3 * 2^B < 2^32) and their carries, summed apart
  const uint32_t lo32 = ((uint32_t)acc & MASK) + ((uint32_t)s2 & MASK) + ((uint32_t)s3 & MASK);
  const uint64_t hi = (acc >> B) + (s2 >> B) + (s3 >> B);
  uint64_t lo = lo32;
  if (k < L) {
    m[k] = (lo32 * K.inv) & MASK;
    lo += (uint64_t)m[k] * K.p[0];
  } else {
    r.v[k - L] = lo32 & MASK;
  }
  acc = hi + (lo >> B);
}

template <class C>
PLK_RX Rx<C> rx_zero() {
  Rx<C> r;
#pragma unroll
  for (int i = 0; i < RxShape<C>::L; ++i) r.v[i] = 0;
  return r;
}

template <class C>
PLK_RX Rx<C> rx_one() {
  constexpr RxConst<C> K = RxK<C>::k;
  Rx<C> r;
#pragma unroll
  for (int i = 0; i < RxShape<C>::L; ++i) r.v[i] = K.one[i];
  return r;
}

// a * b / R' mod p, inputs in [0, 2p) (normalised limbs), output in [0, 2p)
template <class C>
PLK_RX Rx<C> rx_mul(const Rx<C>& a, const Rx<C>& b) {
  constexpr int L = RxShape<C>::L, B = RxShape<C>::B;
  constexpr uint32_t MASK = (1u << B) - 1;
  constexpr RxConst<C> K = RxK<C>::k;
  uint32_t m[L];
  Rx<C> r;
  uint64_t acc = 0;
  if constexpr (!RxSplitOn<C>::value) {
#pragma unroll
    for (int k = 0; k < L; ++k) {
#pragma unroll
      for (int i = 0; i <= k; ++i) acc += (uint64_t)a.v[i] * b.v[k - i];
#pragma unroll
      for (int i = 0; i < k; ++i) acc += (uint64_t)m[i] * K.p[k - i];
      m[k] = ((uint32_t)acc * K.inv) & MASK;
      acc += (uint64_t)m[k] * K.p[0];
      acc >>= B;
    }
#pragma unroll
    for (int k = L; k < 2 * L - 1; ++k) {
#pragma unroll
      for (int i = k - L + 1; i < L; ++i) acc += (uint64_t)a.v[i] * b.v[k - i];
#pragma unroll
      for (int i = k - L + 1; i < L; ++i) acc += (uint64_t)m[i] * K.p[k - i];
      r.v[k - L] = (uint32_t)acc & MASK;
      acc >>= B;
    }
  } else {
    constexpr RxPlan<C, 1> PL = RxPlanK<C, 1>::k;
#pragma unroll
    for (int k = 0; k < 2 * L - 1; ++k) {
      const int i0 = k < L ? 0 : k - L + 1, i1 = k < L ? k : L - 1;
      uint64_t s2 = 0;
#pragma unroll
      for (int i = i0; i <= i1; ++i) rx_madd(acc, a.v[i], b.v[k - i]);
#pragma unroll
      for (int i = i0; i <= i1; ++i)
        if (i < k || k >= L) rx_madd(PL.split[k] ? s2 : acc, m[i], K.p[k - i]);
      rx_column_close<C>(PL.split[k], k, acc, s2, 0, m, r);
    }
  }
  r.v[L - 1] = (uint32_t)acc;
  return r;
}

// (a*b + c*d) / R' mod p with ONE Montgomery reduction: both product columns accumulate
// into the same 64-bit column (the caller bounds the limbs so that 2L products plus L
// reduction products stay below 2^64 — or, for split shapes, each product set and the
// reduction terms in an accumulator of their own — and the value so that
// (ab + cd) / R' + p < 2p).
template <class C>
PLK_RX Rx<C> rx_mul_add(const Rx<C>& a, const Rx<C>& b, const Rx<C>& c, const Rx<C>& d) {
  constexpr int L = RxShape<C>::L, B = RxShape<C>::B;
  constexpr uint32_t MASK = (1u << B) - 1;
  constexpr RxConst<C> K = RxK<C>::k;
  uint32_t m[L];
  Rx<C> r;
  uint64_t acc = 0;
  if constexpr (!RxSplitOn<C>::value) {
#pragma unroll
    for (int k = 0; k < L; ++k) {
#pragma unroll
      for (int i = 0; i <= k; ++i) acc += (uint64_t)a.v[i] * b.v[k - i];
#pragma unroll
      for (int i = 0; i <= k; ++i) acc += (uint64_t)c.v[i] * d.v[k - i];
#pragma unroll
      for (int i = 0; i < k; ++i) acc += (uint64_t)m[i] * K.p[k - i];
      m[k] = ((uint32_t)acc * K.inv) & MASK;
      acc += (uint64_t)m[k] * K.p[0];
      acc >>= B;
    }
#pragma unroll
    for (int k = L; k < 2 * L - 1; ++k) {
#pragma unroll
      for (int i = k - L + 1; i < L; ++i) acc += (uint64_t)a.v[i] * b.v[k - i];
#pragma unroll
      for (int i = k - L + 1; i < L; ++i) acc += (uint64_t)c.v[i] * d.v[k - i];
#pragma unroll
      for (int i = k - L + 1; i < L; ++i) acc += (uint64_t)m[i] * K.p[k - i];
      r.v[k - L] = (uint32_t)acc & MASK;
      acc >>= B;
    }
  } else {
    constexpr RxPlan<C, 2> PL = RxPlanK<C, 2>::k;
#pragma unroll
    for (int k = 0; k < 2 * L - 1; ++k) {
      const int i0 = k < L ? 0 : k - L + 1, i1 = k < L ? k : L - 1;
      uint64_t s2 = 0, s3 = 0;
#pragma unroll
      for (int i = i0; i <= i1; ++i) rx_madd(acc, a.v[i], b.v[k - i]);
#pragma unroll
      for (int i = i0; i <= i1; ++i) rx_madd(PL.split[k] ? s3 : acc, c.v[i], d.v[k - i]);
#pragma unroll
      for (int i = i0; i <= i1; ++i)
        if (i < k || k >= L) rx_madd(PL.split[k] ? s2 : acc, m[i], K.p[k - i]);
      rx_column_close<C>(PL.split[k], k, acc, s2, s3, m, r);
    }
  }
  r.v[L - 1] = (uint32_t)acc;
  return r;
}

// a^2 / R': the cross products a_i a_j (i < j) once, doubled
template <class C>
PLK_RX Rx<C> rx_sqr(const Rx<C>& a) {
  constexpr int L = RxShape<C>::L, B = RxShape<C>::B;
  constexpr uint32_t MASK = (1u << B) - 1;
  constexpr RxConst<C> K = RxK<C>::k;
  uint32_t m[L], a2[L];
#pragma unroll
  for (int i = 0; i < L; ++i) a2[i] = a.v[i] << 1;
  Rx<C> r;
  uint64_t acc = 0;
  if constexpr (!RxSplitOn<C>::value) {
#pragma unroll
    for (int k = 0; k < 2 * L - 1; ++k) {
#pragma unroll
      for (int i = (k < L ? 0 : k - L + 1); 2 * i < k; ++i) acc += (uint64_t)a.v[i] * a2[k - i];
      if ((k & 1) == 0) acc += (uint64_t)a.v[k / 2] * a.v[k / 2];
      if (k < L) {
#pragma unroll
        for (int i = 0; i < k; ++i) acc += (uint64_t)m[i] * K.p[k - i];
        m[k] = ((uint32_t)acc * K.inv) & MASK;
        acc += (uint64_t)m[k] * K.p[0];
      } else {
#pragma unroll
        for (int i = k - L + 1; i < L; ++i) acc += (uint64_t)m[i] * K.p[k - i];
        r.v[k - L] = (uint32_t)acc & MASK;
      }
      acc >>= B;
    }
  } else {
    // the doubled cross products and the square sum to the product column of a * a
    constexpr RxPlan<C, 1> PL = RxPlanK<C, 1>::k;
#pragma unroll
    for (int k = 0; k < 2 * L - 1; ++k) {
      const int i0 = k < L ? 0 : k - L + 1, i1 = k < L ? k : L - 1;
      uint64_t s2 = 0;
#pragma unroll
      for (int i = i0; 2 * i < k; ++i) rx_madd(acc, a.v[i], a2[k - i]);
      if ((k & 1) == 0) rx_madd(acc, a.v[k / 2], a.v[k / 2]);
#pragma unroll
      for (int i = i0; i <= i1; ++i)
        if (i < k || k >= L) rx_madd(PL.split[k] ? s2 : acc, m[i], K.p[k - i]);
      rx_column_close<C>(PL.split[k], k, acc, s2, 0, m, r);
    }
  }
  r.v[L - 1] = (uint32_t)acc;
  return r;
}

// ---- interleaved product groups (split shapes: Fp 13 x 30) ----------------------------
// NP independent Montgomery products computed column by column with their partial products
// interleaved mad by mad: product p's column k is ONE chain on its own accumulator (the
// incoming carry at the head, no second accumulator merged by a 64-bit add), and the chains
// of the NP products alternate, so consecutive v_mad_u64_u32 never depend on each other (a
// dependent pair needs a wait state on gfx950). Every step passes rx_pin so LLVM keeps each
// chain as written instead of reassociating it (which is what costs the merge adds).
// Kinds: kRxMul a*b, kRxSqr a^2 (b unused), kRxMulAdd a*b + c*d (one reduction, rx_mul_add's
// bounds). Same results as rx_mul / rx_sqr / rx_mul_add, bit for bit.
enum : int { kRxMul = 0, kRxSqr = 1, kRxMulAdd = 2 };

// "+v": the accumulator is redefined by the (empty) asm, so the next step of the chain
// depends on it and the volatile asms keep the interleaved order. The hazard recognizer then
// pads a chain's next mad with one s_nop when fewer than three instructions separate it
// from the asm (two-product groups): one wait cycle, against the 64-bit merge add per column
// it replaces. A use-only pin ("v" input) leaves the order to the scheduler, which
// regroups the chains: measured no faster than the plain code (profiles/r04_ubench_acc_pins.txt).
// Round 6 measured what that padding costs (profiles/r06_nop_cost_ab.jsonl, 2^20 proofs, two
// interleaved runs): one more s_nop 0 per step (+3 040 per mixed addition) took the lane form
// of k_accumulate from 6.76 to 6.24e9 additions/s, i.e. ~0.5 issue cycle per s_nop, so the ~440
// it pays are ~1 % of the kernel. Each step written as an inline-asm v_mad_u64_u32 instead (no
// pins; every asm also defines vcc, which the hazard recognizer pads after) drew 2 297 s_nop and
// ran 6.64e9: not kept (commit 3100a20 has both probes).
PLK_RX void rx_pin(uint64_t& v) { __asm__ volatile("" : "+v"(v)); }

template <class C, int NP>
struct RxGroupState {
  uint32_t m[NP][RxShape<C>::L], a2[NP][RxShape<C>::L];
  uint64_t acc[NP];
};

// The mad order of column K: accumulator ids (3p: product p's acc, 3p + 1: its reduction
// accumulator s2, 3p + 2: its second product set s3 — the last two in split columns only),
// greedily taking the accumulator with the most terms left that differs from the previous
// one, so no two consecutive mads share an accumulator whenever the counts allow it.
template <int NP>
struct RxColOrder {
  int n = 0;
  int acc[3 * 26 * 4] = {};  // at most 3 * 2L mads per product per column, L <= 13
};

template <class C, int K, int... KINDS>
constexpr RxColOrder<sizeof...(KINDS)> rx_col_order() {
  constexpr int L = RxShape<C>::L;
  constexpr int NP = sizeof...(KINDS);
  constexpr int kind[NP] = {KINDS...};
  constexpr RxPlan<C, 1> P1{};
  constexpr RxPlan<C, 2> P2{};
  constexpr bool SPLIT_ON = RxSplitOn<C>::value;
  const int i0 = K < L ? 0 : K - L + 1, i1 = K < L ? K : L - 1;
  const int n1 = i1 - i0 + 1;
  const int ncross = (K + 1) / 2 - i0 > 0 ? (K + 1) / 2 - i0 : 0;
  int nred = 0;
  for (int i = i0; i <= i1; ++i)
    if (i < K || K >= L) ++nred;
  int left[3 * NP] = {};
  for (int p = 0; p < NP; ++p) {
    const bool split = SPLIT_ON && (kind[p] == kRxMulAdd ? P2.split[K] : P1.split[K]);
    const int prod = kind[p] == kRxMul ? n1 : kind[p] == kRxSqr ? ncross + ((K & 1) == 0 ? 1 : 0) : 2 * n1;
    if (!split) {
      left[3 * p] = prod + nred;
    } else {
      left[3 * p] = kind[p] == kRxMulAdd ? n1 : prod;
      left[3 * p + 1] = nred;
      left[3 * p + 2] = kind[p] == kRxMulAdd ? n1 : 0;
    }
  }
  RxColOrder<NP> o{};
  int last = -1;
  for (;;) {
    int best = -1;
    for (int q = 0; q < 3 * NP; ++q)
      if (left[q] > 0 && q != last && (best < 0 || left[q] > left[best])) best = q;
    if (best < 0) {  // only the previous accumulator has terms left
      if (last >= 0 && left[last] > 0) best = last;
      else break;
    }
    o.acc[o.n++] = best;
    --left[best];
    last = best;
  }
  return o;
}

}  // namespace plk
#include "rx_asm_gen.hpp"
namespace plk {
// The ASM form of a product group (round 6; the lane form of k_accumulate): each column of an
// Fp group as ONE inline-asm statement holding its interleaved v_mad_u64_u32 in
// rx_col_order's order, so that no empty pin sits between the mads and the hazard recognizer
// pads only where the column's closing instructions read the statement's outputs: 420-440 ->
// 67-77 s_nop and 4 855-4 873 -> 4 501-4 509 instructions in k_accumulate's loop block (same
// 3 056 v_mad_u64_u32; hipcc -S of msm_acc.hip, both lane-form instantiations). The statement's
// text is built here at compile time; its operand list (the accumulator slots, the first
// factors, the variable
// second factors in VGPRs and the limbs of p in SGPRs) comes from rx_asm_gen.hpp
// (tools/gen_rx_asm.py). Measured (profiles/r06_asm_columns_ab.jsonl, three interleaved runs):
// solo additions/s in the 2^20 proof 6.97 -> 7.02e9 and in the 2^16 proof 5.28 -> 5.55e9,
// proofs 32.55 -> 32.80 M (2^20) and 26.28 -> 26.91 M (2^16); the same form in the run sums'
// full additions (triples, at 1 wave per SIMD) measured no better and is not used there.
// Fr (no split columns, one accumulator per product: RxAsmRun1) takes the same form in the
// NTT pass's pairs (ntt.hip twmul2).
struct RxAsmText {
  char s[8192];
  int len;
  constexpr const char* data() const { return s; }
  constexpr unsigned long size() const { return (unsigned long)len; }
};
constexpr void rx_asm_put(RxAsmText& t, const char* x) {
  for (int i = 0; x[i]; ++i) t.s[t.len++] = x[i];
}
constexpr void rx_asm_num(RxAsmText& t, int v) {
  char b[8] = {};
  int n = 0;
  do {
    b[n++] = (char)('0' + v % 10);
    v /= 10;
  } while (v);
  while (n) t.s[t.len++] = b[--n];
}
// Whether mad e of column K multiplies by a constant (a limb of p: a Montgomery reduction
// term), in rx_group_column's term order; `first`: its accumulator starts there.
struct RxAsmTerm {
  int slot, red, first;
};
template <class C, int K, int... KINDS>
struct RxAsmPlan {
  static constexpr int NP = sizeof...(KINDS);
  // split shapes (Fp): 3 slots per product (acc, s2, s3); otherwise (Fr) one, the acc
  static constexpr bool SPL = RxSplitOn<C>::value;
  static constexpr int S = SPL ? 3 * NP : NP;
  RxAsmTerm t[3 * 26 * 4] = {};
  int n = 0, nv = 0, ns = 0;
  int used[3 * NP] = {};  // the slot takes a term in this column
  constexpr RxAsmPlan() {
    constexpr int L = RxShape<C>::L;
    constexpr int kind[NP] = {KINDS...};
    constexpr RxPlan<C, 1> P1{};
    constexpr RxPlan<C, 2> P2{};
    constexpr RxColOrder<NP> ord = rx_col_order<C, K, KINDS...>();
    const int i0 = K < L ? 0 : K - L + 1, i1 = K < L ? K : L - 1;
    const int n1 = i1 - i0 + 1;
    const int ncross = (K + 1) / 2 - i0 > 0 ? (K + 1) / 2 - i0 : 0;
    const int nsq = ncross + ((K & 1) == 0 ? 1 : 0);
    int pos[3 * NP] = {};
    n = ord.n;
    for (int e = 0; e < n; ++e) {
      const int q = ord.acc[e], p = q / 3, which = q % 3;
      const bool split = SPL && (kind[p] == kRxMulAdd ? P2.split[K] : P1.split[K]);
      const int nprod = which != 0 ? 0 : kind[p] == kRxMul ? n1 : kind[p] == kRxSqr ? nsq
                                       : (split ? n1 : 2 * n1);
      const int tt = pos[q]++;
      t[e].slot = SPL ? q : p;
      t[e].red = which == 1 || (which == 0 && tt >= nprod);
      t[e].first = tt == 0 && (which != 0 || K == 0);
      if (t[e].red) ++ns; else ++nv;
      used[q] = 1;
    }
  }
};
// mad e: v_mad_u64_u32 %slot, vcc, %(S + e), %(its second factor), %slot — or 0 as the addend
// when the slot starts there (s2 / s3 of a split column, the first column's accumulators).
// Operands: S slots, N first factors, NV variable second factors, NS constant ones.
template <class C, int K, int... KINDS>
constexpr RxAsmText rx_asm_text() {
  constexpr RxAsmPlan<C, K, KINDS...> P{};
  const int S = P.S, N = P.n;
  RxAsmText t{};
  int jv = 0, js = 0;
  for (int e = 0; e < N; ++e) {
    const RxAsmTerm& m = P.t[e];
    rx_asm_put(t, "v_mad_u64_u32 %");
    rx_asm_num(t, m.slot);
    rx_asm_put(t, ", vcc, %");
    rx_asm_num(t, S + e);
    rx_asm_put(t, ", %");
    rx_asm_num(t, m.red ? S + N + P.nv + js++ : S + N + jv++);
    if (m.first) {
      rx_asm_put(t, ", 0\n");
    } else {
      rx_asm_put(t, ", %");
      rx_asm_num(t, m.slot);
      rx_asm_put(t, "\n");
    }
  }
  return t;
}
template <class C, int K, int... KINDS>
struct RxAsmTextK {
  static constexpr RxAsmText text = rx_asm_text<C, K, KINDS...>();
};

// column K of every product of the group (K a template argument: every bound and branch
// below is a compile-time constant). Each accumulator's terms are taken in a fixed order
// (operand products first, then reduction terms); the interleaving is rx_col_order's.
template <class C, bool ASM, int K, int... KINDS>
PLK_RX void rx_group_column(RxGroupState<C, sizeof...(KINDS)>& g, const Rx<C>* const* a,
                            const Rx<C>* const* b, const Rx<C>* const* c, const Rx<C>* const* d,
                            Rx<C>* const* out) {
  constexpr int L = RxShape<C>::L;
  constexpr int NP = sizeof...(KINDS);
  constexpr int kind[NP] = {KINDS...};
  constexpr RxConst<C> KC = RxK<C>::k;
  constexpr RxPlan<C, 1> P1 = RxPlanK<C, 1>::k;
  constexpr RxPlan<C, 2> P2 = RxPlanK<C, 2>::k;
  constexpr bool SPLIT_ON = RxSplitOn<C>::value;  // Fr (9 x 29): one accumulator per column
  constexpr int i0 = K < L ? 0 : K - L + 1, i1 = K < L ? K : L - 1;
  constexpr int n1 = i1 - i0 + 1;                                      // terms of one a*b column
  constexpr int ncross = (K + 1) / 2 - i0 > 0 ? (K + 1) / 2 - i0 : 0;  // a^2: i0 <= i, 2i < K
  constexpr int nsq = ncross + ((K & 1) == 0 ? 1 : 0);
  constexpr int rfirst = (K < L) ? 0 : i0;  // reduction terms: i in [rfirst, i1], i < K below L
  constexpr int rlast = (K < L) ? K - 1 : i1;
  constexpr RxColOrder<NP> ord = rx_col_order<C, K, KINDS...>();
  uint64_t s2[NP], s3[NP];
  int pos[3 * NP];  // next term of each accumulator
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    s2[p] = s3[p] = 0;
    pos[3 * p] = pos[3 * p + 1] = pos[3 * p + 2] = 0;
  }
  constexpr bool kAsmCol = ASM;
  if constexpr (kAsmCol) {  // the column's mads as one asm statement (see RxAsmText)
    constexpr RxAsmPlan<C, K, KINDS...> PLAN{};
    uint32_t X[PLAN.n], Y[PLAN.nv > 0 ? PLAN.nv : 1], KP[PLAN.ns > 0 ? PLAN.ns : 1];
    int jv = 0, js = 0;
#pragma unroll
    for (int e = 0; e < ord.n; ++e) {
      const int q = ord.acc[e], p = q / 3, which = q % 3;
      const bool split = SPLIT_ON && (kind[p] == kRxMulAdd ? P2.split[K] : P1.split[K]);
      const int t = pos[q]++;
      const int nprod = which != 0 ? 0 : kind[p] == kRxMul ? n1 : kind[p] == kRxSqr ? nsq
                                       : (split ? n1 : 2 * n1);
      if (which == 2) {
        X[e] = c[p]->v[i0 + t]; Y[jv++] = d[p]->v[K - i0 - t];
      } else if (which == 1 || t >= nprod) {
        const int i = rfirst + (which == 1 ? t : t - nprod);
        X[e] = g.m[p][i]; KP[js++] = KC.p[K - i];
      } else if (kind[p] == kRxSqr) {
        if (t < ncross) { X[e] = a[p]->v[i0 + t]; Y[jv++] = g.a2[p][K - i0 - t]; }
        else { X[e] = a[p]->v[K / 2]; Y[jv++] = a[p]->v[K / 2]; }
      } else if (t < n1) {
        X[e] = a[p]->v[i0 + t]; Y[jv++] = b[p]->v[K - i0 - t];
      } else {
        X[e] = c[p]->v[i0 + t - n1]; Y[jv++] = d[p]->v[K - i0 - t + n1];
      }
    }
    if constexpr (SPLIT_ON) {
      // s2 / s3 are output-only operands (rx_asm_gen.hpp); the carried accumulators go in
      uint64_t slot[3 * NP];
#pragma unroll
      for (int p = 0; p < NP; ++p) slot[3 * p] = g.acc[p];
      RxAsmRun<PLAN.nv, PLAN.ns, 3 * NP>::template run<RxAsmTextK<C, K, KINDS...>>(slot, X, Y, KP);
#pragma unroll
      for (int p = 0; p < NP; ++p) {  // a slot the column does not use stays 0 (rx_column_close)
        g.acc[p] = slot[3 * p];
        s2[p] = PLAN.used[3 * p + 1] ? slot[3 * p + 1] : 0;
        s3[p] = PLAN.used[3 * p + 2] ? slot[3 * p + 2] : 0;
      }
    } else {  // one accumulator per product, carried in and out
      RxAsmRun1<PLAN.nv, PLAN.ns, NP>::template run<RxAsmTextK<C, K, KINDS...>>(g.acc, X, Y, KP);
    }
  }
  if constexpr (!kAsmCol) {
#pragma unroll
  for (int e = 0; e < ord.n; ++e) {
    const int q = ord.acc[e], p = q / 3, which = q % 3;
    const bool split = SPLIT_ON && (kind[p] == kRxMulAdd ? P2.split[K] : P1.split[K]);
    const int t = pos[q]++;
    uint64_t& dst = which == 0 ? g.acc[p] : which == 1 ? s2[p] : s3[p];
    // the accumulator's t-th term
    const int nprod = which != 0 ? 0 : kind[p] == kRxMul ? n1 : kind[p] == kRxSqr ? nsq
                                     : (split ? n1 : 2 * n1);
    if (which == 2) {  // c*d of a split mul_add column
      rx_madd(dst, c[p]->v[i0 + t], d[p]->v[K - i0 - t]);
    } else if (which == 1 || t >= nprod) {  // a reduction term
      const int i = rfirst + (which == 1 ? t : t - nprod);
      rx_madd(dst, g.m[p][i], KC.p[K - i]);
    } else if (kind[p] == kRxSqr) {
      if (t < ncross) rx_madd(dst, a[p]->v[i0 + t], g.a2[p][K - i0 - t]);
      else rx_madd(dst, a[p]->v[K / 2], a[p]->v[K / 2]);
    } else if (t < n1) {
      rx_madd(dst, a[p]->v[i0 + t], b[p]->v[K - i0 - t]);
    } else {  // mul_add, non-split: c*d into acc
      rx_madd(dst, c[p]->v[i0 + t - n1], d[p]->v[K - i0 - t + n1]);
    }
    rx_pin(dst);
  }
  }
  (void)rlast;
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    const bool split = SPLIT_ON && (kind[p] == kRxMulAdd ? P2.split[K] : P1.split[K]);
    rx_column_close<C>(split, K, g.acc[p], s2[p], s3[p], g.m[p], *out[p]);
  }
}

template <class C, bool ASM, int... KINDS, int... KS>
PLK_RX void rx_group_columns(RxGroupState<C, sizeof...(KINDS)>& g, const Rx<C>* const* a,
                             const Rx<C>* const* b, const Rx<C>* const* c,
                             const Rx<C>* const* d, Rx<C>* const* out,
                             std::integer_sequence<int, KS...>) {
  (rx_group_column<C, ASM, KS, KINDS...>(g, a, b, c, d, out), ...);
}

// ASM: the columns as single asm statements (Fp only; see RxAsmText)
template <class C, bool ASM, int... KINDS>
PLK_RX void rx_prod_group(const Rx<C>* const* a, const Rx<C>* const* b, const Rx<C>* const* c,
                          const Rx<C>* const* d, Rx<C>* const* out) {
  constexpr int L = RxShape<C>::L;
  constexpr int NP = sizeof...(KINDS);
  constexpr int kind[NP] = {KINDS...};
  RxGroupState<C, NP> g;
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    g.acc[p] = 0;
    if (kind[p] == kRxSqr) {
#pragma unroll
      for (int i = 0; i < L; ++i) g.a2[p][i] = a[p]->v[i] << 1;
    }
  }
  rx_group_columns<C, ASM, KINDS...>(g, a, b, c, d, out,
                                     std::make_integer_sequence<int, 2 * L - 1>{});
#pragma unroll
  for (int p = 0; p < NP; ++p) out[p]->v[L - 1] = (uint32_t)g.acc[p];
}

// the pair / triple forms used by the group law
template <class C, bool ASM = false>
PLK_RX void rx_mul2(const Rx<C>& a0, const Rx<C>& b0, const Rx<C>& a1, const Rx<C>& b1,
                    Rx<C>& o0, Rx<C>& o1) {
  const Rx<C>* a[2] = {&a0, &a1};
  const Rx<C>* b[2] = {&b0, &b1};
  Rx<C>* o[2] = {&o0, &o1};
  rx_prod_group<C, ASM, kRxMul, kRxMul>(a, b, a, b, o);
}
template <class C, bool ASM = false>
PLK_RX void rx_sqr2(const Rx<C>& a0, const Rx<C>& a1, Rx<C>& o0, Rx<C>& o1) {
  const Rx<C>* a[2] = {&a0, &a1};
  Rx<C>* o[2] = {&o0, &o1};
  rx_prod_group<C, ASM, kRxSqr, kRxSqr>(a, a, a, a, o);
}
template <class C>
PLK_RX void rx_mul3(const Rx<C>& a0, const Rx<C>& b0, const Rx<C>& a1, const Rx<C>& b1,
                    const Rx<C>& a2, const Rx<C>& b2, Rx<C>& o0, Rx<C>& o1, Rx<C>& o2) {
  const Rx<C>* a[3] = {&a0, &a1, &a2};
  const Rx<C>* b[3] = {&b0, &b1, &b2};
  Rx<C>* o[3] = {&o0, &o1, &o2};
  rx_prod_group<C, false, kRxMul, kRxMul, kRxMul>(a, b, a, b, o);
}
// (a0 b0 + c0 d0, a1 b1, a2 b2): the fused Y3 beside ZZ3 and ZZZ3 (its 2 product sets
// against their one each: the three accumulators alternate)
template <class C, bool ASM = false>
PLK_RX void rx_mul_add_mul2(const Rx<C>& a0, const Rx<C>& b0, const Rx<C>& c0, const Rx<C>& d0,
                            const Rx<C>& a1, const Rx<C>& b1, const Rx<C>& a2, const Rx<C>& b2,
                            Rx<C>& o0, Rx<C>& o1, Rx<C>& o2) {
  const Rx<C>* a[3] = {&a0, &a1, &a2};
  const Rx<C>* b[3] = {&b0, &b1, &b2};
  const Rx<C>* c[3] = {&c0, &c0, &c0};
  const Rx<C>* d[3] = {&d0, &d0, &d0};
  Rx<C>* o[3] = {&o0, &o1, &o2};
  rx_prod_group<C, ASM, kRxMulAdd, kRxMul, kRxMul>(a, b, c, d, o);
}

// a + b mod 2p-range: [0, 2p) + [0, 2p) -> [0, 2p)
template <class C>
PLK_RX Rx<C> rx_add(const Rx<C>& a, const Rx<C>& b) {
  constexpr int L = RxShape<C>::L, B = RxShape<C>::B;
  constexpr uint32_t MASK = (1u << B) - 1;
  constexpr RxConst<C> K = RxK<C>::k;
  Rx<C> s, d;
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < L; ++i) {
    const uint32_t t = a.v[i] + b.v[i] + c;
    s.v[i] = t & MASK;
    c = t >> B;
  }
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < L; ++i) {
    const uint32_t t = s.v[i] - K.p2[i] - br;
    d.v[i] = t & MASK;
    br = t >> 31;
  }
  // br: s < 2p -> keep s
#pragma unroll
  for (int i = 0; i < L; ++i) s.v[i] = br ? s.v[i] : d.v[i];
  return s;
}

template <class C>
PLK_RX Rx<C> rx_sub(const Rx<C>& a, const Rx<C>& b) {
  constexpr int L = RxShape<C>::L, B = RxShape<C>::B;
  constexpr uint32_t MASK = (1u << B) - 1;
  constexpr RxConst<C> K = RxK<C>::k;
  Rx<C> d, e;
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < L; ++i) {
    const uint32_t t = a.v[i] - b.v[i] - br;
    d.v[i] = t & MASK;
    br = t >> 31;
  }
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < L; ++i) {
    const uint32_t t = d.v[i] + K.p2[i] + c;
    e.v[i] = t & MASK;
    c = t >> B;
  }
#pragma unroll
  for (int i = 0; i < L; ++i) d.v[i] = br ? e.v[i] : d.v[i];
  return d;
}

// a - b + 2p in (0, 4p) without the conditional pass: for operands headed straight into
// rx_mul, which accepts inputs below 8p (Fr: 8r^2 / R' + r < 2r)
template <class C>
PLK_RX Rx<C> rx_sub_lazy(const Rx<C>& a, const Rx<C>& b) {
  constexpr int L = RxShape<C>::L, B = RxShape<C>::B;
  constexpr uint32_t MASK = (1u << B) - 1;
  constexpr RxConst<C> K = RxK<C>::k;
  Rx<C> d;
  int32_t c = 0;
#pragma unroll
  for (int i = 0; i < L; ++i) {
    const int32_t t = (int32_t)(a.v[i] + K.p2[i]) - (int32_t)b.v[i] + c;
    d.v[i] = (uint32_t)t & MASK;
    c = t >> B;  // arithmetic: -1, 0 or +1
  }
  return d;
}

template <class C>
PLK_RX Rx<C> rx_dbl(const Rx<C>& a) {
  return rx_add(a, a);
}

template <class C>
PLK_RX Rx<C> rx_neg(const Rx<C>& a) {
  return rx_sub(rx_zero<C>(), a);
}

// ---- unnormalised differences (feed multiplications only) ---------------------------
// a + c*p - b limb by limb, no carries: a normalised with value < 2p, b normalised with
// value < (c - 1) p. Limbs < 2^(B+2) and value < (c + 2) p — rx_mul / rx_sqr accept such
// operands for shapes whose columns keep headroom (Fr 9 x 29: a 64-bit column of 9 products
// below 2^61.6 plus 9 reduction products below 2^58 stays under 2^64). Split shapes (Fp
// 13 x 30, RxPlan) assume normalised operand limbs: there the difference is carried
// (rx_sub_n, same value range, ~2 more instructions per limb).
template <class C, uint32_t CP>
PLK_RX Rx<C> rx_sub_n(const Rx<C>& a, const Rx<C>& b);

template <class C, uint32_t CP>
PLK_RX Rx<C> rx_sub_u(const Rx<C>& a, const Rx<C>& b) {
  if constexpr (RxSplitOn<C>::value) {
    return rx_sub_n<C, CP>(a, b);
  } else {
    constexpr RxMultiple<C> Q = RxMultipleK<C, CP, true>::k;
    Rx<C> r;
#pragma unroll
    for (int i = 0; i < RxShape<C>::L; ++i) r.v[i] = a.v[i] + Q.v[i] - b.v[i];
    return r;
  }
}

// a + c*p - b with the carries propagated (signed): normalised limbs, value in
// (c*p - max b, c*p + max a) — no conditional pass. a, b normalised (a_i + (cp)_i < 2^31)
template <class C, uint32_t CP>
PLK_RX Rx<C> rx_sub_n(const Rx<C>& a, const Rx<C>& b) {
  constexpr int L = RxShape<C>::L, B = RxShape<C>::B;
  constexpr uint32_t MASK = (1u << B) - 1;
  constexpr RxMultiple<C> Q = RxMultipleK<C, CP, false>::k;
  Rx<C> d;
  int32_t c = 0;
#pragma unroll
  for (int i = 0; i < L; ++i) {
    const int32_t t = (int32_t)(a.v[i] + Q.v[i]) - (int32_t)b.v[i] + c;
    d.v[i] = i == L - 1 ? (uint32_t)t : ((uint32_t)t & MASK);
    c = t >> B;
  }
  return d;
}

// a + c*p - b - 2e, carries propagated (the X3 of the XYZZ addition in one pass); 64-bit
// limb sums where a limb of 2e can exceed 2^31 (B >= 30)
template <class C, uint32_t CP>
PLK_RX Rx<C> rx_sub2_n(const Rx<C>& a, const Rx<C>& b, const Rx<C>& e) {
  constexpr int L = RxShape<C>::L, B = RxShape<C>::B;
  constexpr uint32_t MASK = (1u << B) - 1;
  constexpr RxMultiple<C> Q = RxMultipleK<C, CP, false>::k;
  using S = typename std::conditional<(B >= 30), int64_t, int32_t>::type;
  Rx<C> d;
  S c = 0;
#pragma unroll
  for (int i = 0; i < L; ++i) {
    const S t = (S)(a.v[i] + Q.v[i]) - (S)b.v[i] - ((S)e.v[i] << 1) + c;
    d.v[i] = i == L - 1 ? (uint32_t)t : ((uint32_t)t & MASK);
    c = t >> B;
  }
  return d;
}

// k * a (k small) with the carries propagated: normalised limbs, value k * a
template <class C, uint32_t KM>
PLK_RX Rx<C> rx_small_mul_n(const Rx<C>& a) {
  constexpr int L = RxShape<C>::L, B = RxShape<C>::B;
  constexpr uint32_t MASK = (1u << B) - 1;
  Rx<C> d;
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < L; ++i) {
    const uint64_t t = (uint64_t)a.v[i] * KM + c;
    d.v[i] = i == L - 1 ? (uint32_t)t : ((uint32_t)t & MASK);
    c = (uint32_t)(t >> B);
  }
  return d;
}

// Necessary condition for a - b == k*p with k in [-kneg, kpos] (a, b normalised): the low
// limbs then satisfy (a0 - b0) * (-p^-1) == -k (mod 2^B). False positives ~ (kpos+kneg+1)/2^B.
template <class C>
PLK_RX bool rx_maybe_multiple(uint32_t a0, uint32_t b0, uint32_t kpos, uint32_t kneg) {
  constexpr uint32_t MASK = (1u << RxShape<C>::B) - 1;
  constexpr RxConst<C> K = RxK<C>::k;
  return (((a0 - b0) * K.inv + kpos) & MASK) <= kpos + kneg;
}

// a reduced to [0, 2p), normalised: a * R' / R'. Operands: for unsplit shapes (Fr) any value
// < 16p with limbs < 2^(B+2); for split shapes (Fp 13 x 30) normalised limbs (< 2^B) and a
// value within the split plan's bound (< 12p, RxPlan).
template <class C>
PLK_RX Rx<C> rx_canon(const Rx<C>& a) {
  return rx_mul(a, rx_one<C>());
}

// a == 0 mod p, operands as rx_canon's (unsplit shapes: < 16p, limbs < 2^(B+2); split
// shapes: normalised limbs, < 12p): (a / R') is in [0, 2p)
template <class C>
PLK_RX bool rx_is_zero_u(const Rx<C>& a) {
  Rx<C> one = rx_zero<C>();
  one.v[0] = 1;
  return rx_is_zero(rx_mul(a, one));
}

// a in [0, 2p): a == 0 mod p  <=>  a in {0, p}
template <class C>
PLK_RX bool rx_is_zero(const Rx<C>& a) {
  constexpr int L = RxShape<C>::L;
  constexpr RxConst<C> K = RxK<C>::k;
  uint32_t z = 0, q = 0;
#pragma unroll
  for (int i = 0; i < L; ++i) {
    z |= a.v[i];
    q |= a.v[i] ^ K.p[i];
  }
  return z == 0 || q == 0;
}

// packed N-word value (< 2^(32N)) -> limbs
template <class C>
PLK_RX Rx<C> rx_unpack(const Fe<C>& x) {
  constexpr int L = RxShape<C>::L, B = RxShape<C>::B, N = C::N;
  constexpr uint32_t MASK = (1u << B) - 1;
  Rx<C> r;
#pragma unroll
  for (int i = 0; i < L; ++i) {
    const int bit = i * B, w = bit / 32, sh = bit % 32;
    uint64_t lo = x.v[w];
    if (w + 1 < N) lo |= (uint64_t)x.v[w + 1] << 32;
    const uint32_t t = (uint32_t)(lo >> sh);
    r.v[i] = (i == L - 1) ? t : (t & MASK);
  }
  return r;
}

// limbs (normalised, value < 2^(32N)) -> packed N words
template <class C>
PLK_RX Fe<C> rx_pack(const Rx<C>& r) {
  constexpr int L = RxShape<C>::L, B = RxShape<C>::B, N = C::N;
  Fe<C> x;
#pragma unroll
  for (int w = 0; w < N; ++w) x.v[w] = 0;
#pragma unroll
  for (int i = 0; i < L; ++i) {
    const int bit = i * B, w = bit / 32, sh = bit % 32;
    const uint64_t val = (uint64_t)r.v[i] << sh;
    if (w < N) x.v[w] |= (uint32_t)val;
    if (w + 1 < N) x.v[w + 1] |= (uint32_t)(val >> 32);
  }
  return x;
}

// canonical packed value of a [0, 2p) element (R' domain kept)
template <class C>
PLK_RX Fe<C> rx_pack_canonical(const Rx<C>& r) {
  Fe<C> x = rx_pack(r);
  fe_reduce_once(x);
  return x;
}

// R-domain packed (ff.hpp, canonical) -> R'-domain packed canonical: times 2^(BL - 32N)
template <class C>
PLK_HD Fe<C> fe_to_rx_domain(Fe<C> x) {
  constexpr int SH = RxShape<C>::B * RxShape<C>::L - 32 * C::N;
#pragma unroll
  for (int i = 0; i < SH; ++i) x = fe_dbl(x);
  return x;
}

// ---- constant-operand (Shoup) product in Fr, for the NTT twiddles ----------------------
// x * w mod r for a constant w (canonical, plain — not Montgomery) with the precomputed
// w' = floor(w 2^261 / r): q = floor(x w' / 2^261) from the high columns only (7 .. 16 of
// the 18: the dropped ones are worth < 2^-23 of q, so q is exact or one low), then
// z = x w - q r computed mod 2^261 as x w + q (2^261 - r) in the low 9 columns. 53 + 45 + 45
// mads against Montgomery's 81 + 81, and no per-column digit multiply. x: limbs below 2^31,
// value below 2^261 (every NTT multiplicand); w, w' normalised. Output normalised, [0, 3r)
// (Shoup's [0, 2r) plus one r for the approximate q). Columns stay below 2^64: 9 products
// below 2^60 plus 9 below 2^58.
struct FrShoupK {
  uint32_t rbar[9];  // 2^261 - r
  uint32_t rinv[9];  // r^-1 mod 2^261
};
constexpr FrShoupK kFrShoup = {
    {0x1fffffffu, 0x7u, 0x690040u, 0x4b7fa00u, 0x27faac4u, 0x13fbfb2fu, 0xadf3318u, 0x159acc50u,
     0x1f8c1258u},
    {0x1u, 0x8u, 0x690080u, 0xb480000u, 0x113f9ac4u, 0x9f47ffdu, 0x1f1b9f93u, 0x9e5081au,
     0x1fc2bbc5u}};

PLK_RX Rx<FrCfg> fr_shoup(const Rx<FrCfg>& x, const Rx<FrCfg>& w, const Rx<FrCfg>& wp) {
  constexpr int L = 9, B = 29;
  constexpr uint32_t MASK = (1u << B) - 1;
  uint32_t q[L];
  uint64_t acc = 0;
#pragma unroll
  for (int k = 7; k < 2 * L - 1; ++k) {  // high columns of x w'
#pragma unroll
    for (int i = 0; i < L; ++i)
      if (k - i >= 0 && k - i < L) acc += (uint64_t)x.v[i] * wp.v[k - i];
    if (k >= L) q[k - L] = (uint32_t)acc & MASK;
    acc >>= B;
  }
  q[L - 1] = (uint32_t)acc;
  Rx<FrCfg> z;
  acc = 0;
#pragma unroll
  for (int k = 0; k < L; ++k) {  // low columns of x w + q (2^261 - r)
#pragma unroll
    for (int i = 0; i <= k; ++i) acc += (uint64_t)x.v[i] * w.v[k - i];
#pragma unroll
    for (int i = 0; i <= k; ++i) acc += (uint64_t)q[i] * kFrShoup.rbar[k - i];
    z.v[k] = (uint32_t)acc & MASK;
    acc >>= B;
  }
  return z;
}

// (w, w') from rho = w R' mod r (canonical, an R'-domain twiddle table entry): w = rho / R',
// brought to [0, r); w' = floor(w 2^261 / r) = (2^261 - rho) r^-1 mod 2^261, since
// w 2^261 = w' r + rho exactly.
PLK_RX void fr_shoup_prep(const Rx<FrCfg>& rho, Rx<FrCfg>& w, Rx<FrCfg>& wp) {
  constexpr int L = 9, B = 29;
  constexpr uint32_t MASK = (1u << B) - 1;
  Rx<FrCfg> one = rx_zero<FrCfg>();
  one.v[0] = 1;
  w = rx_unpack(rx_pack_canonical(rx_mul(rho, one)));
  // 2^261 - rho, normalised (rho < r < 2^261)
  Rx<FrCfg> n;
  int32_t br = 0;
#pragma unroll
  for (int i = 0; i < L; ++i) {
    const int32_t t = br - (int32_t)rho.v[i];
    n.v[i] = (uint32_t)t & MASK;
    br = t >> B;  // 0 or -1
  }
  // low 261 bits of n * rinv
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < L; ++k) {
#pragma unroll
    for (int i = 0; i <= k; ++i) acc += (uint64_t)n.v[i] * kFrShoup.rinv[k - i];
    wp.v[k] = (uint32_t)acc & MASK;
    acc >>= B;
  }
}

#undef PLK_RX

}  // namespace plk
