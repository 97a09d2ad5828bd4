// ffr.hpp — redundant-limb Montgomery arithmetic for the gfx950 hot loops (device only).
//
// ff.hpp stores a field element as N packed 32-bit words and multiplies with a 96-bit
// column accumulator: every 32x32 partial product costs v_mad_u64_u32 + v_addc (plus the
// s_nop padding the compiler puts around inline asm). Here an element is L limbs of B < 32
// bits (Fp: 14 x 28, Fr: 9 x 29) so that a whole product-scanning column — at most 2L
// products below 2^(2B) plus the incoming carry — fits one 64-bit accumulator: ONE
// v_mad_u64_u32 per partial product, no carry chain, plain C the scheduler can interleave.
// Measured on MI355X (tools/ubench_limbs.hip): Fp 6.9e10 mul/s vs 4.8e10 packed, Fr 1.64e11
// vs 1.09e11.
//
// Domain: Montgomery with R' = 2^(B*L) (Fp 2^392, Fr 2^261), values kept in [0, 2p) with
// normalised limbs (4p < R', so the product needs no final subtraction). Memory keeps the
// packed layout of ff.hpp (2p < 2^(32N)): kernels unpack on load and pack on store, and a
// buffer holds either R-domain (ff.hpp) or R'-domain values — each buffer's comment says
// which. Conversion R -> R' is a multiplication by 2^(B*L - 32N) (doublings); R' -> R by
// 2^-(B*L - 32N).
#pragma once
#include "ff.hpp"

namespace plk {

template <class C>
struct RxShape;
template <>
struct RxShape<FpCfg> {
  static constexpr int L = 14, B = 28;
  static constexpr uint32_t ONE[12] = {0x0347fcb8u, 0x19d80000u, 0x6d2002b1u, 0x12e00cdeu,
                                       0xa2090c72u, 0x37669f83u, 0xda0f73e0u, 0x09b09b42u,
                                       0x8f1297bbu, 0xa7c515d9u, 0xfcfa012cu, 0x0577a659u};  // 2^392 mod p
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

#define PLK_RX __device__ __forceinline__

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
  r.v[L - 1] = (uint32_t)acc;
  return r;
}

// (a*b + c*d) / R' mod p with ONE Montgomery reduction: both product columns accumulate
// into the same 64-bit column (the caller bounds the limbs so that 2L products plus L
// reduction products stay below 2^64, and the value so that (ab + cd) / R' + p < 2p).
template <class C>
PLK_RX Rx<C> rx_mul_add(const Rx<C>& a, const Rx<C>& b, const Rx<C>& c, const Rx<C>& d) {
  constexpr int L = RxShape<C>::L, B = RxShape<C>::B;
  constexpr uint32_t MASK = (1u << B) - 1;
  constexpr RxConst<C> K = RxK<C>::k;
  uint32_t m[L];
  Rx<C> r;
  uint64_t acc = 0;
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
  r.v[L - 1] = (uint32_t)acc;
  return r;
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
// operands (Fp: a 64-bit column of 14 products below 2^60 plus 14 reduction products below
// 2^56 stays under 2^64; the output (12p)^2 / R' + p < 2p, normalised).
template <class C, uint32_t CP>
PLK_RX Rx<C> rx_sub_u(const Rx<C>& a, const Rx<C>& b) {
  constexpr RxMultiple<C> Q = RxMultipleK<C, CP, true>::k;
  Rx<C> r;
#pragma unroll
  for (int i = 0; i < RxShape<C>::L; ++i) r.v[i] = a.v[i] + Q.v[i] - b.v[i];
  return r;
}

// a + c*p - b with the carries propagated (signed): normalised limbs, value in
// (c*p - max b, c*p + max a) — no conditional pass
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

// a + c*p - b - 2e, carries propagated (the X3 of the XYZZ addition in one pass)
template <class C, uint32_t CP>
PLK_RX Rx<C> rx_sub2_n(const Rx<C>& a, const Rx<C>& b, const Rx<C>& e) {
  constexpr int L = RxShape<C>::L, B = RxShape<C>::B;
  constexpr uint32_t MASK = (1u << B) - 1;
  constexpr RxMultiple<C> Q = RxMultipleK<C, CP, false>::k;
  Rx<C> d;
  int32_t c = 0;
#pragma unroll
  for (int i = 0; i < L; ++i) {
    const int32_t t =
        (int32_t)(a.v[i] + Q.v[i]) - (int32_t)b.v[i] - (int32_t)(e.v[i] << 1) + c;
    d.v[i] = i == L - 1 ? (uint32_t)t : ((uint32_t)t & MASK);
    c = t >> B;
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

// a (any value < 16p, limbs < 2^(B+2)) reduced to [0, 2p), normalised: a * R' / R'
template <class C>
PLK_RX Rx<C> rx_canon(const Rx<C>& a) {
  return rx_mul(a, rx_one<C>());
}

// a == 0 mod p for a value < 16p with limbs < 2^(B+2): (a / R') is in [0, 2p)
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

#undef PLK_RX

}  // namespace plk
