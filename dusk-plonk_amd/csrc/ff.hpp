// ff.hpp — BLS12-381 Fr (255-bit) and Fp (381-bit) Montgomery arithmetic for gfx950.
//
// Restates the field arithmetic of the un-vendored `bls-12-381` crate:
// Fr is 4x64 Montgomery with R = 2^256 (pinned by /root/reference/src/lib.rs:583-588),
// Fp is 6x64 Montgomery with R = 2^384. In registers we use 32-bit limbs (8 for Fr, 12
// for Fp): CDNA4 has no 64x64 multiplier, and the 32x32->64 `v_mad_u64_u32` is the
// natural building block. The memory image is identical to 4/6 little-endian u64 limbs,
// so the ABI layout (include/plk.h) is loaded without any conversion.
//
// Multiplication is CIOS with the "spare bit" shortcut: both moduli have their top
// 32-bit word below 2^31 - 1, so the running value never needs an (N+1)-th word and
// the result lands in [0, 2p) before one conditional subtraction. Every function
// returns canonical (fully reduced) values.
#pragma once
#include <stdint.h>
#include <string.h>
#if !defined(__HIP_DEVICE_COMPILE__) && defined(__x86_64__)
#include <immintrin.h>
#endif

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define PLK_HD __host__ __device__ __forceinline__
#else
#define PLK_HD inline
#endif

namespace plk {

struct FrCfg {
  static constexpr int N = 8;
  // r = 0x73eda753299d7d483339d80809a1d80553bda402fffe5bfeffffffff00000001
  static constexpr uint32_t P[8] = {0x00000001u, 0xffffffffu, 0xfffe5bfeu, 0x53bda402u,
                                    0x09a1d805u, 0x3339d808u, 0x299d7d48u, 0x73eda753u};
  static constexpr uint32_t INV = 0xffffffffu;  // -r^-1 mod 2^32
  static constexpr uint64_t INV64 = 0xfffffffeffffffffull;  // -r^-1 mod 2^64
  // R mod r  (Montgomery one)
  static constexpr uint32_t ONE[8] = {0xfffffffeu, 0x00000001u, 0x00034802u, 0x5884b7fau,
                                      0xecbc4ff5u, 0x998c4fefu, 0xacc5056fu, 0x1824b159u};
  // R^2 mod r
  static constexpr uint32_t R2[8] = {0xf3f29c6du, 0xc999e990u, 0x87925c23u, 0x2b6cedcbu,
                                     0x7254398fu, 0x05d31496u, 0x9f59ff11u, 0x0748d9d9u};
};

struct FpCfg {
  static constexpr int N = 12;
  static constexpr uint32_t P[12] = {0xffffaaabu, 0xb9feffffu, 0xb153ffffu, 0x1eabfffeu,
                                     0xf6b0f624u, 0x6730d2a0u, 0xf38512bfu, 0x64774b84u,
                                     0x434bacd7u, 0x4b1ba7b6u, 0x397fe69au, 0x1a0111eau};
  static constexpr uint32_t INV = 0xfffcfffdu;  // -p^-1 mod 2^32
  static constexpr uint64_t INV64 = 0x89f3fffcfffcfffdull;  // -p^-1 mod 2^64
  static constexpr uint32_t ONE[12] = {0x0002fffdu, 0x76090000u, 0xc40c0002u, 0xebf4000bu,
                                       0x53c758bau, 0x5f489857u, 0x70525745u, 0x77ce5853u,
                                       0xa256ec6du, 0x5c071a97u, 0xfa80e493u, 0x15f65ec3u};
  static constexpr uint32_t R2[12] = {0x1c341746u, 0xf4df1f34u, 0x09d104f1u, 0x0a76e6a6u,
                                      0x4c95b6d5u, 0x8de5476cu, 0x939d83c0u, 0x67eb88a9u,
                                      0xb519952du, 0x9a793e85u, 0x92cae3aau, 0x11988fe5u};
};

template <class C>
struct alignas(16) Fe {
  uint32_t v[C::N];
};

using Fr = Fe<FrCfg>;
using Fp = Fe<FpCfg>;

// ----------------------------------------------------------------------------- basics
template <class C>
PLK_HD Fe<C> fe_zero() {
  Fe<C> r;
#pragma unroll
  for (int i = 0; i < C::N; ++i) r.v[i] = 0;
  return r;
}

template <class C>
PLK_HD Fe<C> fe_one() {
  Fe<C> r;
#pragma unroll
  for (int i = 0; i < C::N; ++i) r.v[i] = C::ONE[i];
  return r;
}

template <class C>
PLK_HD bool fe_is_zero(const Fe<C>& a) {
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < C::N; ++i) acc |= a.v[i];
  return acc == 0;
}

template <class C>
PLK_HD bool fe_eq(const Fe<C>& a, const Fe<C>& b) {
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < C::N; ++i) acc |= a.v[i] ^ b.v[i];
  return acc == 0;
}

// r = a - p if a >= p else a (a < 2p)
template <class C>
PLK_HD void fe_reduce_once(Fe<C>& a) {
  uint32_t d[C::N];
  uint32_t borrow = 0;
#pragma unroll
  for (int i = 0; i < C::N; ++i) {
    uint64_t t = (uint64_t)a.v[i] - C::P[i] - borrow;
    d[i] = (uint32_t)t;
    borrow = (uint32_t)(t >> 63);
  }
  // borrow == 1  <=>  a < p  -> keep a
#pragma unroll
  for (int i = 0; i < C::N; ++i) a.v[i] = borrow ? a.v[i] : d[i];
}

template <class C>
PLK_HD Fe<C> fe_add(const Fe<C>& a, const Fe<C>& b) {
  Fe<C> r;
  uint32_t carry = 0;
#pragma unroll
  for (int i = 0; i < C::N; ++i) {
    uint64_t t = (uint64_t)a.v[i] + b.v[i] + carry;
    r.v[i] = (uint32_t)t;
    carry = (uint32_t)(t >> 32);
  }
  // both moduli leave a spare top bit, so a + b < 2p < 2^(32N): no carry out
  fe_reduce_once(r);
  return r;
}

template <class C>
PLK_HD Fe<C> fe_sub(const Fe<C>& a, const Fe<C>& b) {
  Fe<C> r;
  uint32_t borrow = 0;
#pragma unroll
  for (int i = 0; i < C::N; ++i) {
    uint64_t t = (uint64_t)a.v[i] - b.v[i] - borrow;
    r.v[i] = (uint32_t)t;
    borrow = (uint32_t)(t >> 63);
  }
  // if it went negative, add p back
  uint32_t mask = 0u - borrow;
  uint32_t carry = 0;
#pragma unroll
  for (int i = 0; i < C::N; ++i) {
    uint64_t t = (uint64_t)r.v[i] + (C::P[i] & mask) + carry;
    r.v[i] = (uint32_t)t;
    carry = (uint32_t)(t >> 32);
  }
  return r;
}

template <class C>
PLK_HD Fe<C> fe_neg(const Fe<C>& a) {
  return fe_sub(fe_zero<C>(), a);
}

template <class C>
PLK_HD Fe<C> fe_dbl(const Fe<C>& a) {
  return fe_add(a, a);
}

#if !defined(__HIP_DEVICE_COMPILE__)
// Host path: the same Montgomery product on 64-bit limbs (identical memory image). The
// host only runs the MSM's short serial tail and table set-up, where latency matters.
template <class C>
inline Fe<C> fe_mul_host64(const Fe<C>& a, const Fe<C>& b) {
  constexpr int M = C::N / 2;
  uint64_t A[M], B[M], P[M], t[M];
  for (int i = 0; i < M; ++i) {
    A[i] = (uint64_t)a.v[2 * i] | ((uint64_t)a.v[2 * i + 1] << 32);
    B[i] = (uint64_t)b.v[2 * i] | ((uint64_t)b.v[2 * i + 1] << 32);
    P[i] = (uint64_t)C::P[2 * i] | ((uint64_t)C::P[2 * i + 1] << 32);
    t[i] = 0;
  }
  for (int i = 0; i < M; ++i) {
    unsigned __int128 c = 0;
    for (int j = 0; j < M; ++j) {
      c += (unsigned __int128)A[j] * B[i] + t[j];
      t[j] = (uint64_t)c;
      c >>= 64;
    }
    const uint64_t tn = (uint64_t)c;
    const uint64_t m = t[0] * C::INV64;
    c = (unsigned __int128)m * P[0] + t[0];
    c >>= 64;
    for (int j = 1; j < M; ++j) {
      c += (unsigned __int128)m * P[j] + t[j];
      t[j - 1] = (uint64_t)c;
      c >>= 64;
    }
    t[M - 1] = tn + (uint64_t)c;
  }
  Fe<C> r;
  for (int i = 0; i < M; ++i) {
    r.v[2 * i] = (uint32_t)t[i];
    r.v[2 * i + 1] = (uint32_t)(t[i] >> 32);
  }
  fe_reduce_once(r);
  return r;
}

#if defined(__x86_64__) && !defined(__HIP_DEVICE_COMPILE__)
// The same CIOS product with BMI2/ADX (mulx + add-with-carry intrinsics) on the native
// 64-bit image of the limbs: ~27% lower latency than the __int128 form. The composer's
// witness arithmetic (serial by nature: gate outputs feed the next gate) runs on this.
template <class C>
__attribute__((target("bmi2,adx"))) inline Fe<C> fe_mul_host_adx(const Fe<C>& a, const Fe<C>& b) {
  constexpr int M = C::N / 2;
  typedef unsigned long long u64;
  u64 A[M], Bw[M], P[M], t[M + 2];
#pragma unroll
  for (int i = 0; i < M; ++i) {
    A[i] = (u64)a.v[2 * i] | ((u64)a.v[2 * i + 1] << 32);
    Bw[i] = (u64)b.v[2 * i] | ((u64)b.v[2 * i + 1] << 32);
  }
#pragma unroll
  for (int i = 0; i < M; ++i) P[i] = (u64)C::P[2 * i] | ((u64)C::P[2 * i + 1] << 32);
#pragma unroll
  for (int i = 0; i < M + 2; ++i) t[i] = 0;
#pragma unroll
  for (int i = 0; i < M; ++i) {
    u64 lo[M], hi[M];
#pragma unroll
    for (int j = 0; j < M; ++j) lo[j] = _mulx_u64(A[j], Bw[i], &hi[j]);
    unsigned char c = 0;
#pragma unroll
    for (int j = 0; j < M; ++j) c = _addcarry_u64(c, t[j], lo[j], &t[j]);
    _addcarry_u64(c, t[M], 0, &t[M]);
    c = 0;
#pragma unroll
    for (int j = 0; j < M; ++j) c = _addcarry_u64(c, t[j + 1], hi[j], &t[j + 1]);
    t[M + 1] = c;
    const u64 m = t[0] * C::INV64;
#pragma unroll
    for (int j = 0; j < M; ++j) lo[j] = _mulx_u64(m, P[j], &hi[j]);
    c = 0;
#pragma unroll
    for (int j = 0; j < M; ++j) c = _addcarry_u64(c, t[j], lo[j], &t[j]);
    c = _addcarry_u64(c, t[M], 0, &t[M]);
    t[M + 1] += c;
    c = 0;
#pragma unroll
    for (int j = 0; j < M; ++j) c = _addcarry_u64(c, t[j + 1], hi[j], &t[j]);
    t[M] = t[M + 1] + c;
    t[M + 1] = 0;
  }
  u64 s[M];
  unsigned char br = 0;
  for (int j = 0; j < M; ++j) br = _subborrow_u64(br, t[j], P[j], &s[j]);
  Fe<C> r;  // spare bit: t < 2p
#pragma unroll
  for (int j = 0; j < M; ++j) {
    const u64 w = br ? t[j] : s[j];
    r.v[2 * j] = (uint32_t)w;
    r.v[2 * j + 1] = (uint32_t)(w >> 32);
  }
  return r;
}
#endif
#endif

#if defined(__HIP_DEVICE_COMPILE__)
// ---- gfx950 product-scanning Montgomery multiplication -----------------------------
// (acc, top) is a 96-bit column accumulator: acc = VGPR pair, top = carries past 2^64.
// One product = v_mad_u64_u32 (acc += a*b, carry-out to an SGPR pair) + v_addc_co_u32
// (top += carry): two instructions, where the compiler's CIOS lowering needs ~4.4.
__device__ __forceinline__ void mac96(uint64_t& acc, uint32_t& top, uint32_t a, uint32_t b) {
  uint64_t cy;
  asm("v_mad_u64_u32 %0, %2, %3, %4, %0\n\t"
      "v_addc_co_u32_e64 %1, %2, 0, %1, %2"
      : "+v"(acc), "+v"(top), "=&s"(cy)
      : "v"(a), "v"(b));
}

// same with the second factor a wave-uniform constant (modulus limb) in an SGPR
__device__ __forceinline__ void mac96s(uint64_t& acc, uint32_t& top, uint32_t a, uint32_t b) {
  uint64_t cy;
  asm("v_mad_u64_u32 %0, %2, %3, %4, %0\n\t"
      "v_addc_co_u32_e64 %1, %2, 0, %1, %2"
      : "+v"(acc), "+v"(top), "=&s"(cy)
      : "v"(a), "s"(b));
}

// one product on each of two independent chains in a single asm block (A: both factors
// in VGPRs, B: second factor a modulus limb in an SGPR)
__device__ __forceinline__ void mac96x2(uint64_t& acc, uint32_t& top, uint32_t a, uint32_t b,
                                        uint64_t& acc2, uint32_t& top2, uint32_t a2, uint32_t b2) {
  uint64_t cy, cy2;
  asm("v_mad_u64_u32 %0, %4, %6, %7, %0\n\t"
      "v_mad_u64_u32 %2, %5, %8, %9, %2\n\t"
      "v_addc_co_u32_e64 %1, %4, 0, %1, %4\n\t"
      "v_addc_co_u32_e64 %3, %5, 0, %3, %5"
      : "+v"(acc), "+v"(top), "+v"(acc2), "+v"(top2), "=&s"(cy), "=&s"(cy2)
      : "v"(a), "v"(b), "v"(a2), "s"(b2));
}

// Montgomery product by columns (FIPS / "Comba-Montgomery"): column k accumulates
// sum a_i b_{k-i} (chain A) and sum m_i p_{k-i} (chain B, independent of A; the two are
// interleaved so consecutive v_mad_u64_u32 never depend on each other), then
// m_k = lo * -p^-1 zeroes the low word for k < N; words N..2N-1 are the result (< 2p).
template <class C>
__device__ __forceinline__ Fe<C> fe_mul_dev(const Fe<C>& a, const Fe<C>& b) {
  constexpr int N = C::N;
  uint32_t m[N];
  Fe<C> r;
  uint64_t acc = 0;
  uint32_t top = 0;
#pragma unroll
  for (int k = 0; k < 2 * N - 1; ++k) {
    const int lo_i = k < N ? 0 : k - N + 1;
    const int hi_a = k < N ? k : N - 1;
    const int hi_m = k < N ? k - 1 : N - 1;
    uint64_t accb = 0;
    uint32_t topb = 0;
#pragma unroll
    for (int i = lo_i; i <= hi_a; ++i) {
      if (i <= hi_m)
        mac96x2(acc, top, a.v[i], b.v[k - i], accb, topb, m[i], C::P[k - i]);
      else
        mac96(acc, top, a.v[i], b.v[k - i]);
    }
    if (hi_m >= lo_i) {  // merge chain B into A (64-bit add, carry into top)
      const uint64_t sum = acc + accb;
      top += topb + (sum < accb ? 1u : 0u);
      acc = sum;
    }
    if (k < N) {
      m[k] = (uint32_t)acc * C::INV;
      mac96s(acc, top, m[k], C::P[0]);
    } else {
      r.v[k - N] = (uint32_t)acc;
    }
    acc = (acc >> 32) | ((uint64_t)top << 32);
    top = 0;
  }
  r.v[N - 1] = (uint32_t)acc;
  fe_reduce_once(r);
  return r;
}
#endif

// Montgomery product a*b*R^-1 mod p (CIOS, spare-bit form). The device build uses the
// product-scanning form above; fe_mul_cios is kept as the portable reference lowering.
template <class C>
PLK_HD Fe<C> fe_mul(const Fe<C>& a, const Fe<C>& b) {
#if !defined(__HIP_DEVICE_COMPILE__) && defined(__x86_64__)
  return fe_mul_host_adx(a, b);
#elif !defined(__HIP_DEVICE_COMPILE__)
  return fe_mul_host64(a, b);
#else
  return fe_mul_dev(a, b);
#endif
}

template <class C>
PLK_HD Fe<C> fe_mul_cios(const Fe<C>& a, const Fe<C>& b) {
#if !defined(__HIP_DEVICE_COMPILE__)
  return fe_mul_host64(a, b);
#else
  constexpr int N = C::N;
  uint32_t t[N];
#pragma unroll
  for (int j = 0; j < N; ++j) t[j] = 0;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const uint32_t bi = b.v[i];
    uint64_t c = 0;
#pragma unroll
    for (int j = 0; j < N; ++j) {
      uint64_t s = (uint64_t)a.v[j] * bi + t[j] + c;
      t[j] = (uint32_t)s;
      c = s >> 32;
    }
    const uint32_t tn = (uint32_t)c;
    const uint32_t m = t[0] * C::INV;
    uint64_t s = (uint64_t)m * C::P[0] + t[0];
    c = s >> 32;
#pragma unroll
    for (int j = 1; j < N; ++j) {
      s = (uint64_t)m * C::P[j] + t[j] + c;
      t[j - 1] = (uint32_t)s;
      c = s >> 32;
    }
    t[N - 1] = tn + (uint32_t)c;
  }
  Fe<C> r;
#pragma unroll
  for (int j = 0; j < N; ++j) r.v[j] = t[j];
  fe_reduce_once(r);
  return r;
#endif
}

template <class C>
PLK_HD Fe<C> fe_sqr(const Fe<C>& a) {
  return fe_mul(a, a);
}

template <class C>
PLK_HD Fe<C> fe_to_mont(const Fe<C>& a) {
  Fe<C> r2;
#pragma unroll
  for (int i = 0; i < C::N; ++i) r2.v[i] = C::R2[i];
  return fe_mul(a, r2);
}

template <class C>
PLK_HD Fe<C> fe_from_mont(const Fe<C>& a) {
  Fe<C> one = fe_zero<C>();
  one.v[0] = 1;
  return fe_mul(a, one);
}

// a^e for a little-endian exponent of `words` 32-bit words (square-and-multiply, MSB first)
template <class C>
PLK_HD Fe<C> fe_pow(const Fe<C>& a, const uint32_t* e, int words) {
  Fe<C> r = fe_one<C>();
  for (int w = words - 1; w >= 0; --w) {
    for (int b = 31; b >= 0; --b) {
      r = fe_sqr(r);
      if ((e[w] >> b) & 1u) r = fe_mul(r, a);
    }
  }
  return r;
}

// a^e, square-and-multiply over the significant bits of e only
template <class C>
PLK_HD Fe<C> fe_pow_u64(const Fe<C>& a, uint64_t e) {
  Fe<C> r = fe_one<C>();
  if (e == 0) return r;
  int b = 63;
  while (!((e >> b) & 1ull)) --b;
  r = a;
  for (--b; b >= 0; --b) {
    r = fe_sqr(r);
    if ((e >> b) & 1ull) r = fe_mul(r, a);
  }
  return r;
}

// Fermat inversion a^(p-2); inverse of zero is zero.
template <class C>
PLK_HD Fe<C> fe_inv(const Fe<C>& a) {
  uint32_t e[C::N];
  uint32_t borrow = 2;
#pragma unroll
  for (int i = 0; i < C::N; ++i) {
    uint64_t t = (uint64_t)C::P[i] - borrow;
    e[i] = (uint32_t)t;
    borrow = (uint32_t)(t >> 63);
  }
  return fe_pow(a, e, C::N);
}

}  // namespace plk
