// ubench_limbs.hip — prototype of a redundant-limb Montgomery product for gfx950 and its
// throughput against the packed 32-bit product-scanning multiply in ff.hpp.
//
// Representation: L limbs of B bits held in 32-bit words (Fp: 14 x 28, Fr: 9 x 29), radix
// R' = 2^(B*L). Every partial product is < 2^(2B), so a whole column (at most 2L products
// plus the carry) fits one 64-bit accumulator: each product is ONE v_mad_u64_u32 with no
// carry chain, where the packed form needs mad + addc. Output is "almost Montgomery" in
// [0, 2p) since 4p < R' (no final subtraction).
//
// Correctness check: for random Montgomery-384/256 a, b: a' = a * 2^(B*L - 32*N) (i.e.
// doubling), c' = mul(a', b'), and c' must equal fe_mul(a, b) * 2^(B*L - 32*N) mod p.
// Build: hipcc -O3 --offload-arch=gfx950 tools/ubench_limbs.hip -o tools/ubench_limbs
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#include "../dusk-plonk_amd/csrc/ff.hpp"

using namespace plk;

#define CHECK(x)                                                                      \
  do {                                                                                \
    hipError_t e = (x);                                                               \
    if (e != hipSuccess) {                                                            \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));   \
      return 1;                                                                       \
    }                                                                                 \
  } while (0)

template <class C, int L_, int B_>
struct Red {
  static constexpr int L = L_, B = B_;
  static constexpr uint32_t MASK = (1u << B) - 1;
  static constexpr int SHIFT = B * L - 32 * C::N;  // R' / R = 2^SHIFT
  uint32_t v[L];
};

template <class C, int L, int B>
struct RedCfg {
  uint32_t p[L];
  uint32_t inv;  // -p^-1 mod 2^B
};

template <class C, int L, int B>
__host__ __device__ constexpr RedCfg<C, L, B> make_cfg() {
  RedCfg<C, L, B> c{};
  for (int i = 0; i < L; ++i) {
    uint32_t x = 0;
    for (int k = 0; k < B; ++k) {
      const int bit = i * B + k;
      if (bit < 32 * C::N && ((C::P[bit / 32] >> (bit % 32)) & 1u)) x |= 1u << k;
    }
    c.p[i] = x;
  }
  // inverse of p mod 2^B by Newton iteration, then negate
  uint32_t y = 1;
  for (int k = 0; k < 6; ++k) y = y * (2u - C::P[0] * y);
  c.inv = (0u - y) & ((1u << B) - 1);
  return c;
}

template <class C, int L, int B>
__device__ __forceinline__ void red_mul(uint32_t* r, const uint32_t* a, const uint32_t* b) {
  constexpr RedCfg<C, L, B> K = make_cfg<C, L, B>();
  constexpr uint32_t MASK = (1u << B) - 1;
  uint32_t m[L];
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < L; ++k) {
#pragma unroll
    for (int i = 0; i <= k; ++i) acc += (uint64_t)a[i] * b[k - i];
#pragma unroll
    for (int i = 0; i < k; ++i) acc += (uint64_t)m[i] * K.p[k - i];
    m[k] = ((uint32_t)acc * K.inv) & MASK;
    acc += (uint64_t)m[k] * K.p[0];
    acc >>= B;
  }
#pragma unroll
  for (int k = L; k < 2 * L - 1; ++k) {
#pragma unroll
    for (int i = k - L + 1; i < L; ++i) acc += (uint64_t)a[i] * b[k - i];
#pragma unroll
    for (int i = k - L + 1; i < L; ++i) acc += (uint64_t)m[i] * K.p[k - i];
    r[k - L] = (uint32_t)acc & MASK;
    acc >>= B;
  }
  r[L - 1] = (uint32_t)acc;
}

// Round 3 A/B: 13 x 30-bit Fp limbs, 169 + 169 mads per product instead
// of 196 + 196. Columns no longer fit one 64-bit accumulator (up to 26 terms below 2^60), so
// every column whose worst-case sum could reach 2^64 keeps the products and the reduction
// terms in two accumulators and merges their low B bits and carries (bounds computed at
// compile time from the limb bounds: inputs < 2^(32N) so the top limb has 32N - B(L-1) bits,
// p's top limb fewer).
template <class C, int L, int B>
struct SplitPlan {
  bool split[2 * L - 1];
  constexpr SplitPlan() : split{} {
    constexpr RedCfg<C, L, B> K = make_cfg<C, L, B>();
    const int top_bits = 32 * C::N - B * (L - 1);
    long double carry = 0;  // bound of the incoming carry
    for (int k = 0; k < 2 * L - 1; ++k) {
      long double sum = carry;
      for (int i = 0; i < L; ++i) {
        const int j = k - i;
        if (j < 0 || j >= L) continue;
        const long double ai = (i == L - 1) ? (long double)(1ull << top_bits) : (long double)(1ull << B);
        const long double bj = (j == L - 1) ? (long double)(1ull << top_bits) : (long double)(1ull << B);
        sum += ai * bj;                                    // a_i b_j
        sum += (long double)(1ull << B) * (long double)(K.p[j] + 1);  // m_i p_j
      }
      split[k] = sum >= 18446744073709551616.0L;
      carry = sum / (long double)(1ull << B) + 2;
    }
  }
};

template <class C, int L, int B>
__device__ __forceinline__ void red_mul_split(uint32_t* r, const uint32_t* a, const uint32_t* b) {
  constexpr RedCfg<C, L, B> K = make_cfg<C, L, B>();
  constexpr SplitPlan<C, L, B> S{};
  constexpr uint32_t MASK = (1u << B) - 1;
  uint32_t m[L];
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 2 * L - 1; ++k) {
    const int i0 = k < L ? 0 : k - L + 1, i1 = k < L ? k : L - 1;
    if (!S.split[k]) {
#pragma unroll
      for (int i = i0; i <= i1; ++i) acc += (uint64_t)a[i] * b[k - i];
#pragma unroll
      for (int i = i0; i <= i1; ++i)
        if (i < k || k >= L) acc += (uint64_t)m[i] * K.p[k - i];
      if (k < L) {
        m[k] = ((uint32_t)acc * K.inv) & MASK;
        acc += (uint64_t)m[k] * K.p[0];
      } else {
        r[k - L] = (uint32_t)acc & MASK;
      }
      acc >>= B;
    } else {
      uint64_t s2 = 0;
#pragma unroll
      for (int i = i0; i <= i1; ++i) acc += (uint64_t)a[i] * b[k - i];
#pragma unroll
      for (int i = i0; i <= i1; ++i)
        if (i < k || k >= L) s2 += (uint64_t)m[i] * K.p[k - i];
      uint64_t lo = (uint64_t)(((uint32_t)acc & MASK) + ((uint32_t)s2 & MASK));
      const uint64_t hi = (acc >> B) + (s2 >> B);
      if (k < L) {
        m[k] = ((uint32_t)lo * K.inv) & MASK;
        lo += (uint64_t)m[k] * K.p[0];
      } else {
        r[k - L] = (uint32_t)lo & MASK;
      }
      acc = hi + (lo >> B);
    }
  }
  r[L - 1] = (uint32_t)acc;
}

template <class C, int L, int B>
__device__ void unpack(uint32_t* r, const Fe<C>& x) {
#pragma unroll
  for (int i = 0; i < L; ++i) {
    const int bit = i * B, w = bit / 32, sh = bit % 32;
    uint64_t lo = x.v[w];
    if (w + 1 < C::N) lo |= (uint64_t)x.v[w + 1] << 32;
    r[i] = (uint32_t)(lo >> sh) & ((1u << B) - 1);
  }
}

template <class C, int L, int B>
__device__ Fe<C> pack_reduce(const uint32_t* r) {
  // normalise carries, then pack to 32-bit words (value < 2p < 2^(32N)) and reduce once
  uint32_t t[L];
  uint32_t carry = 0;
#pragma unroll
  for (int i = 0; i < L; ++i) {
    const uint64_t s = (uint64_t)r[i] + carry;
    t[i] = (uint32_t)s & ((1u << B) - 1);
    carry = (uint32_t)(s >> B);
  }
  Fe<C> x;
#pragma unroll
  for (int w = 0; w < C::N; ++w) x.v[w] = 0;
#pragma unroll
  for (int i = 0; i < L; ++i) {
    const int bit = i * B, w = bit / 32, sh = bit % 32;
    const uint64_t val = (uint64_t)t[i] << sh;
    if (w < C::N) x.v[w] |= (uint32_t)val;
    if (w + 1 < C::N) x.v[w + 1] |= (uint32_t)(val >> 32);
  }
  fe_reduce_once(x);
  return x;
}

template <class C>
__device__ Fe<C> dbl_n(Fe<C> x, int n) {
  for (int i = 0; i < n; ++i) x = fe_dbl(x);
  return x;
}

template <class C, int L, int B, bool SPLIT = false>
__global__ void k_check(const Fe<C>* a, const Fe<C>* b, uint32_t n, uint32_t* bad) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  constexpr int SH = B * L - 32 * C::N;
  const Fe<C> c = fe_mul(a[t], b[t]);
  uint32_t ar[L], br[L], cr[L];
  unpack<C, L, B>(ar, dbl_n(a[t], SH));
  unpack<C, L, B>(br, dbl_n(b[t], SH));
  if (SPLIT) red_mul_split<C, L, B>(cr, ar, br);
  else red_mul<C, L, B>(cr, ar, br);
  const Fe<C> got = pack_reduce<C, L, B>(cr);
  if (!fe_eq(got, dbl_n(c, SH))) atomicAdd(bad, 1u);
}

template <class C, int L, int B, int CHAINS, bool SPLIT = false>
__global__ void __launch_bounds__(256) k_red_thr(uint32_t* io, uint32_t iters) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t x[CHAINS][L], y[L];
#pragma unroll
  for (int i = 0; i < L; ++i) y[i] = (io[t * L + i] + i) & ((1u << B) - 1);
#pragma unroll
  for (int c = 0; c < CHAINS; ++c)
#pragma unroll
    for (int i = 0; i < L; ++i) x[c][i] = y[i] ^ c;
  for (uint32_t it = 0; it < iters; ++it) {
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) {
      if (SPLIT) red_mul_split<C, L, B>(x[c], x[c], y);
      else red_mul<C, L, B>(x[c], x[c], y);
    }
  }
#pragma unroll
  for (int i = 0; i < L; ++i) {
    uint32_t s = 0;
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) s ^= x[c][i];
    io[t * L + i] = s;
  }
}

template <class C, int CHAINS>
__global__ void __launch_bounds__(256) k_packed_thr(Fe<C>* io, uint32_t iters) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  Fe<C> x[CHAINS], y = io[t];
#pragma unroll
  for (int i = 0; i < CHAINS; ++i) {
    x[i] = y;
    x[i].v[0] ^= i;
  }
  for (uint32_t it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < CHAINS; ++i) x[i] = fe_mul(x[i], y);
  }
  Fe<C> s = x[0];
#pragma unroll
  for (int i = 1; i < CHAINS; ++i) s = fe_add(s, x[i]);
  io[t] = s;
}

static uint64_t g_state = 0x1234567;
static uint32_t rnd32() {
  g_state += 0x9E3779B97F4A7C15ull;
  uint64_t z = g_state;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return (uint32_t)(z ^ (z >> 31));
}

template <class C, int L, int B, bool SPLIT = false>
int check(const char* name) {
  const uint32_t n = 1 << 16;
  std::vector<Fe<C>> ha(n), hb(n);
  for (uint32_t i = 0; i < n; ++i) {
    for (int k = 0; k < C::N; ++k) {
      ha[i].v[k] = rnd32();
      hb[i].v[k] = rnd32();
    }
    ha[i].v[C::N - 1] &= C::P[C::N - 1] >> 1;  // < p
    hb[i].v[C::N - 1] &= C::P[C::N - 1] >> 1;
  }
  // edge values: 0, 1, p-1
  for (int k = 0; k < C::N; ++k) {
    ha[0].v[k] = 0;
    hb[1].v[k] = C::P[k];
    ha[2].v[k] = C::P[k];
    hb[2].v[k] = C::P[k];
  }
  hb[1].v[0] -= 1;
  ha[2].v[0] -= 1;
  hb[2].v[0] -= 1;
  Fe<C>*da, *db;
  uint32_t* dbad;
  CHECK(hipMalloc(&da, n * sizeof(Fe<C>)));
  CHECK(hipMalloc(&db, n * sizeof(Fe<C>)));
  CHECK(hipMalloc(&dbad, 4));
  CHECK(hipMemset(dbad, 0, 4));
  CHECK(hipMemcpy(da, ha.data(), n * sizeof(Fe<C>), hipMemcpyHostToDevice));
  CHECK(hipMemcpy(db, hb.data(), n * sizeof(Fe<C>), hipMemcpyHostToDevice));
  hipLaunchKernelGGL((k_check<C, L, B, SPLIT>), dim3(n / 256), dim3(256), 0, 0, da, db, n, dbad);
  uint32_t bad = 0;
  CHECK(hipMemcpy(&bad, dbad, 4, hipMemcpyDeviceToHost));
  std::printf("{\"test\":\"%s_check\",\"cases\":%u,\"mismatches\":%u}\n", name, n, bad);
  CHECK(hipFree(da));
  CHECK(hipFree(db));
  CHECK(hipFree(dbad));
  return bad != 0;
}

template <class C, int L, int B, int CHAINS, bool SPLIT = false>
int thr(const char* name, uint32_t blocks, uint32_t iters) {
  const uint32_t total = blocks * 256;
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  float ms;
  uint32_t* io;
  CHECK(hipMalloc(&io, (size_t)total * L * 4));
  CHECK(hipMemset(io, 0x11, (size_t)total * L * 4));
  hipLaunchKernelGGL((k_red_thr<C, L, B, CHAINS, SPLIT>), dim3(blocks), dim3(256), 0, 0, io, 4);
  CHECK(hipEventRecord(e0));
  hipLaunchKernelGGL((k_red_thr<C, L, B, CHAINS, SPLIT>), dim3(blocks), dim3(256), 0, 0, io, iters);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  const double red = (double)total * iters * CHAINS / (ms * 1e-3);
  Fe<C>* io2;
  CHECK(hipMalloc(&io2, (size_t)total * sizeof(Fe<C>)));
  CHECK(hipMemset(io2, 0x11, (size_t)total * sizeof(Fe<C>)));
  hipLaunchKernelGGL((k_packed_thr<C, CHAINS>), dim3(blocks), dim3(256), 0, 0, io2, 4);
  CHECK(hipEventRecord(e0));
  hipLaunchKernelGGL((k_packed_thr<C, CHAINS>), dim3(blocks), dim3(256), 0, 0, io2, iters);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  const double packed = (double)total * iters * CHAINS / (ms * 1e-3);
  std::printf("{\"test\":\"%s_mul\",\"redundant_per_s\":%.4e,\"packed_per_s\":%.4e,\"speedup\":%.3f}\n",
              name, red, packed, red / packed);
  CHECK(hipFree(io));
  CHECK(hipFree(io2));
  return 0;
}

int main() {
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  int bad = 0;
  bad |= check<FpCfg, 14, 28>("fp14x28");
  bad |= check<FrCfg, 9, 29>("fr9x29");
  bad |= check<FpCfg, 13, 30, true>("fp13x30split");
  thr<FpCfg, 14, 28, 2>("fp14x28", cus * 8, 256);
  thr<FpCfg, 13, 30, 2, true>("fp13x30split", cus * 8, 256);
  thr<FrCfg, 9, 29, 4>("fr9x29", cus * 8, 512);
  return bad;
}
