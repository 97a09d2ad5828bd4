// ntt.hip — BLS12-381 Fr NTT family on gfx950: Fft::{dft, idft, coset_dft, coset_idft}.
//
// Reference semantics (poly_commit::Fft, un-vendored): natural order
// in and out, w = ROOT_OF_UNITY^(2^(32-k)), elements[i] = w^i (permutation.rs:148),
// idft scaled by n^-1, cosets over g*H with g = 7 (quotient_poly.rs:54-58,115).
//
// Algorithm: self-sorting (Stockham) decomposition into P passes of radix R = 2^lr.
// A pass reads the R inputs x[i + j*N/R] (j < R) of T consecutive i (coalesced T-wide
// column groups), applies the inter-pass twiddle w_{Rp}^{jk} (k = i mod p), runs the
// R-point sub-DFT in LDS (radix-2 DIF stages, twiddles staged in LDS), and writes
// Y[k + m p] of each length-Rp sub-transform to (i-k)*R + k + m*p. No bit-reversal pass
// is needed: the last pass leaves natural order. The coset pre-scale g^e is fused into
// the first pass' loads, zero padding (len_in < n) into the same loads, and the n^-1
// (or n^-1 g^-e) post-scale into the last pass' stores.
//
// HBM traffic per transform: P * 2 * N * 32 B (P = 3 at N = 2^20..2^24).
#include <cstdlib>
#include <type_traits>

#include "ffr.hpp"
#include "internal.hpp"

namespace plk {

namespace {

constexpr uint32_t kMaxLr = 9;   // radix up to 512 (PLK_NTT_MAX_LR: up to kMaxLrHard)
constexpr uint32_t kMaxLrHard = 10;
// 1024 elements (32 KiB) per workgroup. Round 5: 512-element tiles (twice the workgroups, 22
// KiB of LDS each, so that more tiles are resident and their load / store phases stagger)
// measured slower: dft + idft 2^20 0.291 -> 0.323 ms, 2^23 1.99 -> 2.18 ms, 2^20 proofs -1.5 %
// (profiles/r05_ntt_tile512_ab.jsonl)
constexpr uint32_t kMaxLe = 10;

__device__ __forceinline__ Fr ld_fr(const Fr* p) {
  const uint4* q = reinterpret_cast<const uint4*>(p);
  uint4 a = q[0], b = q[1];
  Fr r;
  r.v[0] = a.x; r.v[1] = a.y; r.v[2] = a.z; r.v[3] = a.w;
  r.v[4] = b.x; r.v[5] = b.y; r.v[6] = b.z; r.v[7] = b.w;
  return r;
}

__device__ __forceinline__ void st_fr(Fr* p, const Fr& v) {
  uint4* q = reinterpret_cast<uint4*>(p);
  q[0] = make_uint4(v.v[0], v.v[1], v.v[2], v.v[3]);
  q[1] = make_uint4(v.v[4], v.v[5], v.v[6], v.v[7]);
}

__device__ __forceinline__ uint32_t bitrev(uint32_t x, uint32_t bits) {
  return bits ? (__builtin_bitreverse32(x) >> (32 - bits)) : 0u;
}

// LDS holds the R-point columns as limb planes of the redundant Fr form (ffr.hpp):
// plane l of element idx at base[l * stride + idx], so each limb access is one
// conflict-free ds_read_b32 / ds_write_b32 across the wave.
using RFr = Rx<FrCfg>;
constexpr int kL = RxShape<FrCfg>::L;

// The data planes use a compile-time stride DS >= E: each limb access is then one
// ds_read/ds_write with an immediate offset from a single address, instead of a v_add per
// plane for a run-time stride. Two strides: the largest E, and kDSSmall for passes of
// E <= 256 (transforms up to 2^16), whose workgroups then hold 15 KiB of LDS instead of 38
// (several proofs in flight share the CUs' LDS with the MSM's tree kernels).
constexpr uint32_t kDS = 1u << kMaxLe;
constexpr uint32_t kDSSmall = 256;

// Measured and removed in round 5 (git history): the first radix-4 step on the
// loaded registers (round 2, within noise, 131 VGPRs), the first radix-4 step of even-radix
// passes in the input loop (round 3, slower), the persistent software-pipelined pass with
// register prefetch (round 3, slower at 2 and 3 waves per SIMD), the last two steps' quad
// exchange through LDS (round 4, between the barrier form and the DPP form kept below), the
// radix-4 products one by one (round 4, slower than the pairs kept below), the
// constant-twiddle Shoup product (round 4, slower) and (round 5, commit 3b467e3) a persistent
// pass for lone transforms whose next tile arrives by LDS-DMA into a staging buffer while the
// current one computes (static LDS arrays so that only the staging reads wait for the DMA, raw
// barriers): 75 KiB LDS and 240 VGPRs, 2 workgroups per CU against 4 — dft + idft 2^20 0.309-
// 0.312 against 0.297 ms, 2^23 2.33-2.36 against 2.07 ms (profiles/r05_ntt_pipe_ab.jsonl).
// k_ntt_pass minimum waves per SIMD (-DPLK_NTT_MINW=4 caps it at 128 VGPRs)
#ifndef PLK_NTT_MINW
#define PLK_NTT_MINW 1
#endif

// Element idx of a data plane sits at word idx ^ ((idx / 32) * 9 mod 32): ds_read_b32 /
// ds_write_b32 bank by word mod 32 per 32-lane half, and the unswizzled columns put the
// bit-reversed output reads on one bank (32-way at the first pass of 2^20 / 2^23: ~15 us of a
// 2^20 transform) and some radix-4 rows on 2 - 4. With the swizzle every 2^20 pass is
// conflict-free and 2^23 keeps 64 extra cycles per workgroup in ~3 000 (bank model over the
// kernel's index patterns, sizes 2^12 .. 2^23). A permutation of the low 5 bits: stays in [0, E).
__device__ __forceinline__ uint32_t swz(uint32_t idx) { return idx ^ (((idx >> 5) * 9u) & 31u); }

template <uint32_t DS>
__device__ __forceinline__ RFr lds_ldd(const uint32_t* base, uint32_t idx) {
  RFr r;
  idx = swz(idx);
#pragma unroll
  for (int l = 0; l < kL; ++l) r.v[l] = base[l * DS + idx];
  return r;
}

template <uint32_t DS>
__device__ __forceinline__ void lds_std(uint32_t* base, uint32_t idx, const RFr& v) {
  idx = swz(idx);
#pragma unroll
  for (int l = 0; l < kL; ++l) base[l * DS + idx] = v.v[l];
}

__device__ __forceinline__ RFr lds_ld(const uint32_t* base, uint32_t stride, uint32_t idx) {
  RFr r;
#pragma unroll
  for (int l = 0; l < kL; ++l) r.v[l] = base[l * stride + idx];
  return r;
}

__device__ __forceinline__ void lds_st(uint32_t* base, uint32_t stride, uint32_t idx, const RFr& v) {
#pragma unroll
  for (int l = 0; l < kL; ++l) base[l * stride + idx] = v.v[l];
}

__device__ __forceinline__ RFr ld_rfr(const Fr* p) { return rx_unpack(ld_fr(p)); }

// a - b + 3r limb by limb, no carries (9 instructions against 27 for rx_sub_lazy; a, b
// normalised below 2r): limbs below 2^29 + 2^30, value in (r, 5r). Only as a multiplicand
// of a normalised twiddle: columns 9 * 2^60 + 9 * 2^58 < 2^64, product 10r^2 / R' + r < 2r
// (ffr.hpp rx_sub_u, R' / r > 70).
__device__ __forceinline__ RFr sub_u(const RFr& a, const RFr& b) { return rx_sub_u<FrCfg, 3>(a, b); }

// ---- lazy butterfly arithmetic --------------------------------------------------------
// Between the radix-2 stages (LDS and registers) values keep normalised limbs and a value
// below 5r instead of [0, 2r): a sum that only feeds the next stage is 9 limb adds, and a
// normalisation is ONE carry pass that also subtracts q r with q = top limb >> 23 (q r
// <= value), against the ~70 instructions of a reduced rx_add. R' / r > 70, so every
// multiplicand below (for canonical twiddles, < r) stays a valid rx_mul operand.
constexpr uint32_t kB = RxShape<FrCfg>::B;
constexpr uint32_t kQMax = 32;  // q of a value < 2^260

struct FrLimbTab {
  uint32_t v[kQMax * kL];
};
// row q: the normalised limbs of 2^261 - q r (the top limb's 2^29 is taken off after the add)
constexpr FrLimbTab make_ztab() {
  FrLimbTab t{};
  for (uint32_t q = 0; q < kQMax; ++q) {
    const RxMultiple<FrCfg> m = rx_multiple<FrCfg>(q, false);  // q r, normalised
    int64_t br = 0;
    for (int i = 0; i < kL; ++i) {  // (2^261 - q r) limb by limb
      const int64_t top = (i == kL - 1) ? (int64_t)1 << kB : 0;
      int64_t d = top - (int64_t)m.v[i] + br;
      br = 0;
      if (i < kL - 1 && d < 0) {
        d += (int64_t)1 << kB;
        br = -1;
      }
      t.v[q * kL + i] = (uint32_t)d;
    }
  }
  return t;
}
__constant__ FrLimbTab kZTab = make_ztab();

// a + c r - b limb by limb, b's limbs below 2^30 - 1 (an unnormalised sum of two normalised
// values): c r with every limb below the top raised by 2^30 (borrowed from the limb above).
// Limbs below 2^31.6: rx_mul's columns stay under 2^64 (9 * 2^60.6 + 9 * 2^58).
template <uint32_t CP>
struct FrRaised2 {
  static constexpr RxMultiple<FrCfg> make() {
    RxMultiple<FrCfg> m = rx_multiple<FrCfg>(CP, false);
    m.v[0] += 2u << kB;
    for (int i = 1; i < kL - 1; ++i) m.v[i] += (2u << kB) - 2u;
    m.v[kL - 1] -= 2u;
    return m;
  }
  static constexpr RxMultiple<FrCfg> k = make();
};
template <uint32_t CP>
__device__ __forceinline__ RFr sub_u2(const RFr& a, const RFr& b) {
  constexpr RxMultiple<FrCfg> Q = FrRaised2<CP>::k;
  RFr r;
#pragma unroll
  for (int i = 0; i < kL; ++i) r.v[i] = a.v[i] + Q.v[i] - b.v[i];
  return r;
}

__device__ __forceinline__ RFr add_u(const RFr& a, const RFr& b) {
  RFr r;
#pragma unroll
  for (int i = 0; i < kL; ++i) r.v[i] = a.v[i] + b.v[i];
  return r;
}

// a (limbs below 2^31, value below 2^260 and >= q r) -> a - q r normalised, q from the
// unnormalised top limb (low by at most 1): value < (q + 2) 2^255 - q r <= 4r for a < 20r,
// < 1.6r for a normalised a < 5r (q exact)
__device__ __forceinline__ RFr reduce_q(const RFr& a, const uint32_t* ztab) {
  constexpr uint32_t MASK = (1u << kB) - 1;
  const uint32_t* z = ztab + (a.v[kL - 1] >> (255 - kB * (kL - 1))) * kL;
  RFr r;
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < kL - 1; ++i) {
    const uint32_t t = a.v[i] + z[i] + c;
    r.v[i] = t & MASK;
    c = t >> kB;
  }
  r.v[kL - 1] = a.v[kL - 1] + z[kL - 1] + c - (1u << kB);
  return r;
}

// Products by the inner (stage) twiddles staged in LDS: Montgomery by w R' (rx_mul, < 2r);
// two at once as interleaved chains (ffr.hpp rx_prod_group, round 4: loop VALU cycles
// 4 137 -> 3 865, dft + idft per step 2^20 0.299-0.301 -> 0.291-0.299 ms, 2^23 2.04 -> 1.99 ms,
// profiles/r04_ntt_grouped_ab.jsonl).
__device__ __forceinline__ RFr twmul(const RFr& a, const uint32_t* twl, uint32_t TS, uint32_t idx) {
  return rx_mul(a, lds_ld(twl, TS, idx));
}
// Round 6: each column of the pair as one asm statement (ffr.hpp RxAsmText): 1 359 -> 1 294
// instructions and 68 -> 1 s_nop in the main pass's loop block (123 -> 1 in the coset pass);
// dft + idft 2^20 0.2844 -> 0.2812 ms, 2^23 1.972 -> 1.946 ms, proofs within noise (three
// interleaved runs, profiles/r06_ntt_asm_pairs_ab.jsonl).
__device__ __forceinline__ void twmul2(const RFr& a0, uint32_t i0, const RFr& a1, uint32_t i1,
                                       const uint32_t* twl, uint32_t TS, RFr& o0, RFr& o1) {
  rx_mul2<FrCfg, true>(a0, lds_ld(twl, TS, i0), a1, lds_ld(twl, TS, i1), o0, o1);
}

// Two radix-2 DIF stages (halves 2h and h) on rows x0..x3 = j, j+h, j+2h, j+3h of one
// column (r = j mod h); outputs o0..o3 belong at rows j, j+h, j+2h, j+3h. Inputs normalised,
// < 5r; outputs normalised, < 4r.
// H1: h == 1, as a template parameter: with a run-time `h == 1` branch assigning the outputs
// on both paths the compiler merged them through an 80-byte scratch object (76 B per lane in
// every k_ntt_pass instantiation: 18 stores and 18 loads per step), so the callers branch
// once per step loop instead.
template <bool H1>
__device__ __forceinline__ void r4_math(const uint32_t* twl, uint32_t TS, const uint32_t* ztab,
                                        uint32_t r, uint32_t h, uint32_t sh1, uint32_t sh2,
                                        const RFr& x0, const RFr& x1, const RFr& x2,
                                        const RFr& x3, RFr& o0, RFr& o1, RFr& o2, RFr& o3) {
  // inputs: normalised, < 5r. Stage of half 2h: twiddle w^(r s1) for x0/x2 (identity
  // when r = 0), w^((r+h) s1) for x1/x3; sums y0, y1 unnormalised (limbs < 2^30, < 10r)
  const RFr y0 = add_u(x0, x2), y1 = add_u(x1, x3);
  if constexpr (H1) {  // r = 0 in every group: no twiddle on x0 / x2 nor in the second stage
    const RFr y2 = reduce_q(rx_sub_u<FrCfg, 6>(x0, x2), ztab);  // < 4r
    const RFr y3 = twmul(rx_sub_u<FrCfg, 6>(x1, x3), twl, TS, 1u << sh1);  // < 3r
    o0 = reduce_q(add_u(y0, y1), ztab);             // < 20r -> < 4r
    o2 = reduce_q(add_u(y2, y3), ztab);             // < 7r -> < 4r
    o1 = reduce_q(sub_u2<11>(y0, y1), ztab);        // < 21r -> < 4r
    o3 = reduce_q(rx_sub_u<FrCfg, 5>(y2, y3), ztab);
  } else {
    // r = 0 groups multiply by w^0 = 1 (twl[0]) under the same bounds as r != 0: the
    // lanes of a wave mix both (columns T < 64), so a branch ran both paths, and
    // straight-line code leaves three independent products (y2, y3, output 1) to
    // interleave. Stage of half h: twiddle w^(r s2) for both pairs; outputs normalised.
    // The step's products go as interleaved pairs (twmul2: ffr.hpp rx_prod_group, no 64-bit
    // merge add per column). Products < 2r.
    RFr y2, y3;
    twmul2(rx_sub_u<FrCfg, 6>(x0, x2), r << sh1, rx_sub_u<FrCfg, 6>(x1, x3), (r + h) << sh1, twl, TS,
           y2, y3);
    // (y0 - y1 + 11r) w and (y2 - y3 + 5r) w
    twmul2(sub_u2<11>(y0, y1), r << sh2, rx_sub_u<FrCfg, 5>(y2, y3), r << sh2, twl, TS, o1, o3);
    o0 = reduce_q(add_u(y0, y1), ztab);  // < 20r -> < 4r
    o2 = reduce_q(add_u(y2, y3), ztab);  // < 6r -> < 4r
  }
}

// r4_math, outputs stored back to LDS at i0..i3
template <uint32_t DS, bool H1>
__device__ __forceinline__ void r4_step(uint32_t* data, const uint32_t* twl, uint32_t TS,
                                        const uint32_t* ztab, uint32_t r, uint32_t h,
                                        uint32_t sh1, uint32_t sh2, uint32_t i0, uint32_t i1,
                                        uint32_t i2, uint32_t i3, const RFr& x0, const RFr& x1,
                                        const RFr& x2, const RFr& x3) {
  RFr o0, o1, o2, o3;
  r4_math<H1>(twl, TS, ztab, r, h, sh1, sh2, x0, x1, x2, x3, o0, o1, o2, o3);
  lds_std<DS>(data, i0, o0);
  lds_std<DS>(data, i2, o2);
  lds_std<DS>(data, i1, o1);
  lds_std<DS>(data, i3, o3);
}

// 4 x 4 transpose of (a0..a3) over the lanes of a quad: lane q ends with element q of lanes
// 0..3 (DPP quad_perm xor 1, then xor 2; lane-dependent selects around each move)
__device__ __forceinline__ void quad_transpose(RFr& a0, RFr& a1, RFr& a2, RFr& a3) {
  const uint32_t lane = __lane_id();
  const bool b0 = lane & 1u, b1 = lane & 2u;
#pragma unroll
  for (int l = 0; l < kL; ++l) {
    const uint32_t s01 = b0 ? a0.v[l] : a1.v[l], s23 = b0 ? a2.v[l] : a3.v[l];
    const uint32_t r01 = (uint32_t)__builtin_amdgcn_mov_dpp((int)s01, 0xB1, 0xF, 0xF, false);
    const uint32_t r23 = (uint32_t)__builtin_amdgcn_mov_dpp((int)s23, 0xB1, 0xF, 0xF, false);
    if (b0) { a0.v[l] = r01; a2.v[l] = r23; } else { a1.v[l] = r01; a3.v[l] = r23; }
    const uint32_t s02 = b1 ? a0.v[l] : a2.v[l], s13 = b1 ? a1.v[l] : a3.v[l];
    const uint32_t r02 = (uint32_t)__builtin_amdgcn_mov_dpp((int)s02, 0x4E, 0xF, 0xF, false);
    const uint32_t r13 = (uint32_t)__builtin_amdgcn_mov_dpp((int)s13, 0x4E, 0xF, 0xF, false);
    if (b1) { a0.v[l] = r02; a1.v[l] = r13; } else { a2.v[l] = r02; a3.v[l] = r13; }
  }
}

// One Stockham pass. PRE: 0 none, 1 multiply input e by pre[e] (coset g^e).
// POST: 0 none, 1 multiply by post_scalar, 2 multiply output e by post[e].
// Data buffers are R-domain (canonical in and out); tw / pre / post / post_scalar are
// R'-domain (ffr.hpp), so every product data x table stays in the R domain.
//
// PRUNE (first pass of a multi-pass plan, input nonzero only in rows j <= R/8 of the pass):
// the first three DIF stages of a zero-padded column have the closed form
//   y[t R/8 + j] = w_R^(j b) (x_j + x_(j+R/8) w_8^b),  b = bitrev3(t),
// with x_(j+R/8) = 0 except for j = 0 — the 8n coset transforms of the prover's
// (n + small)-coefficient polynomials. They are computed directly from the loaded rows
// (7 multiplies per row instead of three stages of butterflies over 8x the rows).
template <int PRE, int POST, int PRUNE, uint32_t DS>
__global__ void __launch_bounds__(256, PLK_NTT_MINW) k_ntt_pass(const Fr* __restrict__ in, Fr* __restrict__ out,
                                                  const Fr* __restrict__ tw,
                                                  const Fr* __restrict__ ptw,
                                                  const Fr* __restrict__ pre,
                                                  const Fr* __restrict__ post, Fr post_scalar,
                                                  uint32_t log_n, uint32_t lp, uint32_t lr,
                                                  uint32_t lt, uint64_t len_in, NttStrides str) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem32[];
  const uint32_t R = 1u << lr, T = 1u << lt, p = 1u << lp;
  const uint32_t E = R << lt, H = R >> 1;
  // kL planes of the TS inner twiddles w_R^x (x < R/2; x < R when pruning)
  const uint32_t TS = PRUNE ? R : H;
  uint32_t* data = smem32;          // kL planes of E (stride DS >= E)
  uint32_t* twl = smem32 + kL * DS;
  uint32_t* ztab = twl + kL * TS;  // kZTab (reduce_q)

  // vector blockIdx.y of a batch: its input, output and scale-table rows (NttBatch::group)
  {
    const uint32_t y = blockIdx.y;
    const uint32_t yi = str.group_in ? y % str.group_in : y, gi = str.group_in ? y / str.group_in : 0;
    in += (size_t)yi * str.in + (size_t)gi * str.in_group;
    out += (size_t)y * str.out;
    if (PRE == 1) pre += (size_t)yi * str.pre;
    if (POST == 2) post += (size_t)(str.group_post ? y % str.group_post : y) * str.post;
  }

  const uint32_t tid = threadIdx.x, bd = blockDim.x;
  const uint32_t nr_log = log_n - lr;  // log2(N/R)

  for (uint32_t x = tid; x < TS; x += bd) lds_st(twl, TS, x, ld_rfr(&tw[(size_t)x << nr_log]));
  for (uint32_t x = tid; x < kQMax * kL; x += bd) ztab[x] = kZTab.v[x];

  // every load of the thread's (at most kLoadIt, E / bd <= 4) elements is issued before the
  // first multiply: one HBM latency per pass instead of one per element
  // The loads are unconditional (clamped indices; the host passes a valid `in` even for
  // len_in = 0) and zero-padding is a select afterwards: a conditional load would merge
  // with its alternative at a join and wait there.
  constexpr uint32_t kLoadIt = 4;
  const uint32_t nit = (E + bd - 1) / bd;  // uniform, <= kLoadIt
  Fr raw[kLoadIt], aux[kLoadIt];           // input; coset factor (PRE) or inter-pass twiddle
  auto issue = [&](uint32_t i0) {          // the loads of the tile of columns i0 .. i0 + T - 1
#pragma unroll
    for (uint32_t c = 0; c < kLoadIt; ++c) {  // all kLoadIt (duplicates past E / bd)
      const uint32_t e = min(tid + c * bd, E - 1);
      const size_t g = (size_t)(i0 + (e & (T - 1))) + ((size_t)(e >> lt) << nr_log);
      const size_t gc = g < len_in ? g : 0;
      raw[c] = ld_fr(&in[gc]);
      if (PRE == 1) aux[c] = ld_fr(&pre[gc]);
    }
    // inter-pass twiddle w_{Rp}^{jk} from the pass table laid out [j][k] (coalesced in k);
    // every (j, k) is in the table and every entry is multiplied below (see there)
    if (PRE != 1 && lp != 0) {
#pragma unroll
      for (uint32_t c = 0; c < kLoadIt; ++c) {
        const uint32_t e = min(tid + c * bd, E - 1);
        aux[c] = ld_fr(&ptw[((size_t)(e >> lt) << lp) + ((i0 + (e & (T - 1))) & (p - 1))]);
      }
    }
  };
  const uint32_t i0 = blockIdx.x << lt;

  // radix-2 stages left: the first radix-4 step's half is 2^(lh-1) (three stages done in
  // closed form when pruning)
  int lh = (int)lr - 1 - (PRUNE ? 3 : 0);
  // odd radix: the first radix-2 stage (half R/2) runs on the loaded registers — a thread's
  // elements c and c + nit/2 are rows j and j + R/2 of one column when E >= 2 bd — and the
  // remaining even count of stages ends in the twiddle-free radix-4 step of halves (2, 1),
  // instead of a last stage of half 1 in its own LDS round trip (one round trip and barrier
  // fewer, R/4 fewer products per column)
  const bool r2first = !PRUNE && (lr & 1) && lr >= 3 && E >= 2 * bd;
  if (PRUNE) {
    __syncthreads();
    // item = (row j < R/8, column t, half hs): blocks 4 hs .. 4 hs + 3 of (j, t)
    const uint32_t R8 = R >> 3;
    for (uint32_t it = tid; it < (E >> 2); it += bd) {
      const uint32_t hs = it & 1, t = (it >> 1) & (T - 1), j = it >> (lt + 1);
      const uint32_t i = i0 + t;
      const size_t g = (size_t)i + ((size_t)j << nr_log);
      RFr x = rx_zero<FrCfg>(), x8 = rx_zero<FrCfg>();
      if (g < len_in) {
        x = ld_rfr(&in[g]);
        if (PRE == 1) x = rx_mul(x, ld_rfr(&pre[g]));
      }
      const size_t g8 = (size_t)i + ((size_t)R8 << nr_log);
      const bool has8 = j == 0 && g8 < len_in;
      if (has8) {
        x8 = ld_rfr(&in[g8]);
        if (PRE == 1) x8 = rx_mul(x8, ld_rfr(&pre[g8]));
      }
#pragma unroll
      for (uint32_t q = 0; q < 4; ++q) {
        const uint32_t blk = 4 * hs + q, b = bitrev(blk, 3);
        RFr v = (j == 0 || b == 0) ? x : rx_mul(x, lds_ld(twl, TS, j * b));
        if (has8) v = rx_add(v, b == 0 ? x8 : rx_mul(x8, lds_ld(twl, TS, R8 * b)));
        lds_std<DS>(data, ((blk * R8 + j) << lt) + t, v);
      }
    }
  }
  if (!PRUNE) {
    issue(i0);
    auto input = [&](uint32_t c) -> RFr {  // element tid + c bd, pre-scaled / twiddled
      const uint32_t e = tid + c * bd;
      const uint32_t t = e & (T - 1), j = e >> lt;
      const uint32_t i = i0 + t;
      const size_t g = (size_t)i + ((size_t)j << nr_log);
      RFr v = rx_zero<FrCfg>();
      if (g < len_in) {
        v = rx_unpack(raw[c]);
        if (PRE == 1) v = rx_mul(v, rx_unpack(aux[c]));
      }
      // inter-pass twiddle: the multiply MUST stay unconditional. A plain idft's last pass
      // reads pass_tw_inv_last, whose entries carry n^-1 (round 5: the idft scaling rides on
      // this table), so its j = 0 / k = 0 entries are n^-1, not one; skipping the "identity"
      // entries would drop the scaling on those rows (test_idft_multipass_identity_rows)
      if (PRE != 1 && lp != 0) v = rx_mul(v, rx_unpack(aux[c]));
      return v;
    };
    {
      // element e = tid + c bd sits at LDS index e = (row << lt) + column. With r2first the
      // upper half's elements (c >= nit / 2: rows j + R/2) meet their partner, which this
      // thread stored at e - E/2 one iteration earlier (read back without a barrier), and the
      // pair's butterfly is stored in place. One loop for both forms: as two code paths the
      // compiler hoisted all four inputs above the branch (137 VGPRs instead of 115)
      if (r2first) __syncthreads();  // twl / ztab staged
#pragma unroll
      for (uint32_t c = 0; c < kLoadIt; ++c) {
        if (c >= nit) break;
        const uint32_t e = tid + c * bd;
        const RFr v = input(c);  // < 2r, normalised
        if (r2first && 2 * c >= nit) {
          const uint32_t el = e - (E >> 1);
          const RFr a = lds_ldd<DS>(data, el);
          lds_std<DS>(data, el, reduce_q(add_u(a, v), ztab));                        // < 1.6r
          lds_std<DS>(data, e, twmul(sub_u(a, v), twl, TS, el >> lt));  // < 2r
        } else if (e < E) {
          lds_std<DS>(data, e, v);
        }
      }
      if (r2first) lh -= 1;
    }
  }
  __syncthreads();

  // R-point DIF (natural in, bit-reversed out) on each of the T columns, two radix-2 stages
  // per LDS round trip: a thread loads x0..x3 = rows j, j+h, j+2h, j+3h, applies the stage
  // of half 2h (pairs x0/x2, x1/x3) and the stage of half h (pairs y0/y1, y2/y3) in
  // registers, and stores once. Same butterflies and twiddles as stage-by-stage radix 2.
  for (; lh >= 1; lh -= 2) {
    const uint32_t h = 1u << (lh - 1);
    const uint32_t sh1 = lr - 1 - lh, sh2 = lr - lh;  // twiddle index shifts of both stages
    // the last two radix-4 steps (halves 8, 4 then 2, 1) exchange data only inside 16-row
    // blocks of one column, between the 4 groups (t, 16B + r), r < 4: with those groups on the
    // 4 lanes of a quad (r lowest) the exchange is a DPP quad transpose in registers, with no
    // LDS round trip and no barrier (round 4: dft + idft 2^20 0.308 -> 0.298-0.306 ms, 2^23
    // 2.10 -> 2.05 ms, profiles/r04_ntt_quadx_ab.jsonl)
    const bool quad = lh == 3 && lr >= 5 && (E >> 2) % bd == 0;
    if (quad) {
      // halves 8 and 4, quad transpose in registers, halves 2 and 1: one LDS round trip
      for (uint32_t g = tid; g < (E >> 2); g += bd) {
        const uint32_t r = g & 3u, t = (g >> 2) & (T - 1), B = g >> (2 + lt);
        const uint32_t j = (B << 4) + r;  // rows j + 4m of the 16-row block B
        RFr x0 = lds_ldd<DS>(data, (j << lt) + t), x1 = lds_ldd<DS>(data, ((j + 4) << lt) + t);
        RFr x2 = lds_ldd<DS>(data, ((j + 8) << lt) + t), x3 = lds_ldd<DS>(data, ((j + 12) << lt) + t);
        RFr o0, o1, o2, o3;
        r4_math<false>(twl, TS, ztab, r, 4, lr - 4, lr - 3, x0, x1, x2, x3, o0, o1, o2, o3);
        quad_transpose(o0, o1, o2, o3);  // lane r now holds rows 16B + 4r + (0, 1, 2, 3)
        const uint32_t jq = (B << 4) + (r << 2);
        r4_step<DS, true>(data, twl, TS, ztab, 0, 1, lr - 2, lr - 1, (jq << lt) + t,
                    ((jq + 1) << lt) + t, ((jq + 2) << lt) + t, ((jq + 3) << lt) + t, o0, o1, o2,
                    o3);
      }
      lh -= 2;  // both steps done
      __syncthreads();
      continue;
    }
    auto steps = [&](auto h1) {
      for (uint32_t g = tid; g < (E >> 2); g += bd) {
        const uint32_t t = g & (T - 1), jg = g >> lt;
        const uint32_t r = jg & (h - 1);
        const uint32_t j = ((jg >> (lh - 1)) << (lh + 1)) + r;
        const uint32_t i0 = (j << lt) + t, i1 = ((j + h) << lt) + t;
        const uint32_t i2 = ((j + 2 * h) << lt) + t, i3 = ((j + 3 * h) << lt) + t;
        const RFr x0 = lds_ldd<DS>(data, i0), x1 = lds_ldd<DS>(data, i1);
        const RFr x2 = lds_ldd<DS>(data, i2), x3 = lds_ldd<DS>(data, i3);
        r4_step<DS, decltype(h1)::value>(data, twl, TS, ztab, r, h, sh1, sh2, i0, i1, i2, i3, x0, x1, x2, x3);
      }
    };
    if (h == 1) steps(std::true_type{});
    else steps(std::false_type{});
    __syncthreads();
  }
  if (lh == 0) {  // odd radix: last stage of half 1 (twiddle-free)
    for (uint32_t b = tid; b < (E >> 1); b += bd) {
      const uint32_t t = b & (T - 1), jb = b >> lt;
      const uint32_t j1 = jb << 1;
      const RFr a = lds_ldd<DS>(data, (j1 << lt) + t);
      const RFr c = lds_ldd<DS>(data, ((j1 + 1) << lt) + t);
      lds_std<DS>(data, (j1 << lt) + t, reduce_q(add_u(a, c), ztab));
      lds_std<DS>(data, ((j1 + 1) << lt) + t, reduce_q(rx_sub_u<FrCfg, 6>(a, c), ztab));
    }
    __syncthreads();
  }

  for (uint32_t o = tid; o < E; o += bd) {
    uint32_t t, m;
    if (p >= T) {
      t = o & (T - 1);
      m = o >> lt;
    } else {  // o = u*pR + m*p + s, t = u*p + s: contiguous output run per workgroup
      const uint32_t s = o & (p - 1);
      m = (o >> lp) & (R - 1);
      t = ((o >> (lp + lr)) << lp) + s;
    }
    const uint32_t i = i0 + t;
    const uint32_t k = i & (p - 1);
    const size_t pos = ((size_t)(i - k) << lr) + k + ((size_t)m << lp);
    RFr v = lds_ldd<DS>(data, (bitrev(m, lr) << lt) + t);  // < 5r
    if (POST == 1) v = rx_mul(v, rx_unpack(post_scalar));
    else if (POST == 2) v = rx_mul(v, ld_rfr(&post[pos]));
    else v = reduce_q(v, ztab);  // < 1.6r
    st_fr(&out[pos], rx_pack_canonical(v));
  }
}

// pass twiddles: out[(j << lp) + k] = w_N^{(j k) << shift} for j < R, k < p (R' domain;
// tw is the R'-domain power table of the same direction)
__global__ void k_pass_twiddles(const Fr* __restrict__ tw, Fr* __restrict__ out, uint32_t lp,
                                uint32_t lr, uint32_t shift) {
  const uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (1ull << (lp + lr))) return;
  const uint64_t j = e >> lp, k = e & ((1ull << lp) - 1);
  st_fr(&out[e], ld_fr(&tw[(j * k) << shift]));
}

// out[e] = in[e] * s (Montgomery product: an R'-domain table times an R-domain scalar stays
// in the R' domain)
__global__ void k_scale_table(const Fr* __restrict__ in, Fr* __restrict__ out, Fr s, uint64_t n) {
  const uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  st_fr(&out[e], fe_mul(ld_fr(&in[e]), s));
}

// in-place R -> R' domain conversion of a table (ffr.hpp)
__global__ void k_table_to_rx(const Fr* in, Fr* out, uint64_t n) {
  const uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  st_fr(&out[e], fe_to_rx_domain(ld_fr(&in[e])));
}

// table[e] = base^e * scale for e < n (exact powers; one pow per element)
__global__ void k_power_table(Fr* __restrict__ out, Fr base, Fr scale, uint64_t n) {
  const uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  st_fr(&out[e], fe_mul(fe_pow_u64(base, e), scale));
}

__global__ void k_copy_pad(const Fr* __restrict__ in, Fr* __restrict__ out, uint64_t len_in,
                           uint64_t n) {
  const uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  st_fr(&out[e], e < len_in ? ld_fr(&in[e]) : fe_zero<FrCfg>());
}

// v_h[i] = (g w^i)^deg - 1 = g^deg * (w^deg)^i - 1
__global__ void k_vanishing(Fr* __restrict__ out, Fr gdeg, Fr wdeg, uint64_t n) {
  const uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  st_fr(&out[e], fe_sub(fe_mul(gdeg, fe_pow_u64(wdeg, e)), fe_one<FrCfg>()));
}

}  // namespace

// ROOT_OF_UNITY = 7^((r-1)/2^32) (Montgomery form), squared down to order 2^log_n
void fr_root_of_unity(uint32_t log_n, Fr& omega) {
  // canonical 0x16a2a19edfe81f20d09b681922c813b4b63683508c2280b93829971f439f0d2b
  static const uint32_t root[8] = {0x439f0d2bu, 0x3829971fu, 0x8c2280b9u, 0xb6368350u,
                                   0x22c813b4u, 0xd09b6819u, 0xdfe81f20u, 0x16a2a19eu};
  Fr w;
  for (int i = 0; i < 8; ++i) w.v[i] = root[i];
  w = fe_to_mont(w);
  for (uint32_t s = log_n; s < 32; ++s) w = fe_sqr(w);
  omega = w;
}

static void plan_domain(plk_domain* d) {
  const uint32_t L = d->log_n;
  d->plan.clear();
  if (L == 0) return;
  // elements per workgroup: keep >= ~256 workgroups when the transform allows it, and at
  // least 2^10 (round 3; PLK_NTT_LE_MIN overrides for experiments). Small transforms (the
  // 2^12..2^16 proofs' 2^12..2^17 ones) then take 1 024-element tiles of >= 4 columns
  // (128-byte runs) instead of 64..256-element tiles of 1..2 columns: fewer, fuller
  // workgroups and no 32-byte strided reads; 2^12 proofs 5.7 -> 6.3 M constraints/s, 2^16
  // 23.4 -> 24.1 M (round 3 sweep, tools/gpu_r03_i.sh; 2^6 / 2^8 / 2^9 / 2^10 tried)
  static const uint32_t le_min = [] {
    const char* e = getenv("PLK_NTT_LE_MIN");
    const int v = e ? atoi(e) : 10;
    return (uint32_t)(v >= 1 && v <= (int)kMaxLe ? v : 10);
  }();
  uint32_t le = L > 8 ? L - 8 : 1;
  if (le < le_min) le = L < le_min ? L : le_min;
  if (le > kMaxLe) le = kMaxLe;
  // radix cap 2^9: 2^17 and 2^18 run in two passes of 2-column tiles (512 rows) instead of
  // three; 2^19 and up keep three passes of >= 4 columns. Round 3 (tools/gpu_r03_lr.sh): cap
  // 2^8 / 2^9 / 2^10 — 2^17 0.110 / 0.095 / 0.095 ms per dft + idft, 2^18 0.122 / 0.113 /
  // 0.113, 2^20 0.31 / 0.31 / 0.34 (two passes of 1-column tiles: 32-byte strided reads);
  // the 2^16 proof (its 2^17 coset transforms) 23.4 -> 25.9 M constraints/s.
  // PLK_NTT_MAX_LR overrides it (up to 10).
  static const uint32_t lr_cap = [] {
    const char* e = getenv("PLK_NTT_MAX_LR");
    const int v = e ? atoi(e) : (int)kMaxLr;
    return (uint32_t)(v >= 1 && v <= (int)kMaxLrHard ? v : kMaxLr);
  }();
  const uint32_t max_lr = le < lr_cap ? le : lr_cap;
  const uint32_t P = (L + max_lr - 1) / max_lr;
  uint32_t lp = 0;
  for (uint32_t q = 0; q < P; ++q) {
    const uint32_t rem = L - lp, left = P - q;
    const uint32_t lr = (rem + left - 1) / left;
    uint32_t lt = le - lr;
    if (lt > L - lr) lt = L - lr;
    d->plan.push_back(NttPass{lp, lr, lt});
    lp += lr;
  }
  d->le = le;
}

int ntt_build_domain(plk_domain* d) {
  const uint64_t n = d->n;
  fr_root_of_unity(d->log_n, d->omega);
  d->omega_inv = fe_inv(d->omega);
  Fr nf = fe_zero<FrCfg>();
  nf.v[0] = (uint32_t)n;
  nf.v[1] = (uint32_t)(n >> 32);
  nf = fe_to_mont(nf);
  d->n_inv = fe_inv(nf);
  Fr g = fe_zero<FrCfg>();
  g.v[0] = 7;
  d->g = fe_to_mont(g);
  d->g_inv = fe_inv(d->g);
  plan_domain(d);

  int st;
  if ((st = d->tw_fwd.alloc(n * sizeof(Fr)))) return st;
  if ((st = d->tw_inv.alloc(n * sizeof(Fr)))) return st;
  if ((st = d->coset_pow.alloc(n * sizeof(Fr)))) return st;
  if ((st = d->icoset_scale.alloc(n * sizeof(Fr)))) return st;
  hipStream_t s = d->ctx->stream;
  const uint32_t bs = 256;
  const uint32_t nb = (uint32_t)((n + bs - 1) / bs);
  const Fr one = fe_one<FrCfg>();
  hipLaunchKernelGGL(k_power_table, dim3(nb), dim3(bs), 0, s, d->tw_fwd.as<Fr>(), d->omega, one, n);
  hipLaunchKernelGGL(k_power_table, dim3(nb), dim3(bs), 0, s, d->tw_inv.as<Fr>(), d->omega_inv, one, n);
  hipLaunchKernelGGL(k_power_table, dim3(nb), dim3(bs), 0, s, d->coset_pow.as<Fr>(), d->g, one, n);
  hipLaunchKernelGGL(k_power_table, dim3(nb), dim3(bs), 0, s, d->icoset_scale.as<Fr>(), d->g_inv,
                     d->n_inv, n);
  // the pass kernel multiplies R-domain data by R'-domain tables (ffr.hpp)
  if ((st = d->tw_fwd_rx.alloc(n * sizeof(Fr)))) return st;
  hipLaunchKernelGGL(k_table_to_rx, dim3(nb), dim3(bs), 0, s, d->tw_fwd.as<Fr>(), d->tw_fwd_rx.as<Fr>(), n);
  hipLaunchKernelGGL(k_table_to_rx, dim3(nb), dim3(bs), 0, s, d->tw_inv.as<Fr>(), d->tw_inv.as<Fr>(), n);
  hipLaunchKernelGGL(k_table_to_rx, dim3(nb), dim3(bs), 0, s, d->coset_pow.as<Fr>(), d->coset_pow.as<Fr>(), n);
  hipLaunchKernelGGL(k_table_to_rx, dim3(nb), dim3(bs), 0, s, d->icoset_scale.as<Fr>(),
                     d->icoset_scale.as<Fr>(), n);
  PLK_HIP_TRY(hipGetLastError());
  // per-pass inter-pass twiddle tables (passes after the first), both directions
  d->pass_tw_fwd.clear();
  d->pass_tw_inv.clear();
  d->pass_tw_fwd.resize(d->plan.size());
  d->pass_tw_inv.resize(d->plan.size());
  for (size_t q = 1; q < d->plan.size(); ++q) {
    const NttPass& ps = d->plan[q];
    const uint64_t cnt = 1ull << (ps.lp + ps.lr);
    const uint32_t shift = d->log_n - ps.lr - ps.lp;
    if ((st = d->pass_tw_fwd[q].alloc(cnt * sizeof(Fr)))) return st;
    if ((st = d->pass_tw_inv[q].alloc(cnt * sizeof(Fr)))) return st;
    const uint32_t pb = (uint32_t)((cnt + bs - 1) / bs);
    hipLaunchKernelGGL(k_pass_twiddles, dim3(pb), dim3(bs), 0, s, d->tw_fwd_rx.as<Fr>(),
                       d->pass_tw_fwd[q].as<Fr>(), ps.lp, ps.lr, shift);
    hipLaunchKernelGGL(k_pass_twiddles, dim3(pb), dim3(bs), 0, s, d->tw_inv.as<Fr>(),
                       d->pass_tw_inv[q].as<Fr>(), ps.lp, ps.lr, shift);
    if (q + 1 == d->plan.size()) {  // (R' x R -> R': still an R'-domain table)
      if ((st = d->pass_tw_inv_last.alloc(cnt * sizeof(Fr)))) return st;
      hipLaunchKernelGGL(k_scale_table, dim3(pb), dim3(bs), 0, s, d->pass_tw_inv[q].as<Fr>(),
                         d->pass_tw_inv_last.as<Fr>(), d->n_inv, cnt);
    }
  }
  PLK_HIP_TRY(hipGetLastError());
  PLK_HIP_TRY(stream_wait(s));
  return PLK_OK;
}

int ntt_run(plk_domain* d, const Fr* in, Fr* out, size_t len_in, int dir, int coset, Fr* scratch,
            hipStream_t stream, uint32_t count, const Fr* pre_table) {
  NttBatch b;
  b.in_stride = b.out_stride = d->n;
  b.pre = pre_table;
  return ntt_run_batch(d, in, out, len_in, dir, coset, scratch, stream, count, b);
}

int ntt_run_batch(plk_domain* d, const Fr* in, Fr* out, size_t len_in, int dir, int coset,
                  Fr* scratch, hipStream_t stream, uint32_t count, const NttBatch& bt) {
  const uint64_t n = d->n;
  if (len_in > n || count == 0) return PLK_E_ARG;
  const Fr* pre_table = bt.pre;
  if (n == 1) {  // size-1 transform: x * pre[0] (forward coset) or x * post[0]; else identity
    if (bt.pre || bt.post) return PLK_E_ARG;  // not needed by any caller
    for (uint32_t v = 0; v < count; ++v) {
      Fr* o = out + v * bt.out_stride;
      const Fr* i = in + v * bt.in_stride;
      if (len_in == 0) {
        PLK_HIP_TRY(hipMemsetAsync(o, 0, sizeof(Fr), stream));
      } else if (i != o) {
        PLK_HIP_TRY(hipMemcpyAsync(o, i, sizeof(Fr), hipMemcpyDeviceToDevice, stream));
      }
    }
    return PLK_OK;
  }
  int st;
  const size_t P = d->plan.size();
  // when the output does not overlap the input, it doubles as one of the ping-pong buffers
  // (passes alternate so the last one lands in it): a batch then needs count * n of scratch
  // instead of 2 count n (the prover's batch of the four wires' 12 coset blocks)
  const uint64_t in_ext = bt.group ? (uint64_t)(count / bt.group - 1) * bt.in_group_stride +
                                         (uint64_t)(bt.group - 1) * bt.in_stride + len_in
                                   : (uint64_t)(count - 1) * bt.in_stride + len_in;
  const uint64_t out_ext = (uint64_t)(count - 1) * bt.out_stride + n;
  const bool out_pp = P >= 2 && bt.out_stride >= n && (len_in == 0 || in + in_ext <= out || out + out_ext <= in);
  if (!scratch) {
    if ((st = d->scratch.alloc(2 * n * sizeof(Fr) * (count > 1 ? count : 1)))) return st;
    scratch = d->scratch.as<Fr>();
  }
  Fr* s1 = scratch;
  Fr* s2 = scratch + n * count;
  const Fr* tw = dir > 0 ? d->tw_fwd_rx.as<Fr>() : d->tw_inv.as<Fr>();
  const Fr n_inv_rx = fe_to_rx_domain(d->n_inv);
  // an all-zero input still has its (clamped, discarded) loads: point them at a live table
  const bool no_input = len_in == 0;
  const Fr* src = no_input ? tw : in;
  for (size_t q = 0; q < P; ++q) {
    const NttPass& ps = d->plan[q];
    Fr* dst = (q + 1 == P) ? out : out_pp ? (((P - 1 - q) & 1) ? s1 : out) : ((q & 1) ? s2 : s1);
    const bool first = q == 0, last = q + 1 == P;
    const uint32_t E = 1u << (ps.lr + ps.lt);
    uint32_t bd = E / 4;
    if (bd < 64) bd = 64;
    if (bd > 256) bd = 256;
    const uint32_t blocks = (uint32_t)(n >> (ps.lr + ps.lt));
    const int pre = (first && dir > 0 && coset) ? 1 : 0;
    // a plain idft's n^-1 comes with the last pass' inter-pass twiddles (pass_tw_inv_last) when
    // the plan has more than one pass: one product per element fewer in that pass
    const bool scaled_tw = last && !first && dir < 0 && !coset;
    const int post = (last && dir < 0 && !scaled_tw) ? (coset ? 2 : 1) : 0;
    const uint64_t lin = first ? len_in : n;
    // zero-padded input (rows j <= R/8 of the first pass only): closed-form first stages
    const bool prune = first && !last && ps.lr >= 4 &&
                       len_in <= ((n >> ps.lr) << (ps.lr - 3)) + (n >> ps.lr);
    const bool small = E <= kDSSmall;
    // (round 3: an LDS floor of 54 / 80 KB per workgroup, i.e. 2 - 3 resident workgroups per
    // CU so that a lone transform's tiles run in staggered generations, measured 3 - 7 %
    // slower at 2^20 and 2^23: the lost occupancy costs more than the overlap gains)
    const size_t lds = ((size_t)(small ? kDSSmall : kDS) + ((1u << ps.lr) >> (prune ? 0 : 1)) + kQMax) *
                       kL * sizeof(uint32_t);
    dim3 grid(blocks, count);
    const Fr* ptw = q == 0 ? nullptr
                    : scaled_tw ? d->pass_tw_inv_last.as<Fr>()
                    : (dir > 0 ? d->pass_tw_fwd[q].as<Fr>() : d->pass_tw_inv[q].as<Fr>());
    NttStrides str;
    str.in = first ? (no_input ? 0 : bt.in_stride) : n * 1;
    str.out = last ? bt.out_stride : n * 1;
    str.pre = bt.pre ? bt.pre_stride : 0;
    str.post = bt.post ? bt.post_stride : 0;
    str.in_group = first && !no_input ? bt.in_group_stride : 0;
    str.group_in = first ? bt.group : 0;
    str.group_post = last ? bt.group : 0;
#define PLK_LAUNCH_DS(PRE, POST, PRUNE, DS)                                               \
  do {                                                                                    \
    const void* kp_ = reinterpret_cast<const void*>(&k_ntt_pass<PRE, POST, PRUNE, DS>);   \
    if (lds > 65536)                                                                      \
      PLK_HIP_TRY(hipFuncSetAttribute(kp_, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds)); \
    hipLaunchKernelGGL((k_ntt_pass<PRE, POST, PRUNE, DS>), grid, dim3(bd), lds, stream, src, dst, \
                       tw, ptw, pre_table ? pre_table : d->coset_pow.as<Fr>(),            \
                       bt.post ? bt.post : d->icoset_scale.as<Fr>(), n_inv_rx, d->log_n,  \
                       ps.lp, ps.lr, ps.lt, lin, str);                                     \
  } while (0)
#define PLK_LAUNCH(PRE, POST, PRUNE)                              \
  do {                                                            \
    if (small) PLK_LAUNCH_DS(PRE, POST, PRUNE, kDSSmall);          \
    else PLK_LAUNCH_DS(PRE, POST, PRUNE, kDS);                     \
  } while (0)
    if (prune) {
      if (pre == 1) PLK_LAUNCH(1, 0, 1);
      else PLK_LAUNCH(0, 0, 1);
    } else if (pre == 0 && post == 0) PLK_LAUNCH(0, 0, 0);
    else if (pre == 1 && post == 0) PLK_LAUNCH(1, 0, 0);
    else if (pre == 0 && post == 1) PLK_LAUNCH(0, 1, 0);
    else if (pre == 0 && post == 2) PLK_LAUNCH(0, 2, 0);
    else if (pre == 1 && post == 1) PLK_LAUNCH(1, 1, 0);
    else PLK_LAUNCH(1, 2, 0);
#undef PLK_LAUNCH_DS
#undef PLK_LAUNCH
    PLK_HIP_TRY(hipGetLastError());
    src = dst;
  }
  return PLK_OK;
}

int ntt_power_table(Fr* out, const Fr& base, const Fr& scale, uint64_t n, bool to_rx,
                    hipStream_t s) {
  if (n == 0) return PLK_OK;
  const uint32_t nb = (uint32_t)((n + 255) / 256);
  hipLaunchKernelGGL(k_power_table, dim3(nb), dim3(256), 0, s, out, base, scale, n);
  if (to_rx) hipLaunchKernelGGL(k_table_to_rx, dim3(nb), dim3(256), 0, s, out, out, n);
  PLK_HIP_TRY(hipGetLastError());
  return PLK_OK;
}

int ntt_vanishing(plk_domain* d, uint64_t deg, Fr* d_out, hipStream_t s) {
  const Fr gdeg = fe_pow_u64(d->g, deg);
  const Fr wdeg = fe_pow_u64(d->omega, deg);
  const uint32_t bs = 256;
  const uint32_t nb = (uint32_t)((d->n + bs - 1) / bs);
  hipLaunchKernelGGL(k_vanishing, dim3(nb), dim3(bs), 0, s, d_out, gdeg, wdeg, (uint64_t)d->n);
  PLK_HIP_TRY(hipGetLastError());
  return PLK_OK;
}

}  // namespace plk
