// prover_kernels.hip — device kernels of Prover::create_proof around the NTT/MSM path
// (SURVEY.md §8f rows 1-3 and §8a a9/a12), all HBM- or VALU-bound elementwise work:
//  * wire gather (prover.rs:109-119), blinding b(X)(X^n - 1) (prover.rs:126-129,193)
//  * grand product z (permutation.rs:205-300): per-gate numerator/denominator, then
//    z_i = N_i * S_i / D (exclusive prefix product of numerators, inclusive suffix product
//    of denominators, ONE inversion) instead of the reference's n inversions + serial scan
//  * quotient over the 8n coset (quotient_poly.rs:74-114,122-262): arithmetic + range
//    widgets + PI + permutation identity/copy terms + L1 term, divided by v_h, whose
//    8 distinct values (period 8) are inverted once on the host
//  * batched polynomial evaluation (linearization_poly.rs:52-73,108)
//  * linear combinations (t split / quot assembly prover.rs:252-259,408-418, r(X),
//    aggregate witness numerators) and Ruffini division by (X - z)
#include <hip/hip_runtime.h>

#include "ffr.hpp"
#include "internal.hpp"
#include "prover.hpp"

namespace plk {

namespace {

__device__ __forceinline__ Fr ldf(const Fr* p) {
  const uint4* q = reinterpret_cast<const uint4*>(p);
  uint4 a = q[0], b = q[1];
  Fr r;
  r.v[0] = a.x; r.v[1] = a.y; r.v[2] = a.z; r.v[3] = a.w;
  r.v[4] = b.x; r.v[5] = b.y; r.v[6] = b.z; r.v[7] = b.w;
  return r;
}

__device__ __forceinline__ void stf(Fr* p, const Fr& v) {
  uint4* q = reinterpret_cast<uint4*>(p);
  q[0] = make_uint4(v.v[0], v.v[1], v.v[2], v.v[3]);
  q[1] = make_uint4(v.v[4], v.v[5], v.v[6], v.v[7]);
}

using RFr = Rx<FrCfg>;
__device__ __forceinline__ RFr ldr(const Fr* p) { return rx_unpack(ldf(p)); }

// a + b + c limb by limb, no carries (a, b, c normalised, each below 2r): limbs below
// 3 * 2^29, value below 6r. Only as a multiplicand of a normalised operand below 6r: columns
// 9 * 1.5 * 2^59 + 9 * 2^58 < 2^64, product 36 r^2 / R' + r < 2r (R' / r > 70).
__device__ __forceinline__ RFr add3_u(const RFr& a, const RFr& b, const RFr& c) {
  RFr r;
#pragma unroll
  for (int l = 0; l < RxShape<FrCfg>::L; ++l) r.v[l] = a.v[l] + b.v[l] + c.v[l];
  return r;
}

// carries propagated: normalised limbs, same value
__device__ __forceinline__ RFr rx_norm(const RFr& a) {
  constexpr uint32_t B = RxShape<FrCfg>::B, MASK = (1u << B) - 1;
  RFr r;
  uint32_t c = 0;
#pragma unroll
  for (int l = 0; l < RxShape<FrCfg>::L; ++l) {
    const uint32_t t = a.v[l] + c;
    r.v[l] = l == RxShape<FrCfg>::L - 1 ? t : (t & MASK);
    c = t >> B;
  }
  return r;
}

inline uint32_t blocks_for(uint64_t n, uint32_t bs) { return (uint32_t)((n + bs - 1) / bs); }

// ---------------------------------------------------------------------------- wires
__global__ void k_gather_wires(const Fr* __restrict__ witness, const uint32_t* __restrict__ idx,
                               uint64_t m, uint64_t n, Fr* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t col = blockIdx.y;
  if (i >= n) return;
  stf(&out[col * n + i], i < m ? ldf(&witness[idx[col * n + i]]) : fe_zero<FrCfg>());
}

// poly[i] -= r_i, poly[n + i] = r_i (i < count): p(X) + b(X)(X^n - 1)
__global__ void k_blind(Fr* __restrict__ poly, uint64_t n, BlindArgs b) {
  const uint32_t i = threadIdx.x;
  if (i >= b.count) return;
  stf(&poly[i], fe_sub(ldf(&poly[i]), b.r[i]));
  stf(&poly[n + i], b.r[i]);
}

// PI(X) = n^-1 sum_i v_i w^(-i j) summed over the few nonzero v_i: one product per public
// input and coefficient instead of a transform (c_k = v_k n^-1 in the R domain times the
// R'-domain table entry lands in the R domain)
__global__ void k_pi_coef(PiDirect pd, const Fr* __restrict__ tw_inv, uint64_t n,
                          Fr* __restrict__ out) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  RFr acc = rx_zero<FrCfg>();
  for (uint32_t k = 0; k < pd.count; ++k)
    acc = rx_add(acc, rx_mul(rx_unpack(pd.c[k]), ldr(&tw_inv[(pd.idx[k] * j) & (n - 1)])));
  stf(&out[j], rx_pack_canonical(acc));
}

// thread 4p + i: coefficient i of polynomial p
__global__ void k_blind_batch(BlindBatch bb, uint64_t n) {
  const uint32_t p = threadIdx.x >> 2, i = threadIdx.x & 3;
  if (p >= bb.npoly || i >= bb.b[p].count) return;
  Fr* poly = bb.poly[p];
  stf(&poly[i], fe_sub(ldf(&poly[i]), bb.b[p].r[i]));
  stf(&poly[n + i], bb.b[p].r[i]);
}

__global__ void k_fill(Fr* __restrict__ out, Fr v, uint64_t n) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) stf(&out[i], v);
}

// ------------------------------------------------------------------- grand product
// num_i = prod_c (w_c + beta k_c w^i + gamma), den_i = prod_c (w_c + beta sigma_c + gamma)
// Redundant limbs: beta and k_c arrive in the R' domain, so beta x and k_c beta x are
// R-domain like the wires and gamma; the factors are carry-free sums (add3_u); a product
// of four R-domain factors is R^4 / R'^3 times the value, and `fix` = R'^4 / R^3 mod r
// (a plain integer) brings it back to R.
__global__ void k_perm_numden(const Fr* __restrict__ wires, const Fr* __restrict__ sigmas,
                              const Fr* __restrict__ elements, uint64_t n, Fr beta_rx, Fr gamma,
                              Fr k1_rx, Fr k2_rx, Fr k3_rx, Fr fix, Fr* __restrict__ num,
                              Fr* __restrict__ den) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const RFr be = rx_unpack(beta_rx), g = rx_unpack(gamma);
  const RFr bx = rx_mul(be, ldr(&elements[i]));
  // the four wire factors written out (a loop over an array of the bX K_c values kept the
  // array in scratch memory)
  auto tn = [&](int c, const RFr& bxk) { return add3_u(ldr(&wires[c * n + i]), g, bxk); };
  auto td = [&](int c) { return add3_u(ldr(&wires[c * n + i]), g, rx_mul(be, ldr(&sigmas[c * n + i]))); };
  RFr nu = rx_norm(tn(0, bx)), de = rx_norm(td(0));
  nu = rx_mul(nu, tn(1, rx_mul(rx_unpack(k1_rx), bx)));
  de = rx_mul(de, td(1));
  nu = rx_mul(nu, tn(2, rx_mul(rx_unpack(k2_rx), bx)));
  de = rx_mul(de, td(2));
  nu = rx_mul(nu, tn(3, rx_mul(rx_unpack(k3_rx), bx)));
  de = rx_mul(de, td(3));
  const RFr f = rx_unpack(fix);
  stf(&num[i], rx_pack_canonical(rx_mul(nu, f)));
  stf(&den[i], rx_pack_canonical(rx_mul(de, f)));
}

// z_i = N_i * S_i * dinv
__global__ void k_mul3(const Fr* __restrict__ a, const Fr* __restrict__ b, Fr c,
                       Fr* __restrict__ out, uint64_t n) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) stf(&out[i], fe_mul(fe_mul(ldf(&a[i]), ldf(&b[i])), c));
}

// ----------------------------------------------------------------------- scans
// 3-phase scan over Fr with op = multiply (MUL) or add; SUFFIX scans from the top.
constexpr uint32_t kScanThreads = 256, kScanPer = 8, kScanBlock = kScanThreads * kScanPer;

template <bool MUL>
__device__ __forceinline__ Fr op(const Fr& a, const Fr& b) {
  return MUL ? fe_mul(a, b) : fe_add(a, b);
}
template <bool MUL>
__device__ __forceinline__ Fr ident() {
  return MUL ? fe_one<FrCfg>() : fe_zero<FrCfg>();
}

// logical index j of a scan in direction SUFFIX maps to physical n-1-j
template <bool SUFFIX>
__device__ __forceinline__ uint64_t phys(uint64_t j, uint64_t n) {
  return SUFFIX ? n - 1 - j : j;
}

template <bool MUL, bool SUFFIX>
__global__ void __launch_bounds__(kScanThreads) k_scan_reduce(const Fr* __restrict__ in, uint64_t n,
                                                              Fr* __restrict__ tot) {
  __shared__ Fr sh[kScanThreads];
  const uint64_t base = (uint64_t)blockIdx.x * kScanBlock + threadIdx.x * kScanPer;
  Fr acc = ident<MUL>();
  for (uint32_t k = 0; k < kScanPer; ++k)
    if (base + k < n) acc = op<MUL>(acc, ldf(&in[phys<SUFFIX>(base + k, n)]));
  sh[threadIdx.x] = acc;
  __syncthreads();
  for (uint32_t h = kScanThreads / 2; h >= 1; h >>= 1) {
    if (threadIdx.x < h) sh[threadIdx.x] = op<MUL>(sh[threadIdx.x], sh[threadIdx.x + h]);
    __syncthreads();
  }
  if (threadIdx.x == 0) stf(&tot[blockIdx.x], sh[0]);
}

// exclusive scan of the block totals in place (single workgroup); tot[nb] = grand total
template <bool MUL>
__global__ void __launch_bounds__(kScanThreads) k_scan_tops(Fr* __restrict__ tot, uint32_t nb) {
  __shared__ Fr sh[kScanThreads];
  const uint32_t per = (nb + kScanThreads - 1) / kScanThreads;
  const uint32_t b0 = threadIdx.x * per;
  Fr acc = ident<MUL>();
  for (uint32_t b = b0; b < b0 + per && b < nb; ++b) acc = op<MUL>(acc, ldf(&tot[b]));
  sh[threadIdx.x] = acc;
  __syncthreads();
  for (uint32_t off = 1; off < kScanThreads; off <<= 1) {
    Fr v = threadIdx.x >= off ? sh[threadIdx.x - off] : ident<MUL>();
    __syncthreads();
    sh[threadIdx.x] = op<MUL>(sh[threadIdx.x], v);
    __syncthreads();
  }
  Fr run = threadIdx.x ? sh[threadIdx.x - 1] : ident<MUL>();
  for (uint32_t b = b0; b < b0 + per && b < nb; ++b) {
    const Fr v = ldf(&tot[b]);
    stf(&tot[b], run);
    run = op<MUL>(run, v);
  }
  if (threadIdx.x == kScanThreads - 1) stf(&tot[nb], sh[kScanThreads - 1]);
}

// Small scans (n <= kScanSingleMax) in ONE dispatch: a workgroup of 1 024 threads, thread t
// owning the per = ceil(n / 1024) consecutive logical elements from t * per (reduce, scan of
// the thread totals, apply). Small proofs are bound by the rate at which the command
// processor takes dispatches (~140 k/s with 16 lanes), and the 3-phase form is 3
// of them per scan.
// (round 5: the 3-phase form from n > 4096 instead measured no faster at 2^13-2^15 proofs,
// profiles/r05_scan_buckets_lds_ab.jsonl)
// The thread totals are scanned inside each wave by shuffles (6 levels, no barrier), the 16
// wave totals by wave 0 the same way, with two barriers in all (round 6; the LDS
// Hillis-Steele scan it replaces took 10 levels over all 16 waves and 20 barriers).
constexpr uint32_t kScanSingleThreads = 1024, kScanSingleMax = 32 * kScanSingleThreads;
constexpr uint32_t kScanSingleWaves = kScanSingleThreads / 64;
__device__ __forceinline__ Fr shfl_up_fr(const Fr& v, uint32_t h) {
  Fr o;
#pragma unroll
  for (int k = 0; k < 8; ++k) o.v[k] = (uint32_t)__shfl_up((int)v.v[k], h, 64);
  return o;
}
// inclusive scan over the 64 lanes of a wave (lane order = operand order)
template <bool MUL>
__device__ __forceinline__ Fr wave_scan_incl(Fr v, uint32_t lane) {
#pragma unroll
  for (uint32_t h = 1; h < 64; h <<= 1) {
    const Fr o = shfl_up_fr(v, h);
    if (lane >= h) v = op<MUL>(o, v);
  }
  return v;
}
// tot[nb] = the grand total, as the 3-phase form leaves it (the grand product's caller reads it)
template <bool MUL, bool SUFFIX, bool EXCL>
__global__ void __launch_bounds__(kScanSingleThreads) k_scan_single(const Fr* __restrict__ in,
                                                                    uint64_t n, Fr* __restrict__ out,
                                                                    Fr* __restrict__ tot, uint32_t nb) {
  __shared__ Fr sh[kScanSingleWaves];
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint32_t per = (uint32_t)((n + kScanSingleThreads - 1) / kScanSingleThreads);
  const uint64_t base = (uint64_t)tid * per;
  Fr acc = ident<MUL>();
  for (uint32_t k = 0; k < per && base + k < n; ++k) acc = op<MUL>(acc, ldf(&in[phys<SUFFIX>(base + k, n)]));
  const Fr incl = wave_scan_incl<MUL>(acc, lane);  // this wave's threads 0 .. lane
  if (lane == 63) sh[wave] = incl;
  __syncthreads();
  if (wave == 0) {  // exclusive prefixes of the wave totals; sh[last] -> the grand total
    const Fr w = lane < kScanSingleWaves ? sh[lane] : ident<MUL>();
    const Fr wi = wave_scan_incl<MUL>(w, lane);
    const Fr we = shfl_up_fr(wi, 1);
    if (lane < kScanSingleWaves) sh[lane] = lane ? we : ident<MUL>();
    if (lane == kScanSingleWaves - 1) stf(&tot[nb], wi);
  }
  __syncthreads();
  const Fr excl_in_wave = shfl_up_fr(incl, 1);
  Fr run = lane ? (wave ? op<MUL>(sh[wave], excl_in_wave) : excl_in_wave)
                : (wave ? sh[wave] : ident<MUL>());
  for (uint32_t k = 0; k < per && base + k < n; ++k) {
    const uint64_t p = phys<SUFFIX>(base + k, n);
    const Fr v = ldf(&in[p]);
    if (EXCL) {
      stf(&out[p], run);
      run = op<MUL>(run, v);
    } else {
      run = op<MUL>(run, v);
      stf(&out[p], run);
    }
  }
}

template <bool MUL, bool SUFFIX, bool EXCL>
__global__ void __launch_bounds__(kScanThreads) k_scan_apply(const Fr* __restrict__ in, uint64_t n,
                                                             const Fr* __restrict__ tot,
                                                             Fr* __restrict__ out) {
  __shared__ Fr sh[kScanThreads];
  const uint64_t base = (uint64_t)blockIdx.x * kScanBlock + threadIdx.x * kScanPer;
  Fr acc = ident<MUL>();
  for (uint32_t k = 0; k < kScanPer; ++k)
    if (base + k < n) acc = op<MUL>(acc, ldf(&in[phys<SUFFIX>(base + k, n)]));
  sh[threadIdx.x] = acc;
  __syncthreads();
  for (uint32_t off = 1; off < kScanThreads; off <<= 1) {
    Fr v = threadIdx.x >= off ? sh[threadIdx.x - off] : ident<MUL>();
    __syncthreads();
    sh[threadIdx.x] = op<MUL>(sh[threadIdx.x], v);
    __syncthreads();
  }
  Fr run = op<MUL>(ldf(&tot[blockIdx.x]), threadIdx.x ? sh[threadIdx.x - 1] : ident<MUL>());
  for (uint32_t k = 0; k < kScanPer; ++k) {
    if (base + k >= n) break;
    const uint64_t p = phys<SUFFIX>(base + k, n);
    const Fr v = ldf(&in[p]);
    if (EXCL) {
      stf(&out[p], run);
      run = op<MUL>(run, v);
    } else {
      run = op<MUL>(run, v);
      stf(&out[p], run);
    }
  }
}

// ------------------------------------------------------------------------ quotient
// Arithmetic, PI, range and permutation terms; FINAL: times 1/v_h and done, else the
// numerator is stored for k_quotient_ext (circuits with logic / curve gates). Keeping those
// widgets out of this kernel holds it at full occupancy (inlined, they need 256 VGPRs).
template <bool FINAL>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3, 3))) k_quotient(QuotientArgs q) {
  // Redundant-limb arithmetic (ffr.hpp) with exponent bookkeeping (QuotientArgs): [e] marks
  // a value stored as x R 2^(-5e); rx_mul(x[e1], y[e2]) = xy[e1 + e2 + 1]; additions need
  // equal exponents. Wires [-1], z / selectors / sigmas / L1 / elements [0].
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t N = q.nq;
  if (i >= N) return;
  // quotient-domain block m (coset g w3^m H_2n), position u; the next row w_n x is u + 2
  const uint64_t blk = i >> q.log_blk, u = i & ((1ull << q.log_blk) - 1);
  const uint64_t nx = (blk << q.log_blk) + ((u + 2) & ((1ull << q.log_blk) - 1));
  const RFr a = ldr(&q.a[i]), b = ldr(&q.b[i]), c = ldr(&q.c[i]), d = ldr(&q.d[i]);
  const RFr z = ldr(&q.z[i]), z_next = ldr(&q.z[nx]);
  // arithmetic widget: q_arith (q_m a b + q_l a + q_r b + q_o c + q_4 d + q_c), terms [0]
  // (pairs of products share one reduction, rx_mul_add; the four terms summed carry-free:
  // limbs below 2^31, value below 8r, times the normalised q_arith: 16 r^2 / R' + r < 2r)
  RFr t = rx_mul(ldr(&q.sel[SEL_QM * N + i]), rx_mul(a, b));
  const RFr lr = rx_mul_add(ldr(&q.sel[SEL_QL * N + i]), a, ldr(&q.sel[SEL_QR * N + i]), b);
  const RFr o4 = rx_mul_add(ldr(&q.sel[SEL_QO * N + i]), c, ldr(&q.sel[SEL_Q4 * N + i]), d);
  const RFr qc = ldr(&q.sel[SEL_QC * N + i]);
#pragma unroll
  for (int l = 0; l < RxShape<FrCfg>::L; ++l) t.v[l] += lr.v[l] + o4.v[l] + qc.v[l];
  t = rx_mul(ldr(&q.sel[SEL_QARITH * N + i]), t);  // [1]
  if (q.pi) t = rx_add(t, ldr(&q.pi[i]));           // public inputs arrive at [1]
  // range widget: sep * q_range * (D(c-4d) + D(b-4c) k + D(a-4b) k^2 + D(d_next-4a) k^3)
  if (q.has_range) {
    const RFr qr = ldr(&q.sel[SEL_QRANGE * N + i]);
    if (!rx_is_zero(qr)) {
      const RFr d_next = ldr(&q.d[nx]);
      const RFr one = rx_unpack(q.rx_one_w), two = rx_unpack(q.rx_two_w),
                three = rx_unpack(q.rx_three_w);  // [-1]
      auto delta = [&](const RFr& f) {          // [-1] -> [-1]
        return rx_mul(rx_mul(f, rx_sub(f, one)), rx_mul(rx_sub(f, two), rx_sub(f, three)));
      };
      auto four = [](const RFr& x) { return rx_dbl(rx_dbl(x)); };
      RFr r = delta(rx_sub(c, four(d)));
      r = rx_add(r, rx_mul(delta(rx_sub(b, four(c))), rx_unpack(q.rx_kappa)));
      r = rx_add(r, rx_mul(delta(rx_sub(a, four(b))), rx_unpack(q.rx_kappa2)));
      r = rx_add(r, rx_mul(delta(rx_sub(d_next, four(a))), rx_unpack(q.rx_kappa3)));
      t = rx_add(t, rx_mul(rx_mul(r, qr), rx_unpack(q.range_sep)));  // [-1] -> [0] -> [1]
    }
  }
  // permutation: alpha [ z (a + bX + g)(b + bK1X + g)(c + bK2X + g)(d + bK3X + g)
  //                    - z_next (a + b s1 + g)(b + b s2 + g)(c + b s3 + g)(d + b s4 + g) ]
  //              + (z - 1) L1(X) alpha^2
  // K1..K3 = 7, 13, 17 (permutation.rs:28-30) by additions
  const RFr bX = rx_mul(rx_unpack(q.rx_bg[blk]), ldr(&q.elements[u]));  // beta s_m w_2n^u [-1]
  const RFr bX2 = rx_dbl(bX), bX4 = rx_dbl(bX2), bX8 = rx_dbl(bX4), bX16 = rx_dbl(bX8);
  const RFr bX7 = rx_sub(bX8, bX), bX13 = rx_add(rx_add(bX8, bX4), bX), bX17 = rx_add(bX16, bX);
  const RFr gm = rx_unpack(q.rx_gamma);  // [-1]
  // the factors are carry-free sums (add3_u), each multiplied by a normalised operand
  RFr id = rx_mul(rx_norm(add3_u(a, bX, gm)), add3_u(b, bX7, gm));
  id = rx_mul(id, add3_u(c, bX13, gm));
  id = rx_mul(id, add3_u(d, bX17, gm));
  id = rx_mul(id, z);  // [0]
  const RFr be = rx_unpack(q.rx_beta);  // [-2]
  RFr cp = rx_norm(add3_u(a, rx_mul(be, ldr(&q.sigma[0 * N + i])), gm));
  cp = rx_mul(cp, add3_u(b, rx_mul(be, ldr(&q.sigma[1 * N + i])), gm));
  cp = rx_mul(cp, add3_u(c, rx_mul(be, ldr(&q.sigma[2 * N + i])), gm));
  cp = rx_mul(cp, add3_u(d, rx_mul(be, ldr(&q.sigma[3 * N + i])), gm));
  cp = rx_mul(cp, z_next);  // [0]
  // alpha^2 L1(X): coset_dft is linear, so alpha^2 * coset_dft(idft(e_0)) equals the
  // reference's coset_dft(idft(alpha^2 e_0)) exactly. alpha (id - cp) + alpha^2 (z - 1) L1
  // with one reduction: (id - cp + 3r) carry-free, (5r * 2r + 2r * 2r) / R' + r < 2r
  const RFr zm1l1 = rx_mul(rx_sub_u<FrCfg, 3>(z, rx_unpack(fe_one<FrCfg>())), ldr(&q.l1[i]));
  const RFr perm = rx_mul_add(rx_sub_u<FrCfg, 3>(id, cp), rx_unpack(q.alpha), zm1l1,
                              rx_unpack(q.rx_alpha2));  // [1]
  if (FINAL) {  // t + perm carry-free (below 4r) times the normalised 1 / v_h
    RFr num = t;
#pragma unroll
    for (int l = 0; l < RxShape<FrCfg>::L; ++l) num.v[l] += perm.v[l];
    stf(&q.out[i], rx_pack_canonical(rx_mul(num, rx_unpack(q.rx_vh[2 * blk + (u & 1)]))));
  } else {
    stf(&q.out[i], rx_pack_canonical(rx_add(t, perm)));  // [1]
  }
}

// out[i] = (out[i] + logic + fixed-base + variable-base terms) / v_h
__global__ void __launch_bounds__(256) k_quotient_ext(QuotientArgs q) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t N = q.nq;
  if (i >= N) return;
  const uint64_t blk = i >> q.log_blk, u = i & ((1ull << q.log_blk) - 1);
  const uint64_t nx = (blk << q.log_blk) + ((u + 2) & ((1ull << q.log_blk) - 1));
  // k_quotient left num at exponent +1 and the wire evaluations are at -1 (QuotientArgs):
  // back to the R domain for the packed arithmetic here
  auto ldw = [&](const Fr* p) { return fe_mul(ldf(p), q.rx_inv32); };
  const Fr a = ldw(&q.a[i]), b = ldw(&q.b[i]), c = ldw(&q.c[i]), d = ldw(&q.d[i]);
  Fr t = fe_mul(ldf(&q.out[i]), q.rx_32);
  // logic widget (dusk-plonk logic gate; zksnarks, un-vendored): quads a = a_next - 4a,
  // b = b_next - 4b, d = d_next - 4d, w = c; sep q_logic (D(a) + D(b) k + D(d) k^2 +
  // (w - ab) k^3 + xor_and(a, b, w, d, q_c) k^4), k = sep^2
  if (q.has_logic) {
    const Fr ql = ldf(&q.sel[SEL_QLOGIC * N + i]);
    if (!fe_is_zero(ql)) {
      const Fr one = fe_one<FrCfg>();
      const Fr two = fe_dbl(one), three = fe_add(two, one), four = fe_dbl(two);
      auto delta = [&](const Fr& f) {
        return fe_mul(fe_mul(f, fe_sub(f, one)), fe_mul(fe_sub(f, two), fe_sub(f, three)));
      };
      const Fr qa = fe_sub(ldw(&q.a[nx]), fe_mul(four, a));
      const Fr qb = fe_sub(ldw(&q.b[nx]), fe_mul(four, b));
      const Fr qd = fe_sub(ldw(&q.d[nx]), fe_mul(four, d));
      const Fr qc = ldf(&q.sel[SEL_QC * N + i]);
      Fr r = delta(qa);
      r = fe_add(r, fe_mul(delta(qb), q.lk));
      r = fe_add(r, fe_mul(delta(qd), q.lk2));
      r = fe_add(r, fe_mul(fe_sub(c, fe_mul(qa, qb)), q.lk3));
      r = fe_add(r, fe_mul(logic_xor_and(qa, qb, c, qd, qc), q.lk4));
      t = fe_add(t, fe_mul(fe_mul(r, ql), q.logic_sep));
    }
  }
  if (q.has_fixed) {
    const Fr qf = ldf(&q.sel[SEL_QFIXED * N + i]);
    if (!fe_is_zero(qf)) {
      const Fr w = widget_fixed_base(a, ldw(&q.a[nx]), b, ldw(&q.b[nx]), c, d, ldw(&q.d[nx]),
                                     ldf(&q.sel[SEL_QL * N + i]), ldf(&q.sel[SEL_QR * N + i]),
                                     ldf(&q.sel[SEL_QC * N + i]), q.fk, q.fk2, q.fk3, q.edwards_d);
      t = fe_add(t, fe_mul(fe_mul(w, qf), q.fixed_sep));
    }
  }
  if (q.has_var) {
    const Fr qv = ldf(&q.sel[SEL_QVAR * N + i]);
    if (!fe_is_zero(qv)) {
      const Fr w = widget_var_base(a, ldw(&q.a[nx]), b, ldw(&q.b[nx]), c, d, ldw(&q.d[nx]),
                                   q.vk, q.vk2, q.edwards_d);
      t = fe_add(t, fe_mul(fe_mul(w, qv), q.var_sep));
    }
  }
  stf(&q.out[i], fe_mul(t, q.vh_inv[2 * blk + (u & 1)]));
}

// t from the three inverse block transforms (pk_coset3_combine, prover.hpp)
__global__ void __launch_bounds__(256) k_coset3_combine(const Fr* __restrict__ in, uint64_t n2,
                                                        Fr c1a, Fr c1b, Fr c1c, Fr c2a, Fr c2b,
                                                        Fr c2c, Fr* __restrict__ out) {
  const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n2) return;
  const RFr b0 = ldr(&in[k]), b1 = ldr(&in[n2 + k]), b2 = ldr(&in[2 * n2 + k]);  // R domain
  stf(&out[k], rx_pack_canonical(rx_add(rx_add(b0, b1), b2)));
  // constants in the R' domain: products land in the R domain
  const RFr e1 = rx_add(rx_mul_add(b0, rx_unpack(c1a), b1, rx_unpack(c1b)), rx_mul(b2, rx_unpack(c1c)));
  stf(&out[n2 + k], rx_pack_canonical(e1));
  const RFr e2 = rx_add(rx_mul_add(b0, rx_unpack(c2a), b1, rx_unpack(c2b)), rx_mul(b2, rx_unpack(c2c)));
  stf(&out[2 * n2 + k], rx_pack_canonical(e2));
}

// ------------------------------------------------------------ scaled table copy
__global__ void k_scale_copy(const Fr* __restrict__ in, Fr c, Fr* __restrict__ out, uint64_t n) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j < n) stf(&out[j], fe_mul(ldf(&in[j]), c));
}

// -------------------------------------------------------------------- evaluation
constexpr uint32_t kEvalThreads = 256, kEvalPer = 16, kEvalBlock = kEvalThreads * kEvalPer;

// x^(b * 4096) from x4096 = x^4096 by square-and-multiply over the bits of b: at most
// 2 log2(b) multiplies, where fe_pow_u64(x, b * 4096) would chain ~1.5 * log2(b * 4096)
// of them (~380 at n = 2^23, run by one thread while its workgroup waits)
__device__ __forceinline__ Fr pow_blocks(Fr x4096, uint64_t b) {
  Fr r = fe_one<FrCfg>();
  for (; b; b >>= 1) {
    if (b & 1) r = fe_mul(r, x4096);
    x4096 = fe_sqr(x4096);
  }
  return r;
}

// the same in the R' domain of ffr.hpp (x4096 and the result R'-domain, [0, 2r))
__device__ __forceinline__ RFr pow_blocks_rx(RFr x4096, uint64_t b) {
  RFr r = rx_one<FrCfg>();
  for (; b; b >>= 1) {
    if (b & 1) r = rx_mul(r, x4096);
    x4096 = rx_sqr(x4096);
  }
  return r;
}

// partial[k][blk] = sum_{j in block} c_j x^j (poly k of the batch). Thread t runs Horner
// in x^256 over c_{block + t + 256 i}, i < kEvalPer (consecutive threads read consecutive
// coefficients: coalesced), giving H_t with sum_j c_j x^j = sum_t x^t H_t; the workgroup
// folds that by halving (H_t += x^h H_{t+h}, h = 128 .. 1) with x^h from 8 squarings; one
// power x^(block start) per block (pow_blocks).
__global__ void __launch_bounds__(kEvalThreads) k_eval_partial(EvalBatch e, Fr* __restrict__ partial,
                                                               uint32_t max_blocks) {
  // redundant-limb arithmetic: coefficients R-domain, powers of x R'-domain (the host
  // converts e.x), so every product lands in the R domain; LDS holds packed [0, 2r) values
  __shared__ Fr sh[kEvalThreads];
  __shared__ Fr xp[9];  // x^(2^l), l = 0..8 (x^256 last), R'
  __shared__ Fr xblock;
  const uint32_t k = blockIdx.y, tid = threadIdx.x;
  const Fr* p = e.poly[k];
  const uint64_t len = e.len[k];
  const uint64_t block0 = (uint64_t)blockIdx.x * kEvalBlock;
  if (block0 >= len) {  // whole block past this polynomial's end (uniform per block)
    if (tid == 0) stf(&partial[(size_t)k * max_blocks + blockIdx.x], fe_zero<FrCfg>());
    return;
  }
  if (tid == 0) {
    RFr t = rx_unpack(e.x[k]);
    for (int l = 0; l < 9; ++l) {
      xp[l] = rx_pack(t);
      t = rx_sqr(t);
    }
    for (int l = 9; l < 12; ++l) t = rx_sqr(t);  // x^4096
    xblock = rx_pack(pow_blocks_rx(t, blockIdx.x));
  }
  __syncthreads();
  const RFr x256 = rx_unpack(xp[8]);
  RFr acc = rx_zero<FrCfg>();
#pragma unroll
  for (int i = (int)kEvalPer - 1; i >= 0; --i) {
    const uint64_t j = block0 + tid + (uint64_t)i * kEvalThreads;
    acc = rx_mul(acc, x256);
    if (j < len) acc = rx_add(acc, ldr(&p[j]));
  }
  sh[tid] = rx_pack(acc);
  __syncthreads();
  for (int l = 7; l >= 0; --l) {
    const uint32_t h = 1u << l;
    if (tid < h)
      sh[tid] = rx_pack(rx_add(rx_unpack(sh[tid]), rx_mul(rx_unpack(sh[tid + h]), rx_unpack(xp[l]))));
    __syncthreads();
  }
  if (tid == 0)
    stf(&partial[(size_t)k * max_blocks + blockIdx.x],
        rx_pack_canonical(rx_mul(rx_unpack(sh[0]), rx_unpack(xblock))));
}

__global__ void __launch_bounds__(kEvalThreads) k_eval_final(const Fr* __restrict__ partial,
                                                             uint32_t nblocks, uint32_t max_blocks,
                                                             Fr* __restrict__ out) {
  __shared__ Fr sh[kEvalThreads];
  const uint32_t k = blockIdx.x;
  Fr acc = fe_zero<FrCfg>();
  for (uint32_t b = threadIdx.x; b < nblocks; b += kEvalThreads)
    acc = fe_add(acc, ldf(&partial[(size_t)k * max_blocks + b]));
  sh[threadIdx.x] = acc;
  __syncthreads();
  for (uint32_t h = kEvalThreads / 2; h >= 1; h >>= 1) {
    if (threadIdx.x < h) sh[threadIdx.x] = fe_add(sh[threadIdx.x], sh[threadIdx.x + h]);
    __syncthreads();
  }
  if (threadIdx.x == 0) stf(&out[k], sh[0]);
}

// Ruffini for small polynomials (len <= kRuffiniSingleMax) in ONE dispatch instead of five
// (pk_ruffini: scale powers, 3-phase scan, scale powers): q_k = z^-(k+1) sum_(i>k) c_i z^i.
// A workgroup of 1 024 threads; thread t owns j in [tE, tE + E) (E = ceil(len / 1024) <= 16).
// Pass 1 (upward) forms y_j = c_j z^j and the thread's sum, parking y_j in q[j]; an exclusive
// suffix scan of the sums over the threads (LDS) gives each thread the sum of y above its
// range; pass 2 walks its range downward with that running sum (2 products per element there
// instead of 4: y_j is read back, not recomputed; 2^12 proofs within noise of the round-3 form,
// profiles/r04_ruffini_park_ab.jsonl). Start powers z^(tE) and z^-(tE+1) (round 6): t = 32 hi +
// lo, so z^(tE) = z^(E lo) z^(32E hi); two waves first build the four 32-entry tables
// z^(E i), z^(32E i), z^-(E i), z^-(32E i) from the host's binary powers (5 products each, in
// parallel), then every thread takes 2 (3) products — 6 dependent products and one barrier
// where the product scans of z^E / z^-E in LDS took 10 levels and 20 barriers. All powers
// R'-domain (the host converts), products in the R domain, outputs canonical: the same field
// values as the five-dispatch form.
constexpr uint32_t kRuffiniThreads = 1024, kRuffiniSingleMax = 16 * kRuffiniThreads;
static_assert(kRuffiniThreads == 32 * 32, "start powers: t = 32 hi + lo");
struct RuffiniPow {
  Fr up[10];  // z^(E 2^b), R'-domain
  Fr dn[10];  // z^-(E 2^b), R'-domain
};
__global__ void __launch_bounds__(kRuffiniThreads) k_ruffini_single(const Fr* __restrict__ c, uint64_t len,
                                                                    uint32_t E, Fr z, Fr zi,
                                                                    RuffiniPow pw2, Fr* __restrict__ q) {
  __shared__ Fr P[4][32];
  __shared__ Fr W[kRuffiniThreads / 64];
  const uint32_t tid = threadIdx.x;
  if (tid < 128) {  // table tb (0: z^(E i), 1: z^(32E i), 2 / 3: the inverses), entry i
    const uint32_t tb = tid >> 5, i = tid & 31;
    RFr v = rx_one<FrCfg>();
#pragma unroll
    for (int b = 0; b < 5; ++b) {
      Fr f;  // word by word (a lane-dependent pick of a by-value argument goes through scratch)
#pragma unroll
      for (int k = 0; k < 8; ++k)
        f.v[k] = tb < 2 ? (tb == 0 ? pw2.up[b].v[k] : pw2.up[b + 5].v[k])
                        : (tb == 2 ? pw2.dn[b].v[k] : pw2.dn[b + 5].v[k]);
      const RFr m = rx_mul(v, rx_unpack(f));
      if ((i >> b) & 1) v = m;
    }
    P[tb][i] = rx_pack(v);
  }
  __syncthreads();
  const uint64_t j0 = (uint64_t)tid * E;
  const uint64_t j1 = j0 + E < len ? j0 + E : (j0 < len ? len : j0);
  const RFr zr = rx_unpack(z), zir = rx_unpack(zi);
  RFr pw = rx_mul(rx_unpack(P[0][tid & 31]), rx_unpack(P[1][tid >> 5]));  // z^j0
  RFr pwi = rx_mul(rx_mul(zir, rx_unpack(P[2][tid & 31])), rx_unpack(P[3][tid >> 5]));  // z^-(j0 + 1)
  Fr loc = fe_zero<FrCfg>(), ylast = fe_zero<FrCfg>();
  for (uint64_t j = j0; j < j1; ++j) {  // pass 1: this thread's sum of y_j
    const Fr y = rx_pack_canonical(rx_mul(ldr(&c[j]), pw));
    loc = fe_add(loc, y);
    // y_j parked in q[j] for pass 2 (q[j] is this thread's and is rewritten there; q holds
    // len - 1 entries, so the top y stays in a register)
    if (j + 1 < len) stf(&q[j], y);
    else ylast = y;
    pw = rx_mul(pw, zr);
    pwi = rx_mul(pwi, zir);
  }
  // inclusive suffix sums of the threads' sums: inside each wave by cross-lane shuffles, then
  // the totals of the waves above from LDS (one barrier instead of a 10-level LDS scan's 20)
  Fr v = loc;
  const uint32_t lane = tid & 63, wave = tid >> 6;
#pragma unroll
  for (uint32_t h = 1; h < 64; h <<= 1) {
    Fr o;
#pragma unroll
    for (int k = 0; k < 8; ++k) o.v[k] = (uint32_t)__shfl_down((int)v.v[k], h, 64);
    if (lane + h < 64) v = fe_add(v, o);
  }
  if (lane == 0) W[wave] = v;
  __syncthreads();
  Fr run = fe_sub(v, loc);  // sum of y_i over i >= j1: this wave's part ...
  for (uint32_t w = wave + 1; w < kRuffiniThreads / 64; ++w) run = fe_add(run, W[w]);  // ... the rest
  // pass 2, downward from j1 - 1: pwi = z^-(j1 + 1) -> z^-(k + 1); y_k back from q[k]
  for (uint64_t k = j1; k-- > j0;) {
    pwi = rx_mul(pwi, zr);
    const bool in_q = k + 1 < len;
    const Fr yk = in_q ? ldf(&q[k]) : ylast;  // read before q[k] is rewritten
    if (in_q) stf(&q[k], rx_pack_canonical(rx_mul(rx_unpack(run), pwi)));
    run = fe_add(run, yk);
  }
}

// ---------------------------------------------------------------- linear combos
// out[j] = sum_t s_t * p_t[j] (p_t[j] = 0 past len_t), j < len_out
// (redundant limbs: the scalars arrive in the R' domain, pk_lincomb)
__global__ void k_lincomb(LinComb lc, Fr* __restrict__ out, uint64_t len_out) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= len_out) return;
  RFr acc = rx_zero<FrCfg>();
  for (uint32_t t = 0; t < lc.terms; ++t)
    if (j < lc.len[t]) acc = rx_add(acc, rx_mul(rx_unpack(lc.s[t]), ldr(&lc.p[t][j])));
  stf(&out[j], rx_pack_canonical(acc));
}

// y_j = c_j x^(j + shift). A block covers 256 x 16 consecutive j; the per-thread start
// powers x^(block start + shift) * (x^16)^t come from an 8-step product scan in LDS. The
// host passes x^16, x^4096 and x^shift (one chain of squarings there instead of one per
// workgroup's first lane, which sat on every launch's critical path).
__global__ void __launch_bounds__(256) k_scale_powers(const Fr* __restrict__ c, uint64_t len, Fr x,
                                                      Fr x16, Fr x4096, Fr xshift,
                                                      Fr* __restrict__ y) {
  // redundant limbs: the powers live in the R' domain (the host converts x, x^16, x^4096
  // and x^shift), so c_j x^j lands in the R domain of c
  __shared__ Fr T[256];
  const uint32_t tid = threadIdx.x;
  const uint64_t jb = (uint64_t)blockIdx.x * 256 * 16;
  RFr v = rx_unpack(x16);
  if (tid == 0) v = rx_mul(pow_blocks_rx(rx_unpack(x4096), blockIdx.x), rx_unpack(xshift));
  T[tid] = rx_pack(v);
  __syncthreads();
  for (uint32_t h = 1; h < 256; h <<= 1) {  // inclusive product scan
    const RFr o = tid >= h ? rx_unpack(T[tid - h]) : rx_one<FrCfg>();
    __syncthreads();
    if (tid >= h) T[tid] = rx_pack(rx_mul(rx_unpack(T[tid]), o));
    __syncthreads();
  }
  const uint64_t j0 = jb + (uint64_t)tid * 16;
  if (j0 >= len) return;
  RFr pw = rx_unpack(T[tid]);
  const RFr xr = rx_unpack(x);
  const uint64_t j1 = j0 + 16 < len ? j0 + 16 : len;
  for (uint64_t j = j0; j < j1; ++j) {
    stf(&y[j], rx_pack_canonical(rx_mul(ldr(&c[j]), pw)));
    pw = rx_mul(pw, xr);
  }
}

}  // namespace

// ============================================================== host launchers
int pk_gather_wires(const Fr* witness, const uint32_t* idx, uint64_t m, uint64_t n, Fr* out,
                    hipStream_t s) {
  hipLaunchKernelGGL(k_gather_wires, dim3(blocks_for(n, 256), 4), dim3(256), 0, s, witness, idx, m,
                     n, out);
  PLK_HIP_TRY(hipGetLastError());
  return PLK_OK;
}

int pk_blind(Fr* poly, uint64_t n, const BlindArgs& b, hipStream_t s) {
  hipLaunchKernelGGL(k_blind, dim3(1), dim3(64), 0, s, poly, n, b);
  PLK_HIP_TRY(hipGetLastError());
  return PLK_OK;
}

int pk_pi_coef(const PiDirect& pd, const Fr* tw_inv, uint64_t n, Fr* out, hipStream_t s) {
  if (pd.count > (uint32_t)kPiDirect || (n & (n - 1))) return PLK_E_ARG;
  hipLaunchKernelGGL(k_pi_coef, dim3(blocks_for(n, 256)), dim3(256), 0, s, pd, tw_inv, n, out);
  PLK_HIP_TRY(hipGetLastError());
  return PLK_OK;
}

int pk_blind_batch(const BlindBatch& bb, uint64_t n, hipStream_t s) {
  hipLaunchKernelGGL(k_blind_batch, dim3(1), dim3(64), 0, s, bb, n);
  PLK_HIP_TRY(hipGetLastError());
  return PLK_OK;
}

int pk_fill(Fr* out, const Fr& v, uint64_t n, hipStream_t s) {
  hipLaunchKernelGGL(k_fill, dim3(blocks_for(n, 256)), dim3(256), 0, s, out, v, n);
  PLK_HIP_TRY(hipGetLastError());
  return PLK_OK;
}

int pk_perm_numden(const Fr* wires, const Fr* sigmas, const Fr* elements, uint64_t n,
                   const Fr& beta, const Fr& gamma, const Fr& k1, const Fr& k2, const Fr& k3,
                   Fr* num, Fr* den, hipStream_t s) {
  Fr fix = fe_zero<FrCfg>();  // 2^276 mod r = R'^4 / R^3 (k_perm_numden)
  fix.v[0] = 1;
  for (int b = 0; b < 4 * RxShape<FrCfg>::B * RxShape<FrCfg>::L - 3 * 256; ++b) fix = fe_dbl(fix);
  hipLaunchKernelGGL(k_perm_numden, dim3(blocks_for(n, 256)), dim3(256), 0, s, wires, sigmas,
                     elements, n, fe_to_rx_domain(beta), gamma, fe_to_rx_domain(k1),
                     fe_to_rx_domain(k2), fe_to_rx_domain(k3), fix, num, den);
  PLK_HIP_TRY(hipGetLastError());
  return PLK_OK;
}

int pk_mul3(const Fr* a, const Fr* b, const Fr& c, Fr* out, uint64_t n, hipStream_t s) {
  hipLaunchKernelGGL(k_mul3, dim3(blocks_for(n, 256)), dim3(256), 0, s, a, b, c, out, n);
  PLK_HIP_TRY(hipGetLastError());
  return PLK_OK;
}

uint64_t pk_scan_tmp_elems(uint64_t n) { return (n + kScanBlock - 1) / kScanBlock + 1; }

int pk_scan(const Fr* in, Fr* out, uint64_t n, bool mul, bool suffix, bool exclusive, Fr* tmp,
            hipStream_t s) {
  if (n == 0) return PLK_OK;
  const uint32_t nb = (uint32_t)((n + kScanBlock - 1) / kScanBlock);
  const bool single = n <= kScanSingleMax;
#define SCAN3(M, S, E)                                                                           \
  do {                                                                                           \
    if (single) {                                                                                \
      hipLaunchKernelGGL((k_scan_single<M, S, E>), dim3(1), dim3(kScanSingleThreads), 0, s, in, n, \
                         out, tmp, nb);                                                          \
      break;                                                                                     \
    }                                                                                            \
    hipLaunchKernelGGL((k_scan_reduce<M, S>), dim3(nb), dim3(kScanThreads), 0, s, in, n, tmp);   \
    hipLaunchKernelGGL((k_scan_tops<M>), dim3(1), dim3(kScanThreads), 0, s, tmp, nb);            \
    hipLaunchKernelGGL((k_scan_apply<M, S, E>), dim3(nb), dim3(kScanThreads), 0, s, in, n, tmp,   \
                       out);                                                                     \
  } while (0)
  if (mul) {
    if (suffix) {
      if (exclusive) SCAN3(true, true, true); else SCAN3(true, true, false);
    } else {
      if (exclusive) SCAN3(true, false, true); else SCAN3(true, false, false);
    }
  } else {
    if (suffix) {
      if (exclusive) SCAN3(false, true, true); else SCAN3(false, true, false);
    } else {
      if (exclusive) SCAN3(false, false, true); else SCAN3(false, false, false);
    }
  }
#undef SCAN3
  PLK_HIP_TRY(hipGetLastError());
  return PLK_OK;
}

int pk_coset3_combine(const Fr* in, uint64_t n2, const Fr* comb, Fr* out, hipStream_t s) {
  hipLaunchKernelGGL(k_coset3_combine, dim3(blocks_for(n2, 256)), dim3(256), 0, s, in, n2, comb[0],
                     comb[1], comb[2], comb[3], comb[4], comb[5], out);
  PLK_HIP_TRY(hipGetLastError());
  return PLK_OK;
}

int pk_quotient(const QuotientArgs& q, hipStream_t s) {
  const dim3 grid(blocks_for(q.nq, 256));
  if (q.has_logic || q.has_fixed || q.has_var) {
    hipLaunchKernelGGL((k_quotient<false>), grid, dim3(256), 0, s, q);
    hipLaunchKernelGGL(k_quotient_ext, grid, dim3(256), 0, s, q);
  } else {
    hipLaunchKernelGGL((k_quotient<true>), grid, dim3(256), 0, s, q);
  }
  PLK_HIP_TRY(hipGetLastError());
  return PLK_OK;
}

uint32_t pk_eval_max_blocks(uint64_t max_len) {
  return (uint32_t)((max_len + kEvalBlock - 1) / kEvalBlock);
}

int pk_scale_copy(const Fr* in, const Fr& c, Fr* out, uint64_t n, hipStream_t s) {
  if (n == 0) return PLK_OK;
  hipLaunchKernelGGL(k_scale_copy, dim3(blocks_for(n, 256)), dim3(256), 0, s, in, c, out, n);
  PLK_HIP_TRY(hipGetLastError());
  return PLK_OK;
}

int pk_eval(const EvalBatch& e, uint32_t count, uint64_t max_len, Fr* partial, Fr* d_out,
            hipStream_t s) {
  const uint32_t mb = pk_eval_max_blocks(max_len ? max_len : 1);
  EvalBatch er = e;  // evaluation points in the R' domain (k_eval_partial)
  for (uint32_t k = 0; k < count; ++k) er.x[k] = fe_to_rx_domain(e.x[k]);
  hipLaunchKernelGGL(k_eval_partial, dim3(mb, count), dim3(kEvalThreads), 0, s, er, partial, mb);
  hipLaunchKernelGGL(k_eval_final, dim3(count), dim3(kEvalThreads), 0, s, partial, mb, mb, d_out);
  PLK_HIP_TRY(hipGetLastError());
  return PLK_OK;
}

int pk_lincomb(const LinComb& lc, Fr* out, uint64_t len_out, hipStream_t s) {
  if (len_out == 0) return PLK_OK;
  LinComb lr = lc;  // scalars in the R' domain (k_lincomb)
  for (uint32_t t = 0; t < lc.terms; ++t) lr.s[t] = fe_to_rx_domain(lc.s[t]);
  hipLaunchKernelGGL(k_lincomb, dim3(blocks_for(len_out, 256)), dim3(256), 0, s, lr, out, len_out);
  PLK_HIP_TRY(hipGetLastError());
  return PLK_OK;
}

int pk_scale_powers(const Fr* c, uint64_t len, const Fr& x, uint64_t shift, Fr* y, hipStream_t s) {
  if (len == 0) return PLK_OK;
  Fr x16 = x;
  for (int i = 0; i < 4; ++i) x16 = fe_sqr(x16);
  Fr x4096 = x16;
  for (int i = 0; i < 8; ++i) x4096 = fe_sqr(x4096);
  const Fr xshift = fe_pow_u64(x, shift);
  hipLaunchKernelGGL(k_scale_powers, dim3(blocks_for((len + 15) / 16, 256)), dim3(256), 0, s, c, len,
                     fe_to_rx_domain(x), fe_to_rx_domain(x16), fe_to_rx_domain(x4096),
                     fe_to_rx_domain(xshift), y);
  PLK_HIP_TRY(hipGetLastError());
  return PLK_OK;
}

// Ruffini: q(X) = (p(X) - p(z)) / (X - z), q_k = z^-(k+1) * sum_{j>k} c_j z^j, len(q) = len - 1.
// tmp holds len elements + scan tmp.
int pk_ruffini(const Fr* c, uint64_t len, const Fr& z, Fr* q, Fr* tmp, Fr* scan_tmp,
               hipStream_t s) {
  if (len <= 1) return PLK_OK;
  int st;
  if (len <= kRuffiniSingleMax) {  // one dispatch (k_ruffini_single)
    const uint32_t E = (uint32_t)((len + kRuffiniThreads - 1) / kRuffiniThreads);
    const Fr zinv = fe_inv(z);
    RuffiniPow pw2;
    Fr up = fe_pow_u64(z, E), dn = fe_pow_u64(zinv, E);
    for (int b = 0; b < 10; ++b) {
      pw2.up[b] = fe_to_rx_domain(up);
      pw2.dn[b] = fe_to_rx_domain(dn);
      up = fe_sqr(up);
      dn = fe_sqr(dn);
    }
    hipLaunchKernelGGL(k_ruffini_single, dim3(1), dim3(kRuffiniThreads), 0, s, c, len, E,
                       fe_to_rx_domain(z), fe_to_rx_domain(zinv), pw2, q);
    PLK_HIP_TRY(hipGetLastError());
    return PLK_OK;
  }
  if ((st = pk_scale_powers(c, len, z, 0, tmp, s))) return st;          // y_j = c_j z^j
  if ((st = pk_scan(tmp, tmp, len, false, true, true, scan_tmp, s))) return st;  // S_j = sum_{i>j} y_i
  const Fr zinv = fe_inv(z);
  return pk_scale_powers(tmp, len - 1, zinv, 1, q, s);                  // q_k = S_k z^-(k+1)
}

}  // namespace plk
