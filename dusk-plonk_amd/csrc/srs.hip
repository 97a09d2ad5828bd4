// srs.hip — PlonkParams::setup (SRS generation) and the MSM window tables, on gfx950.
//
// setup(k, rng) (zksnarks, un-vendored; tests/*.rs:24) restated with an
// explicit secret tau: g1[i] = [tau^i] G1. The MSM (msm.hip) additionally needs
// table[w][i] = 2^(o_w - s_w) * g1[i] in affine form (balanced windows, msm_prepare_srs); both are produced here with XYZZ
// arithmetic and converted to affine by batch inversion (Montgomery's trick, one Fermat
// inversion per kBatchAff points).
#include <hip/hip_runtime.h>

#include "internal.hpp"
#include "msm_common.hpp"
#include "ffr.hpp"

namespace plk {

namespace {

// ---- table construction --------------------------------------------------------------
// temp[i] = 2^c * src[i]  (XYZZ)
__global__ void __launch_bounds__(256) k_double_c(const G1Affine* __restrict__ src, const uint8_t* __restrict__ src_inf,
                           uint64_t n, uint32_t c, G1xyzz* __restrict__ temp) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  G1xyzz acc;
  if (src_inf[i]) {
    acc = xyzz_infinity();
  } else {
    Fp x, y;
    ld_aff(&src[i], x, y);
    acc = xyzz_from_affine(G1Affine{x, y});
  }
  for (uint32_t k = 0; k < c; ++k) acc = xyzz_dbl(acc);
  st_xyzz(&temp[i], acc);
}

// temp[i] = [tau^i] G  (XYZZ), double-and-add on the canonical exponent
__global__ void __launch_bounds__(128) k_srs_powers(Fr tau, G1Affine gen, uint64_t start, uint64_t n,
                                                   G1xyzz* __restrict__ temp) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const Fr s = fe_from_mont(fe_pow_u64(tau, start + i));
  G1xyzz acc = xyzz_infinity();
  for (int b = 254; b >= 0; --b) {
    acc = xyzz_dbl(acc);
    if ((s.v[b >> 5] >> (b & 31)) & 1u) acc = xyzz_add_affine(acc, gen.x, gen.y);
  }
  st_xyzz(&temp[i], acc);
}

// Batch conversion XYZZ -> affine, one thread per kBatchAff consecutive points
// (Montgomery's trick on ZZZ; prefix products kept in `pref`).
__global__ void __launch_bounds__(128) k_batch_affine(const G1xyzz* __restrict__ temp, uint64_t n, Fp* __restrict__ pref,
                               G1Affine* __restrict__ out, uint8_t* __restrict__ out_inf) {
  const uint64_t chunk = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t i0 = chunk * kBatchAff;
  if (i0 >= n) return;
  const uint64_t i1 = i0 + kBatchAff < n ? i0 + kBatchAff : n;
  Fp acc = fe_one<FpCfg>();
  for (uint64_t i = i0; i < i1; ++i) {
    G1xyzz p;
    ld_xyzz(&temp[i], p);
    if (!xyzz_is_inf(p)) acc = fe_mul(acc, p.ZZZ);
    st_fp(reinterpret_cast<uint32_t*>(&pref[i]), acc);
  }
  Fp inv = fe_inv(acc);
  for (uint64_t i = i1; i-- > i0;) {
    G1xyzz p;
    ld_xyzz(&temp[i], p);
    if (xyzz_is_inf(p)) {
      st_aff(&out[i], fe_zero<FpCfg>(), fe_zero<FpCfg>());
      out_inf[i] = 1;
      continue;
    }
    Fp prev = fe_one<FpCfg>();
    if (i > i0) ld_fp(reinterpret_cast<const uint32_t*>(&pref[i - 1]), prev);
    const Fp u = fe_mul(inv, prev);  // 1 / ZZZ_i
    inv = fe_mul(inv, p.ZZZ);
    const Fp zzinv = fe_sqr(fe_mul(p.ZZ, u));
    st_aff(&out[i], fe_mul(p.X, zzinv), fe_mul(p.Y, u));
    out_inf[i] = 0;
  }
}

// The accumulation reads the table in the R' domain of ffr.hpp: x -> x * 2^8 (canonical).
__global__ void __launch_bounds__(256) k_table_to_rx(G1Affine* __restrict__ tab, uint64_t count) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  Fp x, y;
  ld_aff(&tab[i], x, y);
  st_aff(&tab[i], fe_to_rx_domain(x), fe_to_rx_domain(y));
}

}  // namespace

// Window size for an SRS of n points (bucket count 2^(c-1); table W*n, W = ceil(255/c)).
static uint32_t choose_c(size_t n) {
  // PLK_MSM_C (tests, experiments): a fixed window size for every SRS prepared afterwards
  if (const char* e = getenv("PLK_MSM_C")) {
    const int c = atoi(e);
    // the balanced window layout needs (c - 1) ceil(255 / c) <= 255: not c = 21, 23
    if (c >= 8 && c <= 22 && c != 21) return (uint32_t)c;
  }
  // 2^20 points and up: c = 20, 13 windows (16 at c = 16). Entries N * W fall 19 %; the
  // 2^19 buckets (~26 entries each) go through the wide-set sort and the run-sum
  // reduction (msm.hip), ~2.2 additions per bucket. Per MSM: N * ceil(255 / c) mixed
  // additions + ~2.2 * 2^(c-1) full ones is smallest at c = 20 for N = 2^20.
#ifndef PLK_C_HUGE
#define PLK_C_HUGE 20
#endif
  if (n >= (1u << 20)) return PLK_C_HUGE;
  // 2^16 .. 2^20 points: c = 17, 15 windows of exactly 255 bits (no short top window), 2^16
  // buckets through the wide-set path. 2^16 bench (tools/gpu_c_sweep.sh, same box, twice):
  // c = 15 20.3 / 20.3, 16 18.9 / 18.3, 17 20.7 / 21.1 M constraints/s; c = 18 (and 19 at 2^20)
  // collapse to 8.4 (17.6) M: their top windows hold 2 (7) bits, so every scalar's top digit
  // lands in one of 4 (128) buckets of 2^16 (8 192) entries each, summed by single lanes
#ifndef PLK_C_LARGE
#define PLK_C_LARGE 17
#endif
  if (n >= (1u << 16)) return PLK_C_LARGE;
// 2^15 .. 2^16 points: c = 15 (17 windows of exactly 255 bits); 2^16 bench 18.3 -> 19.4 M
// constraints/s against 13 in round 1 (tools/gpu_ab_c.sh); round 5 (balanced windows,
// profiles/r05_window_sizes_ab.jsonl): 2^15 proofs at c = 13 / 14 / 15 20.44 / 20.15 / 20.49 M
#ifndef PLK_C_MID
#define PLK_C_MID 15
#endif
  if (n >= (1u << 15)) return PLK_C_MID;
  // 2^13 .. 2^15 points (round 5): the short top window that made c = 11-14 lose in round 4
  // (a few hot buckets) is gone with the balanced windows, and fewer buckets shorten the
  // reduction tail: 2^14 proofs at c = 13 / 14 / 15 16.86 / 16.71 / 15.70 M (and 17.49 /
  // 17.20 / 16.16 M on another box), 2^13 at c = 10 / 12 / 13 12.48 / 13.09 / 12.80 M; 2^12
  // keeps c = 10 (c = 11 / 12 / 13 9.13 / 9.24 / 9.21 against 9.32 M)
  if (n >= (1u << 14)) return 13;
  if (n >= (1u << 13)) return 12;
  if (n >= (1u << 10)) return 10;
  return 8;
}

int msm_prepare_srs(plk_srs* s, hipStream_t stream) {
  s->c = choose_c(s->n);
  // every window would be c - 1 bits (c = 18: 15 x 17 = 255): that is the c - 1 layout
  if ((s->c - 1) * ((255 + s->c - 1) / s->c) == 255) s->c -= 1;
  s->windows = (255 + s->c - 1) / s->c;  // scalars recoded from [0, (r-1)/2] (< 2^254)
  // balanced windows (round 5): the W windows cover exactly 255 bits, the top `narrow` = c W -
  // 255 of them c - 1 bits wide with digits scaled by 2 (msm.hip digit_at) and table rows
  // pre-divided by 2, so every window spreads over all 2^(c-1) buckets: even buckets hold the
  // wide windows' entries, odd ones also the narrow windows' (c = 20: 8 x 20 + 5 x 19 bits,
  // 16 / 36 entries per 2^20 scalars, every run of >= 2 buckets the same load). Round 4's
  // short top window (c = 20: 14 bits, digits x 32) piled 2^20 entries onto 2^14 buckets,
  // 88 entries against 24: chains in the reduction of a part of a split MSM and in the narrow
  // path's bucket sums (c = 10: 16 buckets at 2.3x)
  s->narrow = s->c * s->windows - 255;
  const size_t n = s->n;
  int st;
  if ((st = s->table.alloc((size_t)s->windows * n * sizeof(G1Affine)))) return st;
  if ((st = s->table_inf.alloc((size_t)s->windows * n))) return st;
  PLK_HIP_TRY(hipMemcpyAsync(s->table.ptr, s->points.ptr, n * sizeof(G1Affine),
                             hipMemcpyDeviceToDevice, stream));
  PLK_HIP_TRY(hipMemcpyAsync(s->table_inf.ptr, s->inf.ptr, n, hipMemcpyDeviceToDevice, stream));
  DevBuf temp, pref;
  if ((st = temp.alloc(n * sizeof(G1xyzz)))) return st;
  if ((st = pref.alloc(n * sizeof(Fp)))) return st;
  G1Affine* tab = s->table.as<G1Affine>();
  uint8_t* tinf = s->table_inf.as<uint8_t>();
  // row w = 2^(o_w - s_w) P (o_w the window's bit offset, s_w = 1 for narrow windows): from
  // row w - 1 by c doublings while both are wide, c - 1 from the first narrow one on
  for (uint32_t w = 1; w < s->windows; ++w) {
    hipLaunchKernelGGL(k_double_c, dim3(cdiv(n, 256)), dim3(256), 0, stream, tab + (w - 1) * n,
                       tinf + (w - 1) * n, (uint64_t)n,
                       w < s->windows - s->narrow ? s->c : s->c - 1, temp.as<G1xyzz>());
    hipLaunchKernelGGL(k_batch_affine, dim3(cdiv(cdiv(n, kBatchAff), 128)), dim3(128), 0, stream,
                       temp.as<G1xyzz>(), (uint64_t)n, pref.as<Fp>(), tab + w * n, tinf + w * n);
    PLK_HIP_TRY(hipGetLastError());
  }
  // table holds R-domain points up to here (each window doubles the previous one); the
  // MSM reads it in the R' domain
  hipLaunchKernelGGL(k_table_to_rx, dim3(cdiv((uint64_t)s->windows * n, 256)), dim3(256), 0, stream,
                     tab, (uint64_t)s->windows * n);
  PLK_HIP_TRY(hipGetLastError());
  PLK_HIP_TRY(stream_wait(stream));
  s->ws.reset(new MsmWorkspace());
  const int r = ws_reserve(s, *s->ws, n, 1, stream);
  if (r != PLK_OK) return r;
  PLK_HIP_TRY(stream_wait(stream));
  return PLK_OK;
}

int srs_generate(plk_srs* s, const Fr& tau_mont, uint64_t start, hipStream_t stream) {
  const size_t n = s->n;
  int st;
  DevBuf temp, pref;
  if ((st = temp.alloc(n * sizeof(G1xyzz)))) return st;
  if ((st = pref.alloc(n * sizeof(Fp)))) return st;
  // G1 generator (Montgomery form)
  static const uint32_t gx[12] = {0xdb22c6bbu, 0xfb3af00au, 0xf97a1aefu, 0x6c55e83fu,
                                  0x171bac58u, 0xa14e3a3fu, 0x9774b905u, 0xc3688c4fu,
                                  0x4fa9ac0fu, 0x2695638cu, 0x3197d794u, 0x17f1d3a7u};
  static const uint32_t gy[12] = {0x46c5e7e1u, 0x0caa2329u, 0xa2888ae4u, 0xd03cc744u,
                                  0x2c04b3edu, 0x00db18cbu, 0xd5d00af6u, 0xfcf5e095u,
                                  0x741d8ae4u, 0xa09e30edu, 0xe3aaa0f1u, 0x08b3f481u};
  G1Affine gen;
  for (int i = 0; i < 12; ++i) {
    gen.x.v[i] = gx[i];
    gen.y.v[i] = gy[i];
  }
  gen.x = fe_to_mont(gen.x);
  gen.y = fe_to_mont(gen.y);
  hipLaunchKernelGGL(k_srs_powers, dim3(cdiv(n, 128)), dim3(128), 0, stream, tau_mont, gen,
                     start, (uint64_t)n, temp.as<G1xyzz>());
  hipLaunchKernelGGL(k_batch_affine, dim3(cdiv(cdiv(n, kBatchAff), 128)), dim3(128), 0, stream,
                     temp.as<G1xyzz>(), (uint64_t)n, pref.as<Fp>(), s->points.as<G1Affine>(),
                     s->inf.as<uint8_t>());
  PLK_HIP_TRY(hipGetLastError());
  PLK_HIP_TRY(stream_wait(stream));
  return PLK_OK;
}

}  // namespace plk
