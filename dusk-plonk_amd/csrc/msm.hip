// msm.hip — G1 multi-scalar multiplication behind KZG commit on gfx950.
//
// Replaces msm_curve_addition inside zksnarks PlonkParams::commit (un-vendored; called at
// prover.rs:133-136,194,262-265,440,452 and key.rs:138-159).
//
// Design (fixed-base Pippenger, all windows folded into one bucket set):
//  * SRS load: table[w][i] = 2^(c*w) * P_i in affine form, w < W = ceil(256/c). The bases
//    of a commit are always an SRS prefix, so the table is built once per SRS and kept
//    resident in HBM (W * n * 96 B: 1.6 GB at n = 2^20, c = 16).
//  * Per MSM: each scalar is recoded into W signed c-bit digits |d| <= 2^(c-1); digit
//    (i, w) sends +-table[w][i] to bucket |d|-1, so there is ONE set of B = 2^(c-1)
//    buckets and no per-window doubling chain.
//  * Counting sort by bucket (atomic histogram -> scan -> atomic scatter). Order inside a
//    bucket is irrelevant: group addition is exact, the canonical affine output is unique.
//  * Bucket accumulation in chunks of CH points (one thread per chunk, XYZZ mixed adds):
//    the dominant kernel, integer-VALU bound; large buckets (skewed scalars) split evenly.
//  * Bucket reduction sum_b (b+1) S_b = sum_j 2^j T_j with T_j = sum of the buckets whose
//    weight has bit j set: two shallow tree kernels produce the c points T_j, and the CPU
//    runs the 2c-op Horner tail and the single inversion to canonical affine.
#include <hip/hip_runtime.h>

#include <vector>

#include "internal.hpp"
#include "msm_common.hpp"

namespace plk {

namespace {

// signed c-bit digit w of canonical scalar s (carry threaded through the caller)
__device__ __forceinline__ int digit_at(const Fr& s, uint32_t w, uint32_t c, uint32_t& carry) {
  const uint32_t o = w * c;
  uint32_t val = 0;
  if (o < 256) {
    const uint32_t wd = o >> 5, sh = o & 31;
    uint64_t two = s.v[wd];
    if (wd + 1 < 8) two |= (uint64_t)s.v[wd + 1] << 32;
    val = (uint32_t)(two >> sh) & ((1u << c) - 1u);
  }
  int d = (int)(val + carry);
  if (d > (int)(1u << (c - 1))) {
    d -= (int)(1u << c);
    carry = 1;
  } else {
    carry = 0;
  }
  return d;
}

__global__ void k_digits_count(const Fr* __restrict__ scalars, uint64_t len, MsmCfg cfg,
                               uint32_t* __restrict__ counts) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= len) return;
  const Fr s = fe_from_mont(ld_fr(&scalars[i]));
  uint32_t carry = 0;
  for (uint32_t w = 0; w < cfg.W; ++w) {
    const int d = digit_at(s, w, cfg.c, carry);
    if (d != 0) atomicAdd(&counts[(d < 0 ? -d : d) - 1], 1u);
  }
}

// single workgroup: offsets = exclusive scan(counts), task_off = exclusive scan(ceil(count/CH))
__global__ void __launch_bounds__(1024) k_scan_buckets(const uint32_t* __restrict__ counts, uint32_t B,
                                                       uint32_t* __restrict__ offsets,
                                                       uint32_t* __restrict__ task_off,
                                                       uint32_t* __restrict__ cursor) {
  __shared__ uint32_t s_cnt[1024], s_tsk[1024];
  const uint32_t tid = threadIdx.x, nt = blockDim.x;
  const uint32_t per = (B + nt - 1) / nt;
  const uint32_t b0 = tid * per;
  uint32_t c_sum = 0, t_sum = 0;
  for (uint32_t b = b0; b < b0 + per && b < B; ++b) {
    c_sum += counts[b];
    t_sum += (counts[b] + kChunk - 1) / kChunk;
  }
  s_cnt[tid] = c_sum;
  s_tsk[tid] = t_sum;
  __syncthreads();
  for (uint32_t off = 1; off < nt; off <<= 1) {
    uint32_t a = tid >= off ? s_cnt[tid - off] : 0, b = tid >= off ? s_tsk[tid - off] : 0;
    __syncthreads();
    s_cnt[tid] += a;
    s_tsk[tid] += b;
    __syncthreads();
  }
  uint32_t c_run = s_cnt[tid] - c_sum, t_run = s_tsk[tid] - t_sum;
  for (uint32_t b = b0; b < b0 + per && b < B; ++b) {
    offsets[b] = c_run;
    task_off[b] = t_run;
    cursor[b] = 0;
    c_run += counts[b];
    t_run += (counts[b] + kChunk - 1) / kChunk;
  }
  if (tid == nt - 1) {
    offsets[B] = s_cnt[tid];
    task_off[B] = s_tsk[tid];
  }
}

__global__ void k_digits_scatter(const Fr* __restrict__ scalars, uint64_t len, MsmCfg cfg,
                                 uint64_t n_srs, const uint32_t* __restrict__ offsets,
                                 uint32_t* __restrict__ cursor, uint32_t* __restrict__ sorted) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= len) return;
  const Fr s = fe_from_mont(ld_fr(&scalars[i]));
  uint32_t carry = 0;
  for (uint32_t w = 0; w < cfg.W; ++w) {
    const int d = digit_at(s, w, cfg.c, carry);
    if (d != 0) {
      const uint32_t b = (uint32_t)((d < 0 ? -d : d) - 1);
      const uint32_t pos = offsets[b] + atomicAdd(&cursor[b], 1u);
      sorted[pos] = (uint32_t)(w * n_srs + i) | (d < 0 ? 0x80000000u : 0u);
    }
  }
}

// task t of bucket b covers sorted[offsets[b] + t*CH, ...+CH)
__global__ void k_make_tasks(const uint32_t* __restrict__ offsets, const uint32_t* __restrict__ task_off,
                             uint32_t B, uint2* __restrict__ tasks) {
  const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const uint32_t start = offsets[b], cnt = offsets[b + 1] - start;
  uint32_t t = task_off[b];
  for (uint32_t o = 0; o < cnt; o += kChunk, ++t) {
    const uint32_t l = cnt - o < kChunk ? cnt - o : kChunk;
    tasks[t] = make_uint2(start + o, l);
  }
}

template <bool HAS_INF>
__global__ void __launch_bounds__(256) k_accumulate(const uint2* __restrict__ tasks,
                                                    const uint32_t* __restrict__ n_tasks,
                                                    const uint32_t* __restrict__ sorted,
                                                    const G1Affine* __restrict__ table,
                                                    const uint8_t* __restrict__ table_inf,
                                                    G1xyzz* __restrict__ partials) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= *n_tasks) return;
  const uint2 task = tasks[t];
  G1xyzz acc = xyzz_infinity();
  for (uint32_t e = task.x; e < task.x + task.y; ++e) {
    const uint32_t code = sorted[e];
    const uint32_t idx = code & 0x7fffffffu;
    if (HAS_INF && table_inf[idx]) continue;
    Fp x, y;
    ld_aff(&table[idx], x, y);
    if (code & 0x80000000u) y = fe_neg(y);
    acc = xyzz_add_affine(acc, x, y);
  }
  st_xyzz(&partials[t], acc);
}

__global__ void __launch_bounds__(128) k_bucket_reduce(const uint32_t* __restrict__ task_off, uint32_t B,
                                const G1xyzz* __restrict__ partials, G1xyzz* __restrict__ buckets) {
  const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  G1xyzz acc = xyzz_infinity();
  for (uint32_t t = task_off[b]; t < task_off[b + 1]; ++t) {
    G1xyzz q;
    ld_xyzz(&partials[t], q);
    acc = xyzz_add(acc, q);
  }
  st_xyzz(&buckets[b], acc);
}

// Workgroup g owns buckets [256g, 256g+256). Thread (j, s) sums the 16 buckets
// 256g + 16s + u whose weight (b+1) has bit j set; then a 16-way LDS tree per j.
// out[g * nbits + j]
__global__ void __launch_bounds__(256) k_bitsum1(const G1xyzz* __restrict__ buckets, uint32_t B,
                                                 uint32_t nbits, G1xyzz* __restrict__ out) {
  __shared__ G1xyzz sh[256];
  const uint32_t tid = threadIdx.x;
  const uint32_t j = tid >> 4, s = tid & 15;
  G1xyzz acc = xyzz_infinity();
  if (j < nbits) {
    for (uint32_t u = 0; u < 16; ++u) {
      const uint32_t b = blockIdx.x * 256 + s * 16 + u;
      if (b < B && (((b + 1) >> j) & 1u)) {
        G1xyzz q;
        ld_xyzz(&buckets[b], q);
        acc = xyzz_add(acc, q);
      }
    }
  }
  sh[tid] = acc;
  __syncthreads();
  for (uint32_t h = 8; h >= 1; h >>= 1) {
    if (s < h) sh[tid] = xyzz_add(sh[tid], sh[tid + h]);
    __syncthreads();
  }
  if (s == 0 && j < nbits) st_xyzz(&out[blockIdx.x * nbits + j], sh[tid]);
}

// Workgroup j sums in[g * nbits + j] over g < G.
__global__ void __launch_bounds__(256) k_bitsum2(const G1xyzz* __restrict__ in, uint32_t G,
                                                 uint32_t nbits, G1xyzz* __restrict__ out) {
  __shared__ G1xyzz sh[256];
  const uint32_t tid = threadIdx.x, j = blockIdx.x;
  G1xyzz acc = xyzz_infinity();
  for (uint32_t g = tid; g < G; g += 256) {
    G1xyzz q;
    ld_xyzz(&in[g * nbits + j], q);
    acc = xyzz_add(acc, q);
  }
  sh[tid] = acc;
  __syncthreads();
  for (uint32_t h = 128; h >= 1; h >>= 1) {
    if (tid < h) sh[tid] = xyzz_add(sh[tid], sh[tid + h]);
    __syncthreads();
  }
  if (tid == 0) st_xyzz(&out[j], sh[0]);
}

// flags[0] |= any nonzero scalar in [from, to)  (commit degree check)
__global__ void k_any_nonzero(const Fr* __restrict__ v, uint64_t from, uint64_t to,
                              uint32_t* __restrict__ flag) {
  const uint64_t i = from + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= to) return;
  if (!fe_is_zero(ld_fr(&v[i]))) atomicOr(flag, 1u);
}

}  // namespace

int ws_reserve(plk_srs* s, size_t len) {
  MsmWorkspace& w = *s->ws;
  if (len <= w.cap_len && w.cap_len) return PLK_OK;
  const size_t B = (size_t)1 << (s->c - 1);
  const size_t entries = (size_t)s->windows * len;
  const size_t max_tasks = entries / kChunk + B + 1;
  const size_t G = (B + 255) / 256;
  int st;
  if ((st = w.counts.alloc(B * 4))) return st;
  if ((st = w.offsets.alloc((B + 1) * 4))) return st;
  if ((st = w.task_off.alloc((B + 1) * 4))) return st;
  if ((st = w.cursor.alloc(B * 4))) return st;
  if ((st = w.sorted.alloc(entries * 4 + 4))) return st;
  if ((st = w.tasks.alloc(max_tasks * sizeof(uint2)))) return st;
  if ((st = w.partials.alloc(max_tasks * sizeof(G1xyzz)))) return st;
  if ((st = w.buckets.alloc(B * sizeof(G1xyzz)))) return st;
  if ((st = w.bits1.alloc(G * s->c * sizeof(G1xyzz)))) return st;
  if ((st = w.bits2.alloc(s->c * sizeof(G1xyzz)))) return st;
  if ((st = w.flag.alloc(16))) return st;
  if (!w.ev0) PLK_HIP_TRY(hipEventCreate(&w.ev0));
  if (!w.ev1) PLK_HIP_TRY(hipEventCreate(&w.ev1));
  w.cap_len = len;
  return PLK_OK;
}

int msm_run(plk_srs* s, const Fr* d_scalars, size_t len, size_t check_len, plk_g1* out,
            hipStream_t stream) {
  if (len > s->n) return PLK_E_ARG;
  int st;
  if ((st = ws_reserve(s, len ? len : 1))) return st;
  MsmWorkspace& w = *s->ws;
  const MsmCfg cfg{s->c, s->windows, 1u << (s->c - 1)};
  const uint32_t B = cfg.B;
  const uint32_t nbits = s->c;  // weights b+1 in [1, 2^(c-1)] need c bits
  const uint32_t G = cdiv(B, 256);

  PLK_HIP_TRY(hipMemsetAsync(w.flag.ptr, 0, 16, stream));
  if (check_len > len) {
    hipLaunchKernelGGL(k_any_nonzero, dim3(cdiv(check_len - len, 256)), dim3(256), 0, stream,
                       d_scalars, (uint64_t)len, (uint64_t)check_len, w.flag.as<uint32_t>());
  }
  PLK_HIP_TRY(hipMemsetAsync(w.counts.ptr, 0, B * 4, stream));
  if (len) {
    hipLaunchKernelGGL(k_digits_count, dim3(cdiv(len, 256)), dim3(256), 0, stream, d_scalars,
                       (uint64_t)len, cfg, w.counts.as<uint32_t>());
  }
  hipLaunchKernelGGL(k_scan_buckets, dim3(1), dim3(1024), 0, stream, w.counts.as<uint32_t>(), B,
                     w.offsets.as<uint32_t>(), w.task_off.as<uint32_t>(), w.cursor.as<uint32_t>());
  if (len) {
    hipLaunchKernelGGL(k_digits_scatter, dim3(cdiv(len, 256)), dim3(256), 0, stream, d_scalars,
                       (uint64_t)len, cfg, (uint64_t)s->n, w.offsets.as<uint32_t>(),
                       w.cursor.as<uint32_t>(), w.sorted.as<uint32_t>());
  }
  hipLaunchKernelGGL(k_make_tasks, dim3(cdiv(B, 256)), dim3(256), 0, stream, w.offsets.as<uint32_t>(),
                     w.task_off.as<uint32_t>(), B, w.tasks.as<uint2>());
  const size_t max_tasks = (size_t)s->windows * len / kChunk + B;
  PLK_HIP_TRY(hipEventRecord(w.ev0, stream));
  if (s->has_inf) {
    hipLaunchKernelGGL(k_accumulate<true>, dim3(cdiv(max_tasks, 256)), dim3(256), 0, stream,
                       w.tasks.as<uint2>(), w.task_off.as<uint32_t>() + B, w.sorted.as<uint32_t>(),
                       s->table.as<G1Affine>(), s->table_inf.as<uint8_t>(), w.partials.as<G1xyzz>());
  } else {
    hipLaunchKernelGGL(k_accumulate<false>, dim3(cdiv(max_tasks, 256)), dim3(256), 0, stream,
                       w.tasks.as<uint2>(), w.task_off.as<uint32_t>() + B, w.sorted.as<uint32_t>(),
                       s->table.as<G1Affine>(), s->table_inf.as<uint8_t>(), w.partials.as<G1xyzz>());
  }
  PLK_HIP_TRY(hipEventRecord(w.ev1, stream));
  hipLaunchKernelGGL(k_bucket_reduce, dim3(cdiv(B, 128)), dim3(128), 0, stream,
                     w.task_off.as<uint32_t>(), B, w.partials.as<G1xyzz>(), w.buckets.as<G1xyzz>());
  hipLaunchKernelGGL(k_bitsum1, dim3(G), dim3(256), 0, stream, w.buckets.as<G1xyzz>(), B, nbits,
                     w.bits1.as<G1xyzz>());
  hipLaunchKernelGGL(k_bitsum2, dim3(nbits), dim3(256), 0, stream, w.bits1.as<G1xyzz>(), G, nbits,
                     w.bits2.as<G1xyzz>());
  PLK_HIP_TRY(hipGetLastError());

  std::vector<G1xyzz> T(nbits);
  uint32_t flag = 0, entries = 0;
  PLK_HIP_TRY(hipMemcpyAsync(&entries, w.offsets.as<uint32_t>() + B, 4, hipMemcpyDeviceToHost,
                             stream));
  PLK_HIP_TRY(hipMemcpyAsync(T.data(), w.bits2.ptr, nbits * sizeof(G1xyzz), hipMemcpyDeviceToHost,
                             stream));
  PLK_HIP_TRY(hipMemcpyAsync(&flag, w.flag.ptr, 4, hipMemcpyDeviceToHost, stream));
  PLK_HIP_TRY(hipStreamSynchronize(stream));
  float ms = 0.f;
  if (hipEventElapsedTime(&ms, w.ev0, w.ev1) == hipSuccess) s->last_accumulate_ms = ms;
  s->last_point_adds = entries;  // nonzero digits = mixed adds in k_accumulate
  if (flag) return PLK_E_DEGREE;

  // host tail: sum_j 2^j T_j (Horner), then canonical affine
  G1xyzz acc = xyzz_infinity();
  for (int j = (int)nbits - 1; j >= 0; --j) {
    acc = xyzz_dbl(acc);
    acc = xyzz_add(acc, T[j]);
  }
  Fp x, y;
  const bool fin = xyzz_to_affine(acc, x, y);
  for (int i = 0; i < 6; ++i) {
    out->x[i] = (uint64_t)x.v[2 * i] | ((uint64_t)x.v[2 * i + 1] << 32);
    out->y[i] = (uint64_t)y.v[2 * i] | ((uint64_t)y.v[2 * i + 1] << 32);
  }
  out->infinity = fin ? 0 : 1;
  return PLK_OK;
}

}  // namespace plk

plk_srs::plk_srs() = default;
plk_srs::~plk_srs() = default;
