// msm.hip — G1 multi-scalar multiplication behind KZG commit on gfx950.
//
// Replaces msm_curve_addition inside zksnarks PlonkParams::commit (un-vendored; called at
// prover.rs:133-136,194,262-265,440,452 and key.rs:138-159).
//
// Design (fixed-base Pippenger, all windows folded into one bucket set):
//  * SRS load (srs.hip): table[w][i] = 2^(c*w) * P_i in affine form, w < W, resident in
//    HBM (W * n * 96 B: 1.6 GB at n = 2^20, c = 16, W = 16). Commit bases are always an
//    SRS prefix, so the table is built once.
//  * Per MSM: each scalar s is first brought to [0, (r-1)/2] (s or r - s with the signs
//    flipped, scalar_half), then recoded into W = ceil(255/c) signed c-bit digits
//    |d| <= 2^(c-1); digit (i, w) sends +-table[w][i] to bucket |d|-1: ONE set of
//    B = 2^(c-1) buckets and no per-window doubling chain.
//  * Counting sort by bucket: per-workgroup LDS histograms (windows of 32 K buckets =
//    128 KiB; c = 17 takes two) written whole, a per-bucket scan over the workgroups
//    (k_block_scan) instead of global atomics, then LDS atomics place each digit. Order
//    inside a bucket is irrelevant: group addition is exact and the canonical affine
//    output is unique.
//  * Bucket accumulation in chunks of CH points (one thread per chunk, XYZZ mixed adds):
//    the dominant kernel, integer-VALU bound.
//  * Bucket reduction sum_b (b+1) S_b = sum_j 2^j T_j (T_j: sums of buckets selected by the
//    bits of their weight, see k_bitsum1): two shallow tree kernels give the c points T_j and
//    the CPU runs the 2c-op Horner tail and the single inversion to canonical affine.
//  * Up to kMaxSlots independent MSMs run as ONE batch (blockIdx.y = slot): the prover's
//    commits come in independent groups (4 wires, 4 quotient chunks, 2 openings), and the
//    latency-bound tail kernels of a batch then cost about what one MSM's tail costs.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "internal.hpp"
#include "msm_common.hpp"
#include "g1r.hpp"

namespace plk {

namespace {

#ifndef PLK_LANE_PARTIALS
#define PLK_LANE_PARTIALS 4  // bucket partials per k_bucket_sum lane aimed at (only c <= 15, SRS < 2^16: 8 -> 4 gave 2^12 3.74 -> 3.93 M constraints/s, tools/gpu_ab_quick.sh)
#endif
#ifndef PLK_CHUNK_TARGET
#define PLK_CHUNK_TARGET 262144  // accumulation tasks aimed at per batch (chunk = entries / this)
#endif
constexpr uint32_t kHistThreads = 1024;
constexpr uint32_t kHistBlocksMax = 256;  // histogram / scatter workgroups per slot

// signed digit w of canonical scalar s (carry threaded through the caller): windows
// 0 .. W - narrow - 1 take c bits, the top `narrow` ones c - 1 bits (plk_srs::narrow), their
// digits (|d| <= 2^(c-2)) scaled by 2 so that they span the bucket range too
__device__ __forceinline__ int digit_at(const Fr& s, uint32_t w, const MsmCfg& cfg, uint32_t& carry) {
  const uint32_t wn = cfg.W - cfg.narrow;  // first narrow window
  const bool nar = w >= wn;
  const uint32_t c = cfg.c - (nar ? 1u : 0u);
  const uint32_t o = nar ? wn * cfg.c + (w - wn) * c : w * cfg.c;
  uint32_t val = 0;
  if (o < 256) {
    // words wd, wd + 1 by a 3-level select tree: indexing s.v with a run-time wd put the
    // scalar in scratch memory (k_sort_one: 272 B per lane, k_hist / k_scatter: 48)
    const uint32_t wd = o >> 5, sh = o & 31;
    const bool b0 = wd & 1, b1 = wd & 2, b2 = wd & 4;
    uint64_t p[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {  // pair (2k + b0, 2k + b0 + 1)
      const uint32_t lo = b0 ? s.v[2 * k + 1] : s.v[2 * k];
      const uint32_t hi = b0 ? (k < 3 ? s.v[2 * k + 2] : 0u) : s.v[2 * k + 1];
      p[k] = ((uint64_t)hi << 32) | lo;
    }
    const uint64_t q0 = b1 ? p[1] : p[0], q1 = b1 ? p[3] : p[2];
    const uint64_t two = b2 ? q1 : q0;
    val = (uint32_t)(two >> sh) & ((1u << c) - 1u);
  }
  int d = (int)(val + carry);
  if (d > (int)(1u << (c - 1))) {
    d -= (int)(1u << c);
    carry = 1;
  } else {
    carry = 0;
  }
  return nar ? d * 2 : d;
}

// Every digit of s, f(w, d) for w = 0 .. W-1 in order. C = 0: digit_at with the run-time
// window layout. C = the SRS's c (10, 12, 13, 15, 17, 20 — the window sizes choose_c picks): the
// layout is a compile-time constant, the loop unrolls and each digit is a funnel shift
// (v_alignbit_b32) of two known words, a mask and the carry test — ~6 instructions instead
// of digit_at's ~25 (word select tree, 64-bit shift). The sort kernels extract every digit of
// every scalar twice (histogram and scatter); k_sort_one does it for a whole commit on one
// workgroup.
template <uint32_t C, class F>
__device__ __forceinline__ void each_digit(const Fr& s, const MsmCfg& cfg, F&& f) {
  if constexpr (C == 0) {
    uint32_t carry = 0;
    for (uint32_t w = 0; w < cfg.W; ++w) f(w, digit_at(s, w, cfg, carry));
  } else {
    constexpr uint32_t W = (255 + C - 1) / C, NAR = C * W - 255, WN = W - NAR;
    static_assert(NAR < W, "balanced windows need (C - 1) W <= 255");
    uint32_t carry = 0;
#pragma unroll
    for (uint32_t w = 0; w < W; ++w) {
      const bool nar = w >= WN;
      const uint32_t cw = nar ? C - 1 : C;
      const uint32_t o = nar ? WN * C + (w - WN) * (C - 1) : w * C;
      const uint32_t wd = o >> 5, sh = o & 31;
      uint32_t val = sh == 0 ? s.v[wd]
                             : __builtin_amdgcn_alignbit(wd + 1 < 8 ? s.v[wd + 1 < 8 ? wd + 1 : 7] : 0u,
                                                         s.v[wd], sh);
      val &= (1u << cw) - 1u;
      int d = (int)(val + carry);
      if (d > (int)(1u << (cw - 1))) {
        d -= (int)(1u << cw);
        carry = 1;
      } else {
        carry = 0;
      }
      f(w, nar ? d * 2 : d);
    }
  }
}

__device__ __forceinline__ void slot_range(uint32_t len, uint32_t& i0, uint32_t& i1) {
  const uint32_t per = (len + gridDim.x - 1) / gridDim.x;
  i0 = blockIdx.x * per;
  i1 = min(len, i0 + per);
}

// Canonical scalar in [0, (r-1)/2]: s, or r - s with the digit signs flipped (s P = (r - s)(-P)).
// With s < 2^254 the signed c-bit recoding needs W = ceil(255 / c) windows (c = 17: 15).
__device__ __forceinline__ Fr scalar_half_v(const Fr& raw, bool& neg) {
  const Fr s = fe_from_mont(raw);
  const Fr t = fe_neg(s);
  bool lt = false;  // t < s
#pragma unroll
  for (int k = 7; k >= 0; --k) {
    if (t.v[k] != s.v[k]) {
      lt = t.v[k] < s.v[k];
      break;
    }
  }
  neg = lt;
  return lt ? t : s;
}
__device__ __forceinline__ Fr scalar_half(const Fr* p, bool& neg) { return scalar_half_v(ld_fr(p), neg); }

// f(i, canonical half of scalar i, its sign flip) for i = i0 + t, i0 + t + step, ... < i1 in
// order, with kScalarLoads scalars loaded before the first is processed: the sort passes are
// bound by load latency (one scalar in flight per thread before), not by bytes
constexpr uint32_t kScalarLoads = 4;
template <class F>
__device__ __forceinline__ void for_scalars(const Fr* __restrict__ sc, uint32_t i0, uint32_t i1,
                                            uint32_t t, uint32_t step, F&& f) {
  uint32_t i = i0 + t;
  for (; i + (kScalarLoads - 1) * step < i1; i += kScalarLoads * step) {
    Fr raw[kScalarLoads];
#pragma unroll
    for (uint32_t u = 0; u < kScalarLoads; ++u) raw[u] = ld_fr(&sc[i + u * step]);
#pragma unroll
    for (uint32_t u = 0; u < kScalarLoads; ++u) {
      bool neg;
      const Fr s = scalar_half_v(raw[u], neg);
      f(i + u * step, s, neg);
    }
  }
  for (; i < i1; i += step) {
    bool neg;
    const Fr s = scalar_half_v(ld_fr(&sc[i]), neg);
    f(i, s, neg);
  }
}

// LDS histograms cover at most kLdsBuckets buckets (128 KiB); larger bucket sets (c = 17)
// are processed in bucket windows, each a fresh pass over the workgroup's scalars.
constexpr uint32_t kLdsBuckets = 32768;

// Pass 1: LDS histogram of this workgroup's digits, written whole to
// blockhist[slot][blk][b] (no global atomics).
template <uint32_t C>
__global__ void __launch_bounds__(kHistThreads) k_hist(MsmBatch batch, MsmCfg cfg,
                                                       uint32_t* __restrict__ blockhist) {
  extern __shared__ __attribute__((aligned(16))) uint32_t hist[];
  const uint32_t slot = blockIdx.y, B = cfg.B;
  uint32_t i0, i1;
  slot_range(batch.len[slot], i0, i1);
  const Fr* sc = batch.scalars[slot];
  uint32_t* out = blockhist + ((size_t)slot * gridDim.x + blockIdx.x) * B;
  for (uint32_t b0 = 0; b0 < B; b0 += kLdsBuckets) {
    const uint32_t nb = min(kLdsBuckets, B - b0);
    for (uint32_t b = threadIdx.x; b < nb; b += blockDim.x) hist[b] = 0;
    __syncthreads();
    for_scalars(sc, i0, i1, threadIdx.x, blockDim.x, [&](uint32_t, const Fr& s, bool) {
      each_digit<C>(s, cfg, [&](uint32_t, int d) {
        const uint32_t b = (uint32_t)(d < 0 ? -d : d) - 1u - b0;  // wraps for d == 0
        if (d != 0 && b < nb) atomicAdd(&hist[b], 1u);
      });
    });
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < nb; b += blockDim.x) out[b0 + b] = hist[b];
    __syncthreads();
  }
}

// Per bucket, over the histogram workgroups: blockhist becomes the exclusive running count
// (each workgroup's first position inside the bucket) and counts[b] the bucket total.
// Workgroup (0, slot) also clears the slot's kChunkMax-word counters zero_a / zero_b when
// given (the wide path's tail-length counters, used by k_fine and k_make_tasks_wide) — two
// memset dispatches fewer per batch.
__global__ void k_block_scan(uint32_t* __restrict__ blockhist, uint32_t nblk, uint32_t B,
                             uint32_t* __restrict__ counts, uint32_t* __restrict__ zero_a,
                             uint32_t* __restrict__ zero_b) {
  const uint32_t slot = blockIdx.y;
  if (blockIdx.x == 0 && zero_a) {  // a loop: kChunkMax (PLK_CHUNK_MAX) may exceed the block
    for (uint32_t l = threadIdx.x; l < (uint32_t)kChunkMax; l += blockDim.x) {
      zero_a[(size_t)slot * kChunkMax + l] = 0;
      zero_b[(size_t)slot * kChunkMax + l] = 0;
    }
  }
  const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  uint32_t* h = blockhist + (size_t)slot * nblk * B + b;
  uint32_t run = 0, k = 0;
  for (; k + 8 <= nblk; k += 8) {  // 8 loads in flight before the stores
    uint32_t v[8];
#pragma unroll
    for (uint32_t u = 0; u < 8; ++u) v[u] = h[(size_t)(k + u) * B];
#pragma unroll
    for (uint32_t u = 0; u < 8; ++u) {
      h[(size_t)(k + u) * B] = run;
      run += v[u];
    }
  }
  for (; k < nblk; ++k) {
    const uint32_t v = h[(size_t)k * B];
    h[(size_t)k * B] = run;
    run += v;
  }
  counts[(size_t)slot * B + b] = run;
}

// single workgroup per slot: offsets = exclusive scan(counts),
// task_off = exclusive scan(ceil(count / CH)) (where each bucket's partial sums go), and the
// EXECUTION order of the tasks: all full tasks (CH entries) first in bucket order, then the
// partial tails grouped by length, longest first, so that a wavefront's lanes run tasks of
// (nearly) the same length. len_cur[slot][l] = first execution slot of the tails of length l.
// The counts are staged in LDS first (dynamic, B words; one coalesced pass): the two walks
// over each thread's contiguous buckets then read LDS instead of issuing one dependent
// global load per bucket.
__global__ void __launch_bounds__(1024) k_scan_buckets(const uint32_t* __restrict__ counts_g,
                                                       uint32_t B, uint32_t chunk,
                                                       uint32_t* __restrict__ offsets,
                                                       uint32_t* __restrict__ task_off,
                                                       uint32_t* __restrict__ full_off,
                                                       uint32_t* __restrict__ len_cur) {
  __shared__ uint32_t s_cnt[1024], s_tsk[1024], s_full[1024], s_len[kChunkMax];
  extern __shared__ __attribute__((aligned(16))) uint32_t counts[];
  const uint32_t slot = blockIdx.y;
  counts_g += (size_t)slot * B;
  for (uint32_t b = threadIdx.x; b < B; b += blockDim.x) counts[b] = counts_g[b];
  offsets += (size_t)slot * (B + 1);
  task_off += (size_t)slot * (B + 1);
  full_off += (size_t)slot * B;
  len_cur += (size_t)slot * kChunkMax;
  const uint32_t tid = threadIdx.x, nt = blockDim.x;
  if (tid < kChunkMax) s_len[tid] = 0;
  __syncthreads();
  const uint32_t per = (B + nt - 1) / nt;
  const uint32_t b0 = tid * per;
  uint32_t c_sum = 0, t_sum = 0, f_sum = 0;
  for (uint32_t b = b0; b < b0 + per && b < B; ++b) {
    const uint32_t c = counts[b];
    c_sum += c;
    t_sum += (c + chunk - 1) / chunk;
    f_sum += c / chunk;
    if (c % chunk) atomicAdd(&s_len[c % chunk], 1u);
  }
  s_cnt[tid] = c_sum;
  s_tsk[tid] = t_sum;
  s_full[tid] = f_sum;
  __syncthreads();
  for (uint32_t off = 1; off < nt; off <<= 1) {
    uint32_t a = tid >= off ? s_cnt[tid - off] : 0, b = tid >= off ? s_tsk[tid - off] : 0;
    uint32_t f = tid >= off ? s_full[tid - off] : 0;
    __syncthreads();
    s_cnt[tid] += a;
    s_tsk[tid] += b;
    s_full[tid] += f;
    __syncthreads();
  }
  uint32_t c_run = s_cnt[tid] - c_sum, t_run = s_tsk[tid] - t_sum, f_run = s_full[tid] - f_sum;
  for (uint32_t b = b0; b < b0 + per && b < B; ++b) {
    offsets[b] = c_run;
    task_off[b] = t_run;
    full_off[b] = f_run;
    c_run += counts[b];
    t_run += (counts[b] + chunk - 1) / chunk;
    f_run += counts[b] / chunk;
  }
  if (tid == nt - 1) {
    offsets[B] = s_cnt[tid];
    task_off[B] = s_tsk[tid];
  }
  if (tid == 0) {  // tails after the full tasks, longest first
    uint32_t run = s_full[nt - 1];
    for (uint32_t l = chunk - 1; l >= 1; --l) {
      len_cur[l] = run;
      run += s_len[l];
    }
  }
}

// Pass 2: this workgroup's positions start at offsets[b] + blockhist[slot][blk][b]; each
// digit takes the next one with an LDS atomic (bucket windows as in k_hist).
template <uint32_t C>
__global__ void __launch_bounds__(kHistThreads) k_scatter(MsmBatch batch, MsmCfg cfg,
                                                          uint64_t n_srs,
                                                          const uint32_t* __restrict__ offsets,
                                                          const uint32_t* __restrict__ blockhist,
                                                          uint32_t* __restrict__ sorted,
                                                          uint64_t sorted_stride) {
  extern __shared__ __attribute__((aligned(16))) uint32_t hist[];
  const uint32_t slot = blockIdx.y, B = cfg.B;
  const uint32_t* off = offsets + (size_t)slot * (B + 1);
  const uint32_t* bh = blockhist + ((size_t)slot * gridDim.x + blockIdx.x) * B;
  uint32_t i0, i1;
  slot_range(batch.len[slot], i0, i1);
  const Fr* sc = batch.scalars[slot];
  uint32_t* out = sorted + (size_t)slot * sorted_stride;
  for (uint32_t b0 = 0; b0 < B; b0 += kLdsBuckets) {
    const uint32_t nb = min(kLdsBuckets, B - b0);
    for (uint32_t b = threadIdx.x; b < nb; b += blockDim.x) hist[b] = off[b0 + b] + bh[b0 + b];
    __syncthreads();
    for_scalars(sc, i0, i1, threadIdx.x, blockDim.x, [&](uint32_t i, const Fr& s, bool neg) {
      each_digit<C>(s, cfg, [&](uint32_t w, int d) {
        const uint32_t b = (uint32_t)(d < 0 ? -d : d) - 1u - b0;
        if (d != 0 && b < nb) {
          const uint32_t pos = atomicAdd(&hist[b], 1u);
          out[pos] = (uint32_t)(w * n_srs + i) | (((d < 0) != neg) ? 0x80000000u : 0u);
        }
      });
    });
    __syncthreads();
  }
}

// Task t of bucket b covers sorted[offsets[b] + t*CH, ...+CH) and writes its partial sum to
// partials[task_off[b] + t]; its execution slot is full_off[b] + t for a full task, or the
// next slot of its length class for the tail. tasks[slot] = {first entry, partial index |
// (length - 1) << kTaskShift}.
__global__ void k_make_tasks(const uint32_t* __restrict__ offsets,
                             const uint32_t* __restrict__ task_off,
                             const uint32_t* __restrict__ full_off, uint32_t* __restrict__ len_cur,
                             uint32_t B, uint32_t chunk, uint2* __restrict__ tasks,
                             uint64_t task_stride) {
  // tails: ranks inside the workgroup from LDS atomics, one global atomic per (workgroup,
  // length) for the base
  __shared__ uint32_t s_cnt[kChunkMax], s_base[kChunkMax];
  const uint32_t slot = blockIdx.y, tid = threadIdx.x;
  const uint32_t b = blockIdx.x * blockDim.x + tid;
  for (uint32_t l = tid; l < kChunkMax; l += blockDim.x) s_cnt[l] = 0;
  __syncthreads();
  offsets += (size_t)slot * (B + 1);
  task_off += (size_t)slot * (B + 1);
  tasks += (size_t)slot * task_stride;
  uint32_t start = 0, t0 = 0, nfull = 0, tail = 0, rank = 0;
  if (b < B) {
    start = offsets[b];
    const uint32_t cnt = offsets[b + 1] - start;
    t0 = task_off[b];
    nfull = cnt / chunk;
    tail = cnt - nfull * chunk;
    if (tail) rank = atomicAdd(&s_cnt[tail], 1u);
  }
  __syncthreads();
  for (uint32_t l = tid; l < kChunkMax; l += blockDim.x)
    if (s_cnt[l]) s_base[l] = atomicAdd(&len_cur[(size_t)slot * kChunkMax + l], s_cnt[l]);
  __syncthreads();
  if (b >= B) return;
  uint32_t x = full_off[(size_t)slot * B + b];
  for (uint32_t t = 0; t < nfull; ++t, ++x)
    tasks[x] = make_uint2(start + t * chunk, (t0 + t) | ((chunk - 1) << kTaskShift));
  if (tail)
    tasks[s_base[tail] + rank] =
        make_uint2(start + nfull * chunk, (t0 + nfull) | ((tail - 1) << kTaskShift));
}

// Small bucket sets (B <= kSortSmallMax: the 2^12-size commits, c <= 13) in ONE dispatch per
// batch instead of three: k_block_scan + k_scan_buckets + k_make_tasks on one workgroup per
// slot (the bucket counts and the tail-length cursors in LDS, so the tail ranks need no global
// atomics). Small proofs are bound by the rate at which the command processor takes
// dispatches, not by these kernels' work. The task layout is k_make_tasks' (full
// tasks in bucket order, then the tails grouped by length, longest first).
constexpr uint32_t kSortSmallMax = 4096;
__global__ void __launch_bounds__(1024) k_sort_small(uint32_t* __restrict__ blockhist, uint32_t nblk,
                                                     uint32_t B, uint32_t chunk,
                                                     uint32_t* __restrict__ offsets,
                                                     uint32_t* __restrict__ task_off,
                                                     uint2* __restrict__ tasks, uint64_t task_stride) {
  __shared__ uint32_t s_count[kSortSmallMax];
  __shared__ uint32_t s_c[1024], s_t[1024], s_f[1024], s_len[kChunkMax], s_cur[kChunkMax];
  const uint32_t slot = blockIdx.y, tid = threadIdx.x, nt = blockDim.x;
  blockhist += (size_t)slot * nblk * B;
  offsets += (size_t)slot * (B + 1);
  task_off += (size_t)slot * (B + 1);
  tasks += (size_t)slot * task_stride;
  if (tid < kChunkMax) s_len[tid] = 0;
  // per bucket, over the histogram workgroups: exclusive running counts (k_block_scan)
  for (uint32_t b = tid; b < B; b += nt) {
    uint32_t* h = blockhist + b;
    uint32_t run = 0, k = 0;
    for (; k + 8 <= nblk; k += 8) {
      uint32_t v[8];
#pragma unroll
      for (uint32_t u = 0; u < 8; ++u) v[u] = h[(size_t)(k + u) * B];
#pragma unroll
      for (uint32_t u = 0; u < 8; ++u) {
        h[(size_t)(k + u) * B] = run;
        run += v[u];
      }
    }
    for (; k < nblk; ++k) {
      const uint32_t v = h[(size_t)k * B];
      h[(size_t)k * B] = run;
      run += v;
    }
    s_count[b] = run;
  }
  __syncthreads();
  // offsets / task offsets / full-task offsets over each thread's contiguous buckets
  // (k_scan_buckets)
  const uint32_t per = (B + nt - 1) / nt;
  const uint32_t b0 = min(tid * per, B), b1 = min(b0 + per, B);
  uint32_t c_sum = 0, t_sum = 0, f_sum = 0;
  for (uint32_t b = b0; b < b1; ++b) {
    const uint32_t c = s_count[b];
    c_sum += c;
    t_sum += (c + chunk - 1) / chunk;
    f_sum += c / chunk;
    if (c % chunk) atomicAdd(&s_len[c % chunk], 1u);
  }
  s_c[tid] = c_sum;
  s_t[tid] = t_sum;
  s_f[tid] = f_sum;
  __syncthreads();
  for (uint32_t off = 1; off < nt; off <<= 1) {
    const uint32_t a = tid >= off ? s_c[tid - off] : 0, t = tid >= off ? s_t[tid - off] : 0;
    const uint32_t f = tid >= off ? s_f[tid - off] : 0;
    __syncthreads();
    s_c[tid] += a;
    s_t[tid] += t;
    s_f[tid] += f;
    __syncthreads();
  }
  if (tid == 0) {  // tails after the full tasks, longest first
    uint32_t run = s_f[nt - 1];
    for (uint32_t l = chunk - 1; l >= 1; --l) {
      s_cur[l] = run;
      run += s_len[l];
    }
    offsets[B] = s_c[nt - 1];
    task_off[B] = s_t[nt - 1];
  }
  __syncthreads();
  // the task records (k_make_tasks), tail ranks from LDS cursors
  uint32_t c_run = s_c[tid] - c_sum, t_run = s_t[tid] - t_sum, f_run = s_f[tid] - f_sum;
  for (uint32_t b = b0; b < b1; ++b) {
    const uint32_t cnt = s_count[b];
    offsets[b] = c_run;
    task_off[b] = t_run;
    const uint32_t nfull = cnt / chunk, tail = cnt - nfull * chunk;
    for (uint32_t t = 0; t < nfull; ++t)
      tasks[f_run + t] = make_uint2(c_run + t * chunk, (t_run + t) | ((chunk - 1) << kTaskShift));
    if (tail)
      tasks[atomicAdd(&s_cur[tail], 1u)] =
          make_uint2(c_run + nfull * chunk, (t_run + nfull) | ((tail - 1) << kTaskShift));
    c_run += cnt;
    t_run += (cnt + chunk - 1) / chunk;
    f_run += nfull;
  }
}

// Small batches (B <= kSortSmallMax and at most kSortOneMax scalars per slot: the 2^12-size
// proofs' commits) sorted in ONE dispatch (round 4: one workgroup per slot; round 5: a few,
// split by bucket range, below) instead of three (k_hist,
// k_sort_small, k_scatter) or four (with k_any_nonzero): the commit degree check, an LDS
// histogram over all of the slot's digits, the scans and task records of k_sort_small, then
// the scatter with LDS cursors. Small proofs are bound by the command processor's dispatch
// rate, so the dispatches matter more than the single workgroup's latency. The
// order of the entries inside a bucket differs from the multi-workgroup sort; the bucket's
// sum (exact XYZZ arithmetic, canonical affine result) does not.
// Measured (profiles/r04_sortone_runsum_shoup_ab.jsonl, one box, interleaved): 2^12 proofs
// 7.48 / 7.84 against 7.05 / 7.45 M constraints/s with the multi-dispatch sort.
// Round 4 also measured the 2^14-size proofs' commits (c = 15: 2^14 buckets, ~2^14 scalars
// per slot) through one workgroup re-reading the scalars for the scatter: no faster
// (profiles/r04_sort_one_big_ab.jsonl; removed in round 5).
constexpr uint32_t kSortOneMax = 8192;  // scalars per slot held in registers
// workgroups per slot, each taking 1/kSortOneParts of the buckets (round 5, three interleaved
// runs against one workgroup, profiles/r05_sort_one_parts_ab.jsonl: lone 2^12 MSM 0.394 ->
// 0.347 ms, 2^12 proofs 8.81 -> 9.10 M, 2^13 within noise; 8 workgroups the same as 4)
constexpr uint32_t kSortOneParts = 4;
// HOLD: the slot's scalars (<= kSortOneMax) stay in registers between the histogram and the
// scatter; otherwise (<= kSortOneBig, the 2^14-size commits at c = 13) both passes read them
// from memory, 4 ahead per thread (for_scalars)
constexpr uint32_t kSortOneBig = 32768;
template <uint32_t C, bool HOLD>
__global__ void __launch_bounds__(1024) k_sort_one(MsmBatch batch, MsmCfg cfg, uint64_t n_srs,
                                                   uint32_t chunk, uint32_t* __restrict__ sorted,
                                                   uint64_t sorted_stride,
                                                   uint32_t* __restrict__ offsets,
                                                   uint32_t* __restrict__ task_off,
                                                   uint2* __restrict__ tasks, uint64_t task_stride,
                                                   uint32_t* __restrict__ flag, uint32_t gen) {
  // Workgroup x of the slot's gridDim.x owns buckets [bl, bh): every workgroup histograms ALL
  // the slot's digits (LDS atomics; the offsets of its range follow from the counts below it,
  // so no workgroup waits for another), then writes the task records and scatters the
  // entries of its own range only — the scattered 4-byte stores, which one CU's memory path
  // took most of the kernel's time for, spread over gridDim.x CUs.
  __shared__ uint32_t s_count[kSortSmallMax];
  __shared__ uint32_t s_c[1024], s_t[1024], s_f[1024], s_len[kChunkMax], s_cur[kChunkMax],
      s_pre[kChunkMax];
  const uint32_t slot = blockIdx.y, tid = threadIdx.x, nt = 1024, B = cfg.B;  // blockDim.x
  const uint32_t bpart = B / gridDim.x;  // B and gridDim.x powers of two, B >= gridDim.x
  const uint32_t bl = blockIdx.x * bpart, bh = bl + bpart;
  const uint32_t len = batch.len[slot];
  const Fr* sc = batch.scalars[slot];
  offsets += (size_t)slot * (B + 1);
  task_off += (size_t)slot * (B + 1);
  tasks += (size_t)slot * task_stride;
  uint32_t* out = sorted + (size_t)slot * sorted_stride;
  // the commit's degree check (k_any_nonzero): a nonzero scalar in [len, check_len)
  if (blockIdx.x == 0)
    for (uint64_t i = (uint64_t)len + tid; i < batch.check_len[slot]; i += nt)
      if (!fe_is_zero(ld_fr(&sc[i]))) flag[slot] = gen;  // every writer stores the same value
  for (uint32_t b = tid; b < B; b += nt) s_count[b] = 0;
  for (uint32_t l = tid; l < kChunkMax; l += nt) s_len[l] = s_pre[l] = 0;
  __syncthreads();
  // HOLD: this thread's scalars (i = tid + k nt, at most kSortOneMax / 1024 of them), brought
  // to [0, (r-1)/2] once and kept in registers for both passes
  constexpr uint32_t kPer = HOLD ? kSortOneMax / 1024 : 1;
  Fr sv[kPer];
  bool sneg[kPer];
  auto hist_digits = [&](const Fr& x) {
    each_digit<C>(x, cfg, [&](uint32_t, int d) {
      if (d != 0) atomicAdd(&s_count[(uint32_t)(d < 0 ? -d : d) - 1u], 1u);
    });
  };
  if constexpr (HOLD) {
#pragma unroll
    for (uint32_t k = 0; k < kPer; ++k) {
      const uint32_t i = tid + k * nt;
      sneg[k] = false;
      if (i < len) sv[k] = scalar_half(&sc[i], sneg[k]);
    }
#pragma unroll
    for (uint32_t k = 0; k < kPer; ++k) {  // histogram of every digit of the slot
      if (tid + k * nt >= len) break;
      hist_digits(sv[k]);
    }
  } else {
    for_scalars(sc, 0, len, tid, nt, [&](uint32_t, const Fr& x, bool) { hist_digits(x); });
  }
  __syncthreads();
  // offsets / task offsets / full-task offsets over each thread's contiguous buckets (all B:
  // every workgroup derives the same global layout), the tail-length counts over all buckets
  // and over the buckets below this workgroup's range (its tail ranks start after those)
  const uint32_t per = (B + nt - 1) / nt;
  const uint32_t b0 = min(tid * per, B), b1 = min(b0 + per, B);
  uint32_t c_sum = 0, t_sum = 0, f_sum = 0;
  for (uint32_t b = b0; b < b1; ++b) {
    const uint32_t c = s_count[b];
    c_sum += c;
    t_sum += (c + chunk - 1) / chunk;
    f_sum += c / chunk;
    if (c % chunk) {
      atomicAdd(&s_len[c % chunk], 1u);
      if (b < bl) atomicAdd(&s_pre[c % chunk], 1u);
    }
  }
  s_c[tid] = c_sum;
  s_t[tid] = t_sum;
  s_f[tid] = f_sum;
  __syncthreads();
  for (uint32_t off = 1; off < nt; off <<= 1) {
    const uint32_t a = tid >= off ? s_c[tid - off] : 0, t = tid >= off ? s_t[tid - off] : 0;
    const uint32_t f = tid >= off ? s_f[tid - off] : 0;
    __syncthreads();
    s_c[tid] += a;
    s_t[tid] += t;
    s_f[tid] += f;
    __syncthreads();
  }
  if (tid == 0) {  // tails after the full tasks, longest first; this range's after those below
    uint32_t run = s_f[nt - 1];
    for (uint32_t l = chunk - 1; l >= 1; --l) {
      s_cur[l] = run + s_pre[l];
      run += s_len[l];
    }
    if (blockIdx.x == 0) {
      offsets[B] = s_c[nt - 1];
      task_off[B] = s_t[nt - 1];
    }
  }
  __syncthreads();
  uint32_t c_run = s_c[tid] - c_sum, t_run = s_t[tid] - t_sum, f_run = s_f[tid] - f_sum;
  for (uint32_t b = b0; b < b1; ++b) {
    const uint32_t cnt = s_count[b];
    if (b >= bl && b < bh) {
      s_count[b] = c_run;
      offsets[b] = c_run;
      task_off[b] = t_run;
      const uint32_t nfull = cnt / chunk, tail = cnt - nfull * chunk;
      for (uint32_t t = 0; t < nfull; ++t)
        tasks[f_run + t] = make_uint2(c_run + t * chunk, (t_run + t) | ((chunk - 1) << kTaskShift));
      if (tail)
        tasks[atomicAdd(&s_cur[tail], 1u)] =
            make_uint2(c_run + nfull * chunk, (t_run + nfull) | ((tail - 1) << kTaskShift));
    }
    c_run += cnt;
    t_run += (cnt + chunk - 1) / chunk;
    f_run += cnt / chunk;
  }
  __syncthreads();
  auto scatter_digits = [&](const Fr& x, bool neg, uint32_t i) {
    each_digit<C>(x, cfg, [&](uint32_t w, int d) {
      const uint32_t b = (uint32_t)(d < 0 ? -d : d) - 1u;  // d = 0: wraps past bh
      if (b - bl < bpart) {
        const uint32_t pos = atomicAdd(&s_count[b], 1u);
        out[pos] = (uint32_t)(w * n_srs + i) | (((d < 0) != neg) ? 0x80000000u : 0u);
      }
    });
  };
  if constexpr (HOLD) {
#pragma unroll
    for (uint32_t k = 0; k < kPer; ++k) {  // scatter (k_scatter) of this workgroup's buckets
      const uint32_t i = tid + k * nt;
      if (i >= len) break;
      scatter_digits(sv[k], sneg[k], i);
    }
  } else {
    for_scalars(sc, 0, len, tid, nt,
                [&](uint32_t i, const Fr& x, bool neg) { scatter_digits(x, neg, i); });
  }
}

// ---- wide bucket sets (B > kLdsBuckets, c >= 17): two-level radix sort ----------------
// One LDS histogram cannot hold the buckets, and per-(workgroup, bucket) runs of ~1 entry
// make a direct scatter write-amplified. Instead: (1) coarse bins of kFine consecutive
// buckets — per-workgroup LDS histograms, a per-bin scan over the workgroups and a scatter
// of (code, bucket) pairs into bin order (runs of ~100 entries per (workgroup, bin));
// (2) one workgroup per bin counting-sorts its entries by bucket inside the bin's own
// region (LDS counters, writes that stay in one L2), emitting the bucket offsets and the
// per-bucket task counts on the way; (3) the task records, as k_make_tasks does.
constexpr uint32_t kFineBits = 10;  // 2^10 buckets per coarse bin = threads of k_fine
// A bucket-range part (parts > 1) of 2^(c-1) / parts buckets keeps >= 256 coarse bins (k_fine
// / k_make_tasks_wide workgroups) with bins of 2^FB buckets, FB = max(8, 10 - log2 parts)
constexpr uint32_t kFineBitsMin = 8;
constexpr uint32_t kCoarseMax = 4096;        // coarse bins (B <= 2^22, c <= 23)
// bucket reduction: runs of K = 2^rb buckets per lane. Batches of several MSMs (the
// prover's commit groups, with other proofs' kernels beside them) take 16. A lone MSM's
// run-sum chains are latency-bound with the chip otherwise idle, so its rb is the largest
// rb <= kRunBits that still gives kRunLanes run lanes: K = 8 at 2^20, 2 at 2^16 (lone
// 2^16 MSM 1.14 -> 1.01 ms in round 2). Applied to batches too it cost the 2^16 proof
// 22 -> 18 M constraints/s (more bit-sum groups, NR / 256, in every commit group).
constexpr uint32_t kRunBits = 4, kRunBitsMin = 1;
// run lanes aimed at: 65536 (one wave per SIMD) — with the 4-lane k_bitsum1 a lone 2^20
// MSM then runs rb = 3, 256 bit-sum groups: 3.44 -> 3.34 ms (131072: rb = 2, 512 groups)
constexpr size_t kRunLanes = 65536;
// kRunLanes, or PLK_RUN_LANES from the environment (sweeps)
inline size_t run_lanes() {
  static const size_t v = [] {
    const char* e = getenv("PLK_RUN_LANES");
    const long long x = e ? atoll(e) : 0;
    return x > 0 ? (size_t)x : kRunLanes;
  }();
  return v;
}
// a batch's rb: kRunBits, or PLK_RUN_BITS_BATCH from the environment (sweeps; 1 .. 8)
inline uint32_t batch_run_bits() {
  static const uint32_t v = [] {
    const char* e = getenv("PLK_RUN_BITS_BATCH");
    const int x = e ? atoi(e) : 0;
    return x >= 1 && x <= 8 ? (uint32_t)x : kRunBits;
  }();
  return v;
}
inline uint32_t run_bits(uint32_t B, uint32_t slots) {
  if (slots > 1) return std::min<uint32_t>(batch_run_bits(), 31 - __builtin_clz(B));
  uint32_t rb = kRunBits;
  while (rb > kRunBitsMin && (size_t)(B >> rb) < run_lanes()) --rb;
  return rb;
}

// Exclusive scan over the workgroup of K values per thread (wave shuffles, then the wave
// totals through LDS); tot = the workgroup totals. sh: K * 32 words.
template <int K>
__device__ __forceinline__ void block_scan_excl(uint32_t (&v)[K], uint32_t (&tot)[K], uint32_t* sh) {
  const uint32_t lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  uint32_t inc[K];
#pragma unroll
  for (int k = 0; k < K; ++k) inc[k] = v[k];
#pragma unroll
  for (uint32_t o = 1; o < 64; o <<= 1) {
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const uint32_t t = __shfl_up(inc[k], o, 64);
      if (lane >= o) inc[k] += t;
    }
  }
  if (lane == 63) {
#pragma unroll
    for (int k = 0; k < K; ++k) sh[k * 32 + wid] = inc[k];
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < K; ++k) {
    uint32_t base = 0, total = 0;
    for (uint32_t w = 0; w < nw; ++w) {
      const uint32_t s = sh[k * 32 + w];
      base += w < wid ? s : 0u;
      total += s;
    }
    v[k] = base + inc[k] - v[k];
    tot[k] = total;
  }
  __syncthreads();
}

// Wide pass 1: per-workgroup histogram of the coarse bins (bucket >> kFineBits), written whole
template <uint32_t C>
__global__ void __launch_bounds__(kHistThreads) k_chist(MsmBatch batch, MsmCfg cfg, uint32_t NC,
                                                        uint32_t fb, uint32_t* __restrict__ blockhist) {
  __shared__ uint32_t hist[kCoarseMax];
  const uint32_t slot = blockIdx.y;
  uint32_t i0, i1;
  slot_range(batch.len[slot], i0, i1);
  const Fr* sc = batch.scalars[slot];
  for (uint32_t b = threadIdx.x; b < NC; b += blockDim.x) hist[b] = 0;
  __syncthreads();
  for_scalars(sc, i0, i1, threadIdx.x, blockDim.x, [&](uint32_t, const Fr& s, bool) {
    each_digit<C>(s, cfg, [&](uint32_t, int d) {
      const uint32_t b = (uint32_t)(d < 0 ? -d : d) - 1u - cfg.b_lo;  // d = 0: wraps past B
      if (b < cfg.B) atomicAdd(&hist[b >> fb], 1u);
    });
  });
  __syncthreads();
  uint32_t* out = blockhist + ((size_t)slot * gridDim.x + blockIdx.x) * NC;
  for (uint32_t b = threadIdx.x; b < NC; b += blockDim.x) out[b] = hist[b];
}

// Wide pass 2 (after k_block_scan over the bins): every workgroup scans the bin totals into
// bin offsets (workgroup 0 also stores them), then each digit's (code, bucket) takes the next
// slot of its bin in this workgroup's range.
template <uint32_t C>
__global__ void __launch_bounds__(kHistThreads) k_cscatter(MsmBatch batch, MsmCfg cfg, uint32_t NC,
                                                           uint32_t fb, uint64_t n_srs,
                                                           const uint32_t* __restrict__ ccounts,
                                                           const uint32_t* __restrict__ blockhist,
                                                           uint32_t* __restrict__ coarse_off,
                                                           uint2* __restrict__ tmp, uint64_t tmp_stride) {
  __shared__ uint32_t hist[kCoarseMax];
  __shared__ uint32_t sh[32];
  const uint32_t slot = blockIdx.y, tid = threadIdx.x;
  const uint32_t* cc = ccounts + (size_t)slot * NC;
  const uint32_t* bh = blockhist + ((size_t)slot * gridDim.x + blockIdx.x) * NC;
  uint32_t* co = coarse_off + (size_t)slot * (NC + 1);
  uint32_t loc[4], v[1], tot[1];
  v[0] = 0;
#pragma unroll
  for (uint32_t q = 0; q < 4; ++q) {
    const uint32_t b = 4 * tid + q;
    loc[q] = b < NC ? cc[b] : 0u;
    v[0] += loc[q];
  }
  block_scan_excl<1>(v, tot, sh);
  uint32_t run = v[0];
#pragma unroll
  for (uint32_t q = 0; q < 4; ++q) {
    const uint32_t b = 4 * tid + q;
    if (b < NC) {
      if (blockIdx.x == 0) co[b] = run;
      hist[b] = run + bh[b];
    }
    run += loc[q];
  }
  if (blockIdx.x == 0 && tid == 0) co[NC] = tot[0];
  __syncthreads();
  uint32_t i0, i1;
  slot_range(batch.len[slot], i0, i1);
  const Fr* sc = batch.scalars[slot];
  uint2* out = tmp + (size_t)slot * tmp_stride;
  for_scalars(sc, i0, i1, tid, blockDim.x, [&](uint32_t i, const Fr& s, bool neg) {
    each_digit<C>(s, cfg, [&](uint32_t w, int d) {
      const uint32_t b = (uint32_t)(d < 0 ? -d : d) - 1u - cfg.b_lo;  // d = 0: wraps past B
      if (b < cfg.B) {
        const uint32_t pos = atomicAdd(&hist[b >> fb], 1u);
        out[pos] = make_uint2((uint32_t)(w * n_srs + i) | (((d < 0) != neg) ? 0x80000000u : 0u), b);
      }
    });
  });
}

// Wide pass 3: one workgroup per (bin, slot), one thread per bucket of the bin. Counting sort
// of the bin's entries by bucket into its own region of `sorted`; bucket offsets (global),
// per-bucket task and full-task offsets relative to the bin, the bin's totals and the
// global histogram of tail lengths (for the execution order of the tasks).
// loads in flight per thread and pass (8 measured no faster in round 5:
// profiles/r05_sort_prefetch_readback_ab.jsonl)
constexpr uint32_t kFineLoads = 4;
template <uint32_t FB>
__global__ void __launch_bounds__(1u << FB) k_fine(uint32_t B, uint32_t NC, uint32_t chunk,
                                                const uint32_t* __restrict__ coarse_off,
                                                const uint2* __restrict__ tmp, uint64_t tmp_stride,
                                                uint32_t* __restrict__ sorted, uint64_t sorted_stride,
                                                uint32_t* __restrict__ offsets,
                                                uint32_t* __restrict__ task_rel,
                                                uint32_t* __restrict__ full_rel,
                                                uint32_t* __restrict__ bin_tot,
                                                uint32_t* __restrict__ len_count) {
  constexpr uint32_t kFine = 1u << FB;
  __shared__ uint32_t cnt[kFine];
  __shared__ uint32_t s_len[kChunkMax];
  __shared__ uint32_t sh[3 * 32];
  const uint32_t slot = blockIdx.y, bin = blockIdx.x, tid = threadIdx.x;
  const uint32_t lo = coarse_off[(size_t)slot * (NC + 1) + bin];
  const uint32_t hi = coarse_off[(size_t)slot * (NC + 1) + bin + 1];
  const uint2* in = tmp + (size_t)slot * tmp_stride;
  cnt[tid] = 0;
  if (tid < kChunkMax) s_len[tid] = 0;
  __syncthreads();
  {  // kFineLoads loads in flight per thread, then their atomics
    uint32_t e = lo + tid;
    for (; e + (kFineLoads - 1) * kFine < hi; e += kFineLoads * kFine) {
      uint32_t k[kFineLoads];
#pragma unroll
      for (uint32_t u = 0; u < kFineLoads; ++u) k[u] = in[e + u * kFine].y;
#pragma unroll
      for (uint32_t u = 0; u < kFineLoads; ++u) atomicAdd(&cnt[k[u] & (kFine - 1)], 1u);
    }
    for (; e < hi; e += kFine) atomicAdd(&cnt[in[e].y & (kFine - 1)], 1u);
  }
  __syncthreads();
  const uint32_t c = cnt[tid];
  if (c % chunk) atomicAdd(&s_len[c % chunk], 1u);
  uint32_t v[3] = {c, (c + chunk - 1) / chunk, c / chunk}, tot[3];
  block_scan_excl<3>(v, tot, sh);  // its barriers also order the s_len atomics and cnt reads
  const uint32_t b = bin * kFine + tid;  // B = NC * kFine
  offsets[(size_t)slot * (B + 1) + b] = lo + v[0];
  task_rel[(size_t)slot * B + b] = v[1];
  full_rel[(size_t)slot * B + b] = v[2];
  if (tid == 0) {
    bin_tot[(size_t)slot * 2 * NC + bin] = tot[1];
    bin_tot[(size_t)slot * 2 * NC + NC + bin] = tot[2];
    if (bin == NC - 1) offsets[(size_t)slot * (B + 1) + B] = hi;
  }
  if (tid < kChunkMax && s_len[tid]) atomicAdd(&len_count[(size_t)slot * kChunkMax + tid], s_len[tid]);
  cnt[tid] = v[0];  // cursor of bucket tid, relative to lo
  __syncthreads();
  uint32_t* out = sorted + (size_t)slot * sorted_stride + lo;
  uint32_t e = lo + tid;
  for (; e + (kFineLoads - 1) * kFine < hi; e += kFineLoads * kFine) {
    uint2 x[kFineLoads];
    uint32_t pos[kFineLoads];
#pragma unroll
    for (uint32_t u = 0; u < kFineLoads; ++u) x[u] = in[e + u * kFine];
#pragma unroll
    for (uint32_t u = 0; u < kFineLoads; ++u) pos[u] = atomicAdd(&cnt[x[u].y & (kFine - 1)], 1u);
#pragma unroll
    for (uint32_t u = 0; u < kFineLoads; ++u) out[pos[u]] = x[u].x;
  }
  for (; e < hi; e += kFine) {
    const uint2 x = in[e];
    out[atomicAdd(&cnt[x.y & (kFine - 1)], 1u)] = x.x;
  }
}

// Wide pass 4: task records in the layout of k_make_tasks (full tasks first, bucket order;
// tails grouped by length, longest first). Bin bases are sums of the bin totals below.
template <uint32_t FB>
__global__ void __launch_bounds__(1u << FB) k_make_tasks_wide(uint32_t B, uint32_t NC, uint32_t chunk,
                                                           const uint32_t* __restrict__ offsets,
                                                           const uint32_t* __restrict__ task_rel,
                                                           const uint32_t* __restrict__ full_rel,
                                                           const uint32_t* __restrict__ bin_tot,
                                                           const uint32_t* __restrict__ len_count,
                                                           uint32_t* __restrict__ len_fill,
                                                           uint32_t* __restrict__ task_off,
                                                           uint2* __restrict__ tasks,
                                                           uint64_t task_stride) {
  __shared__ uint32_t s_cnt[kChunkMax], s_base[kChunkMax], s_lc[kChunkMax], sh[4 * 32];
  const uint32_t slot = blockIdx.y, bin = blockIdx.x, tid = threadIdx.x;
  const uint32_t* bt = bin_tot + (size_t)slot * 2 * NC;
  uint32_t v[4] = {0, 0, 0, 0}, tot[4];
  for (uint32_t q = tid; q < NC; q += blockDim.x) {
    const uint32_t a = bt[q], f = bt[NC + q];
    v[0] += q < bin ? a : 0u;
    v[1] += q < bin ? f : 0u;
    v[2] += a;
    v[3] += f;
  }
  if (tid < kChunkMax) {
    s_cnt[tid] = 0;
    s_lc[tid] = len_count[(size_t)slot * kChunkMax + tid];
  }
  block_scan_excl<4>(v, tot, sh);
  const uint32_t task_base = tot[0], full_base = tot[1], task_total = tot[2], full_total = tot[3];
  const uint32_t b = (bin << FB) + tid;
  const uint32_t* off = offsets + (size_t)slot * (B + 1);
  const uint32_t start = off[b], cnt = off[b + 1] - start;
  const uint32_t t0 = task_base + task_rel[(size_t)slot * B + b];
  const uint32_t f0 = full_base + full_rel[(size_t)slot * B + b];
  task_off[(size_t)slot * (B + 1) + b] = t0;
  if (b == B - 1) task_off[(size_t)slot * (B + 1) + B] = task_total;
  const uint32_t nfull = cnt / chunk, tail = cnt - nfull * chunk;
  uint32_t rank = 0;
  if (tail) rank = atomicAdd(&s_cnt[tail], 1u);
  __syncthreads();
  if (tid < kChunkMax && s_cnt[tid]) {
    uint32_t base = full_total;  // tails of length l start after all longer tails
    for (uint32_t l = tid + 1; l < kChunkMax; ++l) base += s_lc[l];
    s_base[tid] = base + atomicAdd(&len_fill[(size_t)slot * kChunkMax + tid], s_cnt[tid]);
  }
  __syncthreads();
  tasks += (size_t)slot * task_stride;
  for (uint32_t t = 0; t < nfull; ++t)
    tasks[f0 + t] = make_uint2(start + t * chunk, (t0 + t) | ((chunk - 1) << kTaskShift));
  if (tail)
    tasks[s_base[tail] + rank] =
        make_uint2(start + nfull * chunk, (t0 + nfull) | ((tail - 1) << kTaskShift));
}

// Bucket sums S_b = sum of bucket b's accumulation partials (task_off[b] .. task_off[b+1]):
// 2^lp lanes per bucket (consecutive lanes of one wave, 2^lp <= 16), each adding every
// 2^lp-th partial, then a tree over the lanes through cross-lane shuffles of the packed
// point (no LDS: these long add chains would otherwise hold 48 KiB of a CU's LDS per
// workgroup while other proofs' kernels wait for it). 2^lp is sized on the host to the
// partials per bucket, so the sequential chain stays ~PLK_LANE_PARTIALS additions at every
// MSM size, unless the grid is already full.
__device__ __forceinline__ RFp shfl_down_rfp(const RFp& v, uint32_t h) {
  Fp x = rx_pack(v);
#pragma unroll
  for (int i = 0; i < 12; ++i) x.v[i] = __shfl_down(x.v[i], h, 64);
  return rx_unpack(x);
}

__device__ __forceinline__ G1R shfl_down_g1r(const G1R& v, uint32_t h) {
  G1R o;
  o.X = shfl_down_rfp(v.X, h);
  o.Y = shfl_down_rfp(v.Y, h);
  o.ZZ = shfl_down_rfp(v.ZZ, h);
  o.ZZZ = shfl_down_rfp(v.ZZZ, h);
  return o;
}

// Sum over groups of w consecutive lanes (w a power of two <= 64, groups aligned; e = lane
// index in the group): lane e = 0 of each group ends with the group's sum. LAZY: g1r_add_lazy
// (straight-line, exceptional cases repaired after; ~275 VGPRs) or the branching g1r_add
// (~205 VGPRs: two waves per SIMD). One dependent addition costs a lone wave 12.5 / 14.3 us
// (tools/ubench_tail.hip, profiles/r03_ubench_tail.txt).
template <bool LAZY>
__device__ __forceinline__ G1R g1r_add_t(const G1R& a, const G1R& b) {
  return LAZY ? g1r_add_lazy(a, b) : g1r_add(a, b);
}
template <bool LAZY>
__device__ __forceinline__ G1R shfl_tree(G1R acc, uint32_t e, uint32_t w) {
  for (uint32_t h = w >> 1; h >= 1; h >>= 1) {
    const G1R o = shfl_down_g1r(acc, h);
    if (e < h) acc = g1r_add_t<LAZY>(acc, o);
  }
  return acc;
}

// QUAD: every "lane" of the reduction trees (k_bucket_sum, k_bitsum1/2) is a quad of 4 lanes
// holding the same values, adding with g1r_add_quad (g1r.hpp: one product per lane, ~3.5
// products issued per addition instead of ~15) — these trees are a chain of dependent
// additions on a few waves, so their time is one wave's issue of each level. Shuffles move by
// whole quads. Which form a batch takes: MsmWorkspace::tail_quad.
template <bool QUAD>
struct TailUnit {
  static constexpr uint32_t S = QUAD ? 4 : 1;  // lanes per unit
  uint32_t u, l;                               // unit index, lane in the unit
  __device__ explicit TailUnit(uint32_t tid) : u(tid / S), l(tid % S) {}
  template <bool LAZY>
  __device__ __forceinline__ G1R add(const G1R& a, const G1R& b) const {
    if constexpr (QUAD) return g1r_add_quad(a, b, l);
    else return g1r_add_t<LAZY>(a, b);
  }
  __device__ __forceinline__ G1R down(const G1R& v, uint32_t h) const { return shfl_down_g1r(v, h * S); }
  // sum over groups of w consecutive units (aligned, inside one wave), e = unit in the group
  template <bool LAZY>
  __device__ __forceinline__ G1R tree(G1R acc, uint32_t e, uint32_t w) const {
    for (uint32_t h = w >> 1; h >= 1; h >>= 1) {
      const G1R o = down(acc, h);
      if (e < h) acc = add<LAZY>(acc, o);
    }
    return acc;
  }
};

// k_bitsum1: the branching addition (single-lane form) at two waves per SIMD (2 workgroups of
// 256 per CU: a lone 2^20 MSM's 512 groups in one round instead of two)
#ifndef PLK_BITSUM_WAVES
#define PLK_BITSUM_WAVES 2
#endif

template <bool QUAD>
__global__ void __launch_bounds__(256) k_bucket_sum(const uint32_t* __restrict__ task_off,
                                                    uint32_t B, uint32_t lp, uint64_t task_stride,
                                                    const G1xyzz* __restrict__ partials,
                                                    G1xyzz* __restrict__ bsum) {
  const uint32_t slot = blockIdx.y;
  const TailUnit<QUAD> T(blockIdx.x * 256 + threadIdx.x);  // unit = one lane of the bucket's 2^lp
  const uint32_t P = 1u << lp, s = T.u & (P - 1);
  const uint32_t b = T.u >> lp;
  task_off += (size_t)slot * (B + 1);
  partials += (size_t)slot * task_stride;
  // the branching g1r_add here: ~200 VGPRs (2 waves per SIMD) against ~325 for the lazy form
  G1R acc = g1r_infinity();
  if (b < B)
    for (uint32_t t = task_off[b] + s; t < task_off[b + 1]; t += P) acc = T.template add<false>(acc, ld_g1r(&partials[t]));
  acc = T.template tree<false>(acc, s, P);  // units s < h add unit s + h (same bucket)
  if (s == 0 && T.l == 0 && b < B) st_g1r(&bsum[(size_t)slot * B + b], QUAD ? g1r_lazy_finish(acc) : acc);
}

#ifndef PLK_RUNSUM_WAVES
#define PLK_RUNSUM_WAVES 1  // ~270 VGPRs; a 2-wave cap spills in the loop (runsum1 3.43 -> 3.07 ms per proof uncapped)
#endif
// Wide bucket sets, reduction: runs of K = 2^rb consecutive buckets b = rK + t.
//   sum_b (b + 1) S_b = sum_r (T_r + rK Y_r) = K (sum_r (r + 1) Y_r - sum_r Y_r) + sum_r T_r,
//   R_(r,t) = sum_(t' >= t) S_(rK+t') (suffix sums), Y_r = R_(r,0), T_r = sum_t R_(r,t).
// 2 additions per bucket with every lane busy (the bit-sum trees over 2^19 buckets left most
// lanes idle); the weighted sum over the runs is the bit-sum reduction, sum_r Y_r (its A)
// and sum_r T_r extra outputs of it, the host multiplies by K. Two kernels with ONE
// accumulator each (both chains in one lane need 3 live points: over 256 VGPRs).
//
// Step 1, lane r: the suffix sums R_(r,t), t = K-1 .. 0, straight from the bucket's
// accumulation partials (S_b is never formed: R += S_b is the same sum taken partial by
// partial), stored lazily (X < 8p, Y < 4p fit the packed layout) to rsum[b].
__global__ void __launch_bounds__(256, PLK_RUNSUM_WAVES) k_runsum1(const uint32_t* __restrict__ task_off, uint32_t B, uint32_t rb,
                                                 uint64_t task_stride,
                                                 const G1xyzz* __restrict__ partials,
                                                 G1xyzz* __restrict__ rsum) {
  const uint32_t K = 1u << rb;
  const uint32_t slot = blockIdx.y, NR = B >> rb;
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= NR) return;
  task_off += (size_t)slot * (B + 1);
  partials += (size_t)slot * task_stride;
  rsum += (size_t)slot * B;
  // the rare path's copy of the accumulator waits in LDS, not in 56 live registers
  __shared__ G1xyzz s_prev[256];
  G1xyzz* prev = &s_prev[threadIdx.x];
  G1R R = g1r_infinity();
  uint32_t pe = task_off[r * K + K];
  for (uint32_t t = K; t-- > 0;) {
    const uint32_t b = r * K + t;
    const uint32_t p0 = task_off[b];
    for (uint32_t p = p0; p < pe; ++p) {
      st_g1r(prev, R);
      G1R c = g1r_add_lazy_sl(R, ld_g1r(&partials[p]));
      if (rx_is_zero(c.ZZ)) c = g1r_add_lazy_fix(ld_g1r(prev), ld_g1r(&partials[p]), c.X);  // rare
      R = c;
    }
    pe = p0;
    st_g1r(&rsum[b], R);
  }
}

// Step 2, lane r: T_r = sum_t R_(r,t) and Y_r = R_(r,0) (canonical [0, 2p) coordinates for
// the bit sums).
__global__ void __launch_bounds__(256, PLK_RUNSUM_WAVES) k_runsum2(uint32_t B, uint32_t rb, const G1xyzz* __restrict__ rsum,
                                                 G1xyzz* __restrict__ ys, G1xyzz* __restrict__ ts) {
  const uint32_t K = 1u << rb;
  const uint32_t slot = blockIdx.y, NR = B >> rb;
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= NR) return;
  rsum += (size_t)slot * B + (size_t)r * K;
  __shared__ G1xyzz s_prev[256];  // as in k_runsum1
  G1xyzz* prev = &s_prev[threadIdx.x];
  G1R T = ld_g1r(&rsum[0]);
  for (uint32_t t = 1; t < K; ++t) {
    st_g1r(prev, T);
    G1R c = g1r_add_lazy_sl(T, ld_g1r(&rsum[t]));
    if (rx_is_zero(c.ZZ)) c = g1r_add_lazy_fix(ld_g1r(prev), ld_g1r(&rsum[t]), c.X);  // rare
    T = c;
  }
  st_g1r(&ys[(size_t)slot * NR + r], g1r_lazy_finish(ld_g1r(&rsum[0])));
  st_g1r(&ts[(size_t)slot * NR + r], g1r_lazy_finish(T));
}

// Bucket reduction sum_b (b+1) S_b, split per workgroup g of 256 buckets b = 256g + u,
// u = 16a + c (a, c < 16):
//   sum_u (256g + u + 1) S_(g,u) = sum_(j<8) 2^j T_j(g) + (256g + 1) A_g,
//   T_j(g) = sum of S_(g,u) over u with bit j set,  A_g = sum_u S_(g,u).
// With row sums Row_a = sum_c S_(g,16a+c) and column sums Col_c = sum_a S_(g,16a+c), T_j for
// j < 4 is a sum of the 8 columns with bit j of c set and T_(4+i) a sum of the 8 rows with
// bit i of a set; A_g is the sum of the rows: 480 + 71 additions per 256 buckets instead of
// the 1 144 of bit sums taken over the buckets themselves.
// k_bitsum1 (one workgroup per g): the bucket sums S (k_bucket_sum), the 32
// row / column sums (8 consecutive lanes each: one addition, then a 3-level shuffle tree),
// then the 9 outputs from them (wave 0). out[slot][g][0..7] = T_j(g), [8] = A_g; with `zin`
// (wide bucket sets) also [9] = the plain sum of the group's 256 Z values (k_runsum).
constexpr uint32_t kBitsumOut = 10;

// k_bitsum1's fold of k_bitsum2 (done == nullptr: off): per-slot arrival counters (zero
// between batches), the readback record's bit sums and entry counts, as k_bitsum2 takes them
struct BitsumFold {
  uint32_t* done;
  G1xyzz* out2;
  const uint32_t* offsets;
  uint32_t* entries;
  uint32_t B, nbits, nout;
};
constexpr uint32_t kFoldMaxGroups = 16;

// k-th of the 8 indices in [0, 16) with bit j set
__device__ __forceinline__ uint32_t with_bit(uint32_t k, uint32_t j) {
  return ((k >> j) << (j + 1)) | (1u << j) | (k & ((1u << j) - 1u));
}

// threads of k_bitsum1: 4 units per row / column sum, 1 or 4 lanes per unit. Quads stay at 8
// waves per workgroup (2 per SIMD: the quad addition needs ~250 VGPRs), so with Z (48 sums) the
// group takes TWO workgroups (blockIdx.z = role): the 32 row / column sums and their outputs
// 0..8, and the 16 plain-sum rows and output 9, side by side instead of 8-member chains
constexpr uint32_t bitsum1_threads(bool z, bool quad) {
  return quad ? 512 : (z ? 192 : 128);
}
template <bool Z, bool QUAD>
__global__ void __launch_bounds__(bitsum1_threads(Z, QUAD), PLK_BITSUM_WAVES) k_bitsum1(uint32_t B, const G1xyzz* __restrict__ bsum,
                                                                           const G1xyzz* __restrict__ zin,
                                                                           G1xyzz* __restrict__ out,
                                                                           BitsumFold fold) {
  // the group's values (buckets or run sums Y; with Z also the 256 plain-sum values) are
  // read straight from HBM and the trees run over cross-lane shuffles: LDS holds only the
  // NS row / column sums (9 KiB instead of 105 — a resident k_bitsum1 used to keep the other
  // proofs' NTT passes off its CU).
  // The NS sums of 16 take 4 consecutive units each, and each unit first adds its 4 members
  // in sequence (every unit busy), then a 2-level shuffle tree: 3 + 2 levels on NS / 16 waves.
  // The tree kernels are issue-bound — a wave issues the whole addition however few of its
  // lanes are active — so units idle in a shuffle level cost as much as busy ones: 8 units
  // per sum with 2 members each (3-level tree) issued twice the wave-additions (round 3:
  // 8 waves x 4 levels + 4 against 3 waves x 5 levels + 4 per group).
  constexpr uint32_t NS = Z ? 48 : 32;
  constexpr bool SPLIT = Z && QUAD;  // two workgroups per group (bitsum1_threads)
  constexpr uint32_t NSU = 4, MEM = 16 / NSU;  // units per sum, members per unit
  constexpr uint32_t NU = bitsum1_threads(Z, QUAD) / TailUnit<QUAD>::S;  // units
  constexpr bool LZ = false;
  __shared__ G1xyzz sh[NS];
  const uint32_t slot = blockIdx.y, g = blockIdx.x, tid = threadIdx.x;
  const uint32_t role = SPLIT ? blockIdx.z : 0;
  const TailUnit<QUAD> T(tid);
  out += ((size_t)slot * gridDim.x + g) * kBitsumOut;
  auto value = [&](uint32_t x) -> G1R {  // x < 256: bsum, else zin; past B: infinity
    const uint32_t b = g * 256 + (x & 255);
    const G1xyzz* src = x < 256 ? bsum : zin;
    return b < B ? ld_g1r(&src[(size_t)slot * B + b]) : g1r_infinity();
  };
  {  // sum q < 16: row a = q (members 16q + c); 16 <= q < 32: column c = q - 16 (members
     // c + 16a); q >= 32 (Z): row q - 32 of the plain-sum values. Unit e < NSU of the sum's
     // NSU takes members MEM e .. MEM e + MEM - 1 of its row / column.
    const uint32_t q = T.u / NSU + (role ? 32 : 0), e = T.u % NSU;
    auto member = [&](uint32_t i) {  // i-th member of sum q, i < 16
      return q < 16 ? 16 * q + i : q < 32 ? (q - 16) + 16 * i : 256 + 16 * (q - 32) + i;
    };
    if (q < NS && (!SPLIT || role || q < 32)) {  // uniform per sum (its NSU units)
      G1R acc = value(member(MEM * e));
#pragma unroll 1
      for (uint32_t i = 1; i < MEM; ++i) acc = T.template add<LZ>(acc, value(member(MEM * e + i)));
      acc = T.template tree<LZ>(acc, e, NSU);
      if (e == 0 && T.l == 0) st_g1r(&sh[q], acc);
    }
  }
  __syncthreads();
  // units 0..31 = T_0..T_7, 4 units each (2 terms per unit); units 32..39 = A_g, 8 units
  // (rows 2e, 2e + 1); with Z units 40..47 = the plain sum (its rows 2e, 2e + 1); then trees
  // (unit groups never straddle a wave: 4 or 8 units of 1 or 4 lanes, aligned)
  if (T.u < 64) {
    // (SPLIT: role 0 the units 0..39, role 1 the plain sum as units 40..47)
    const uint32_t t = role ? 40 + T.u : T.u;
    const bool on = role ? T.u < 8 : t < (Z && !SPLIT ? 48u : 40u);
    const uint32_t s = t < 32 ? t >> 2 : t < 40 ? 8 : 9, e = t < 32 ? t & 3 : (t - 32) & 7;
    const uint32_t w = t < 32 ? 4 : 8;
    uint32_t i0 = 0, i1 = 0;
    if (s < 4) {  // columns c with bit s
      i0 = 16 + with_bit(2 * e, s);
      i1 = 16 + with_bit(2 * e + 1, s);
    } else if (s < 8) {  // rows a with bit s - 4
      i0 = with_bit(2 * e, s - 4);
      i1 = with_bit(2 * e + 1, s - 4);
    } else if (on) {  // all rows (A_g) / all plain-sum rows
      i0 = (s == 8 ? 0 : 32) + 2 * e;
      i1 = i0 + 1;
    }
    G1R acc = g1r_infinity();
    if (on) acc = T.template add<LZ>(ld_g1r(&sh[i0]), ld_g1r(&sh[i1]));
    for (uint32_t h = 4; h >= 1; h >>= 1) {  // groups of w consecutive units
      const G1R o = T.down(acc, h);
      if (on && e < h && h < w) acc = T.template add<LZ>(acc, o);
    }
    if (on && e == 0 && T.l == 0) st_g1r(&out[s], acc);
  }
  if (!fold.done) return;
  // few groups (G <= kFoldMaxGroups): the slot's last workgroup to finish runs k_bitsum2's sums
  // here (one dispatch fewer per batch; small proofs are dispatch-rate bound). Release this
  // group's outputs, count it in, and the last one acquires the others' before reading them.
  __shared__ uint32_t s_last;
  __threadfence();
  __syncthreads();
  if (tid == 0) s_last = atomicAdd(&fold.done[slot], 1u) == gridDim.x * gridDim.z - 1 ? 1u : 0u;
  __syncthreads();
  if (!s_last) return;
  __threadfence();
  const G1xyzz* in = out - (size_t)g * kBitsumOut;  // this slot's groups
  const uint32_t e = T.u & 7, G = gridDim.x;
  for (uint32_t j0 = 0; j0 < fold.nout; j0 += NU / 8) {  // uniform trip count: the trees shuffle
    const uint32_t j = j0 + (T.u >> 3);
    G1R acc = g1r_infinity();
    if (j < fold.nout) {  // output j: 8 units, unit e takes the groups g = e mod 8
      for (uint32_t gg = e; gg < G; gg += 8) {
        const G1xyzz* v = &in[(size_t)gg * kBitsumOut];
        if (j >= fold.nbits) {  // wide sets: the plain sums (j = nbits) and the A_g (nbits + 1)
          acc = T.template add<LZ>(acc, ld_g1r(&v[j == fold.nbits ? 9 : 8]));
        } else if (j < 8) {
          acc = T.template add<LZ>(acc, ld_g1r(&v[j]));
          if (j == 0) acc = T.template add<LZ>(acc, ld_g1r(&v[8]));
        } else if ((gg >> (j - 8)) & 1u) {
          acc = T.template add<LZ>(acc, ld_g1r(&v[8]));
        }
      }
    }
    acc = T.template tree<LZ>(acc, e, 8);
    if (j < fold.nout && e == 0 && T.l == 0) st_g1r(&fold.out2[(size_t)slot * fold.nout + j], g1r_lazy_finish(acc));
  }
  if (tid == 0) {
    fold.entries[slot] = fold.offsets[(size_t)slot * (fold.B + 1) + fold.B];
    fold.done[slot] = 0;  // ready for the next batch (stream order)
  }
}

// Workgroup j of slot: T_j = sum_g T_j(g) for 0 < j < 8; T_0 = sum_g (T_0(g) + A_g);
// T_(8+i) = sum_(g: bit i of g) A_g; wide bucket sets: j = nbits sum_g of the plain sums,
// j = nbits + 1 sum_g A_g.
// Also the batch's readback record (ReadbackHeader): workgroup (0, slot) copies the slot's
// entry count (its point additions, offsets[B]) next to the flags k_any_nonzero stamped, so
// the host reads flags, counts and bit sums with ONE copy.
// k_bitsum2's additions: lazy (the branching g1r_add measured no faster, round 2)
// QUAD: 128 units of 4 lanes (8 waves, 2 per SIMD: the quad addition's ~250 VGPRs)
constexpr uint32_t kBitsum2Units(bool quad) { return quad ? 128 : 256; }
template <bool QUAD>
__global__ void __launch_bounds__(QUAD ? 512 : 256) k_bitsum2(const G1xyzz* __restrict__ in, uint32_t G,
                                                 uint32_t nbits, uint32_t nout,
                                                 G1xyzz* __restrict__ out,
                                                 const uint32_t* __restrict__ offsets, uint32_t B,
                                                 uint32_t* __restrict__ entries) {
  constexpr uint32_t UPW = QUAD ? 16 : 64;  // units per wave
  constexpr bool LZ = true;
  __shared__ G1xyzz sh[16];
  const uint32_t slot = blockIdx.y, tid = threadIdx.x, j = blockIdx.x;
  const TailUnit<QUAD> T(tid);
  if (j == 0 && tid == 0) entries[slot] = offsets[(size_t)slot * (B + 1) + B];
  in += (size_t)slot * G * kBitsumOut;
  // lazy additions (one wave per SIMD is all this narrow kernel runs); the stored totals are
  // finished to [0, 2p) for the host. A unit's first term is taken as is (adding it to
  // infinity would run the repair path).
  G1R acc = g1r_infinity();
  bool have = false;
  for (uint32_t g = T.u; g < G; g += kBitsum2Units(QUAD)) {
    const G1xyzz* e = &in[(size_t)g * kBitsumOut];
    // wide sets: j = nbits sums the plain sums, nbits + 1 the A_g
    uint32_t i0 = kBitsumOut, i1 = kBitsumOut;  // kBitsumOut: none
    if (j >= nbits) i0 = j == nbits ? 9 : 8;
    else if (j < 8) i0 = j, i1 = j == 0 ? 8 : kBitsumOut;
    else if ((g >> (j - 8)) & 1u) i0 = 8;
    for (uint32_t i : {i0, i1}) {
      if (i == kBitsumOut) continue;
      const G1R v = ld_g1r(&e[i]);
      if (have) acc = T.template add<LZ>(acc, v);
      else acc = v;
      have = true;
    }
  }
  // units >= G hold infinity: a shuffle tree over each wave's min(G, UPW) units, then the
  // wave totals (up to 4 / 8) through LDS
  uint32_t w0 = 1;
  while (w0 < min(G, UPW)) w0 <<= 1;
  acc = T.template tree<LZ>(acc, T.u % UPW, w0);
  const uint32_t gu = min(G, kBitsum2Units(QUAD)), nw = gu > UPW ? (gu + UPW - 1) / UPW : 1;  // waves holding values
  if (T.u % UPW == 0 && T.l == 0 && T.u / UPW < nw) st_g1r(&sh[T.u / UPW], acc);
  __syncthreads();
  if (T.u < UPW) {  // wave 0: unit e < nw/2 adds a pair of wave totals, then a tree
    const uint32_t e = T.u, np = (nw + 1) / 2;
    acc = g1r_infinity();
    if (e < np) {
      acc = ld_g1r(&sh[2 * e]);
      if (2 * e + 1 < nw) acc = T.template add<LZ>(acc, ld_g1r(&sh[2 * e + 1]));
    }
    uint32_t w = 1;
    while (w < np) w <<= 1;
    acc = T.template tree<LZ>(acc, e, w);
    if (e == 0 && T.l == 0) st_g1r(&out[(size_t)slot * nout + j], g1r_lazy_finish(acc));
  }
}

// flag[slot] = gen if any scalar in [len, check_len) is nonzero (commit degree check). The
// flags are stamped with the batch's generation number instead of being cleared per batch:
// a stale flag holds an older generation, so no memset dispatch is needed. Every writer
// stores the same value, so a plain store does (no atomic: the flags live in mapped host
// memory, where an atomic would need the platform's PCIe atomics).
__global__ void k_any_nonzero(MsmBatch batch, uint32_t* __restrict__ flag, uint32_t gen) {
  const uint32_t slot = blockIdx.y;
  const uint64_t i = (uint64_t)batch.len[slot] + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= batch.check_len[slot]) return;
  if (!fe_is_zero(ld_fr(&batch.scalars[slot][i]))) flag[slot] = gen;
}

}  // namespace

// R'-domain [0, 2p) packed coordinates (ffr.hpp) -> canonical R-domain: x * 2^-SH
// (SH = BL - 384 = 6) as the R-domain product x * 2^(384 - SH) / 2^384.
static Fp fp_rx_to_r(Fp x) {
  constexpr int SH = RxShape<FpCfg>::B * RxShape<FpCfg>::L - 32 * FpCfg::N;
  static_assert(SH > 0 && SH < 32, "R' / R shift");
  fe_reduce_once(x);
  Fp k = fe_zero<FpCfg>();
  k.v[11] = 1u << (32 - SH);  // 2^(384 - SH) (< p)
  return fe_mul(x, k);
}
static G1xyzz rx_to_r_domain(const G1xyzz& p) {
  G1xyzz r;
  r.X = fp_rx_to_r(p.X);
  r.Y = fp_rx_to_r(p.Y);
  r.ZZ = fp_rx_to_r(p.ZZ);
  r.ZZZ = fp_rx_to_r(p.ZZZ);
  return r;
}

// STMT with CC = the SRS's window size as a compile-time constant for the sizes choose_c
// picks (each_digit's unrolled form), 0 (run-time layout) otherwise
#define PLK_BY_C(c_, ...)                          \
  switch (c_) {                                    \
    case 10: { constexpr uint32_t CC = 10; __VA_ARGS__; } break; \
    case 12: { constexpr uint32_t CC = 12; __VA_ARGS__; } break; \
    case 13: { constexpr uint32_t CC = 13; __VA_ARGS__; } break; \
    case 15: { constexpr uint32_t CC = 15; __VA_ARGS__; } break; \
    case 17: { constexpr uint32_t CC = 17; __VA_ARGS__; } break; \
    case 20: { constexpr uint32_t CC = 20; __VA_ARGS__; } break; \
    default: { constexpr uint32_t CC = 0; __VA_ARGS__; } break;  \
  }

int ws_reserve(plk_srs* s, MsmWorkspace& w, size_t len, uint32_t slots, hipStream_t stream) {
  const bool same_shape = w.cap_c == s->c && w.cap_windows == s->windows;
  if (same_shape && len <= w.cap_len && slots <= w.cap_slots && w.cap_len) return PLK_OK;
  // buffers only ever grow (DevBuf::alloc), so re-sizing for another shape keeps the larger
  // of the old and new needs; the strides below always match the current shape
  len = std::max(len, w.cap_len);
  slots = std::max(slots, w.cap_slots);
  const size_t B = (size_t)1 << (s->c - 1);
  const bool wide = B > kLdsBuckets;
  const size_t NC = B >> kFineBits;
  // runs over all slots of a batch (run_bits: a batch runs B >> kRunBits per slot, a lone
  // MSM fewer than 2 kRunLanes unless rb = kRunBits)
  const size_t max_runs =
      std::max<size_t>(slots * (B >> std::min(kRunBits, batch_run_bits())), B >> kRunBitsMin);
  if (wide && NC > kCoarseMax) return PLK_E_ARG;
  const size_t entries = (size_t)s->windows * len;
  // small shapes (k_sort_one's) may run tasks of kChunkSmall points (msm_run_batch)
  const uint32_t chunk_min = (!wide && B <= kSortSmallMax && len <= kSortOneMax) ? kChunkSmall : kChunkMin;
  const size_t max_tasks = entries / chunk_min + B + 1;
  const size_t groups = wide ? (max_runs + 255) / 256 : slots * ((B + 255) / 256);
  if (max_tasks >= ((size_t)1 << kTaskShift)) return PLK_E_ARG;  // task records: partial index bits
  int st;
  const size_t hb = wide ? NC : B;  // histogram bins: coarse bins or buckets
  if ((st = w.counts.alloc(slots * hb * 4))) return st;
  if ((st = w.offsets.alloc(slots * (B + 1) * 4))) return st;
  if ((st = w.task_off.alloc(slots * (B + 1) * 4))) return st;
  if ((st = w.blockhist.alloc(slots * kHistBlocksMax * hb * 4))) return st;
  if ((st = w.full_off.alloc(slots * B * 4))) return st;
  if ((st = w.len_cur.alloc(slots * kChunkMax * 4))) return st;
  if ((st = w.sorted.alloc(slots * (entries + 1) * 4))) return st;
  if ((st = w.tasks.alloc(slots * max_tasks * sizeof(uint2)))) return st;
  if ((st = w.partials.alloc(slots * max_tasks * sizeof(G1xyzz)))) return st;
  if (wide) {
    if ((st = w.tmp.alloc(slots * entries * sizeof(uint2)))) return st;
    if ((st = w.task_rel.alloc(slots * B * 4))) return st;
    if ((st = w.bin_tot.alloc(slots * 2 * NC * 4))) return st;
    if ((st = w.len_fill.alloc(slots * kChunkMax * 4))) return st;
    if ((st = w.coarse_off.alloc(slots * (NC + 1) * 4))) return st;
    if ((st = w.rsum.alloc(slots * B * sizeof(G1xyzz)))) return st;
    if ((st = w.ys.alloc(max_runs * sizeof(G1xyzz)))) return st;
    if ((st = w.zs.alloc(max_runs * sizeof(G1xyzz)))) return st;
  } else {
    if ((st = w.bsum.alloc(slots * B * sizeof(G1xyzz)))) return st;
  }
  if ((st = w.bits1.alloc(groups * kBitsumOut * sizeof(G1xyzz)))) return st;
  {  // k_bitsum1's fold counters: zero between batches (the last workgroup resets its slot's)
    void* before = w.done.ptr;
    if ((st = w.done.alloc(kMaxSlots * sizeof(uint32_t)))) return st;
    if (w.done.ptr != before) PLK_HIP_TRY(hipMemsetAsync(w.done.ptr, 0, kMaxSlots * sizeof(uint32_t), stream));
  }
  {  // readback record: header (flags, entry counts) then the bit sums (nout <= 32 per slot),
     // in coherent mapped host memory (round 5: the per-batch copy dispatch it replaces cost
     // small proofs a dispatch per commit group). The previous batch has completed (every
     // batch ends with a host wait), so the host may clear it.
    void* before = w.host_out.ptr;
    if ((st = w.host_out.alloc(sizeof(ReadbackHeader) + (size_t)kMaxSlots * 32 * sizeof(G1xyzz),
                               hipHostMallocMapped | hipHostMallocCoherent | hipHostMallocPortable)))
      return st;
    if (w.host_out.ptr != before) {  // fresh memory: the flags start at generation 0
      std::memset(w.host_out.ptr, 0, sizeof(ReadbackHeader));
      w.gen = 0;
      PLK_HIP_TRY(hipHostGetDevicePointer(&w.out_dev, w.host_out.ptr, 0));
    }
  }
  if (!w.ev0) PLK_HIP_TRY(hipEventCreate(&w.ev0));
  if (!w.ev1) PLK_HIP_TRY(hipEventCreate(&w.ev1));
  const int lds = (int)(std::min<uint32_t>((uint32_t)B, kLdsBuckets) * 4);
  if (!wide)  // k_scan_buckets stages the B counts (narrow sets: B <= kLdsBuckets)
    PLK_HIP_TRY(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_scan_buckets),
                                    hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  PLK_BY_C(s->c,
           PLK_HIP_TRY(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_hist<CC>),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, lds));
           PLK_HIP_TRY(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_scatter<CC>),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, lds)))
  w.cap_len = len;
  w.cap_slots = slots;
  w.cap_chunk_min = chunk_min;
  w.cap_c = s->c;
  w.cap_windows = s->windows;
  w.task_stride = max_tasks;
  w.sorted_stride = entries + 1;
  return PLK_OK;
}

// Runs `count` independent MSMs on the same SRS as one batch. For slot k: scalars
// d_scalars[k][0 .. lens[k]) (lens[k] <= n_srs) against the SRS prefix, and if
// check_lens[k] > lens[k] the tail [lens[k], check_lens[k]) must be zero (else that slot
// reports PLK_E_DEGREE). statuses[k] receives each slot's status.
// the bit-sum kernels of one batch (k_bitsum2 folded into k_bitsum1 when fold.done is set)
template <bool QUAD, bool QUAD2>
static void bitsum_launch(bool wide, uint32_t G, uint32_t slots, uint32_t NR, uint32_t B,
                          MsmWorkspace& w, const BitsumFold& fold, uint32_t nbits, uint32_t nout,
                          G1xyzz* bits_dev, ReadbackHeader* hdr_dev, hipStream_t stream) {
  if (wide) {
    hipLaunchKernelGGL((k_bitsum1<true, QUAD>), dim3(G, slots, QUAD ? 2 : 1), dim3(bitsum1_threads(true, QUAD)), 0, stream, NR,
                       (const G1xyzz*)w.ys.as<G1xyzz>(), (const G1xyzz*)w.zs.as<G1xyzz>(),
                       w.bits1.as<G1xyzz>(), fold);
  } else {
    hipLaunchKernelGGL((k_bitsum1<false, QUAD>), dim3(G, slots), dim3(bitsum1_threads(false, QUAD)), 0, stream, B,
                       (const G1xyzz*)w.bsum.as<G1xyzz>(), (const G1xyzz*)nullptr,
                       w.bits1.as<G1xyzz>(), fold);
  }
  if (!fold.done) {
    hipLaunchKernelGGL(k_bitsum2<QUAD2>, dim3(nout, slots), dim3(kBitsum2Units(QUAD2) * TailUnit<QUAD2>::S), 0, stream, w.bits1.as<G1xyzz>(),
                       G, nbits, nout, bits_dev, (const uint32_t*)w.offsets.as<uint32_t>(), B,
                       hdr_dev->entries);
  }
}

bool msm_parts_ok(const plk_srs* s, uint32_t parts) {
  if (parts == 0 || (parts & (parts - 1))) return false;
  // a part's bucket range stays a wide set's (two-level sort, run sums): >= 2^14 buckets
  return parts == 1 ||
         ((1u << (s->c - 1)) > kLdsBuckets && ((1u << (s->c - 1)) / parts) >= (1u << 14));
}

int msm_run_batch(plk_srs* s, MsmWorkspace& w, const Fr* const* d_scalars, const size_t* lens,
                  const size_t* check_lens, size_t count, plk_g1* outs, int* statuses,
                  hipStream_t stream, uint32_t part, uint32_t parts) {
  if (count == 0) return PLK_OK;
  if (count > kMaxSlots) return PLK_E_ARG;
  if (!msm_parts_ok(s, parts) || part >= parts) return PLK_E_ARG;
  size_t max_len = 0, max_tail = 0, total_entries = 0;
  MsmBatch batch{};
  for (size_t k = 0; k < count; ++k) {
    if (lens[k] > s->n) return PLK_E_ARG;
    batch.scalars[k] = d_scalars[k];
    batch.len[k] = (uint32_t)lens[k];
    batch.check_len[k] = check_lens ? check_lens[k] : lens[k];
    max_len = std::max(max_len, lens[k]);
    if (batch.check_len[k] > lens[k])
      max_tail = std::max<size_t>(max_tail, batch.check_len[k] - lens[k]);
    total_entries += (size_t)s->windows * lens[k];
  }
  int st;
  if ((st = ws_reserve(s, w, max_len ? max_len : 1, (uint32_t)count, stream))) return st;
  // B: the buckets this call reduces (all 2^(c-1), or a part's range of them)
  const uint32_t B_all = 1u << (s->c - 1), B = B_all / parts;
  const MsmCfg cfg{s->c, s->windows, B, s->narrow, part * B};
  // wide bucket sets: two-level sort and run-sum reduction; the bit sums then run over the
  // NR = B / 2^rb runs instead of the buckets
  const bool wide = B_all > kLdsBuckets;
  const uint32_t rb = run_bits(B, (uint32_t)count);
  // coarse-bin width (wide sets): 2^10 buckets, finer for a part's narrower range
  uint32_t fb = kFineBits;
  while (fb > kFineBitsMin && (1u << (kFineBits - fb)) < parts) --fb;
  const uint32_t NC = B >> fb, NR = B >> rb;
  const uint32_t G = cdiv(wide ? NR : B, 256);  // a power of two
  if (parts > 1 && NR != 256u * G) return PLK_E_DEVICE;  // the part offset's Horner seed below
  const uint32_t nbits = 8 + (uint32_t)__builtin_ctz(G);  // T_0..T_7 of u, one per bit of g
  const uint32_t nout = nbits + (wide ? 2u : 0u);         // + sum_r T_r, sum_r Y_r
  const uint32_t slots = (uint32_t)count;
  // chunk so that the accumulation grid holds ~2 waves of the chip's resident threads. Wide
  // sets in a batch have few entries per bucket and enough tasks anyway: one task per bucket.
  // A lone wide MSM below ~2^18 points (configs[2]-style commits at 2^16) would leave one
  // task of ~15-35 dependent additions per bucket on a half-empty chip: it takes the chunk
  // formula too (16 at 2^16, 52 at 2^20)
  const bool small_batch = !wide && B <= kSortSmallMax && max_len <= kSortOneMax;
  // the task-length floor: kChunkSmall for small batches when the workspace was sized for it
  const uint32_t chunk_floor = small_batch ? std::max(kChunkSmall, w.cap_chunk_min) : kChunkMin;
  const uint32_t chunk_fit = (uint32_t)std::min<size_t>(
      kChunkMax, std::max<size_t>(chunk_floor, total_entries / parts / PLK_CHUNK_TARGET));
  const uint32_t chunk = wide && count > 1 ? kChunkMax : chunk_fit;
  const size_t max_tasks_used = (size_t)s->windows * max_len / chunk + B;
  if (max_tasks_used + 1 > w.task_stride) return PLK_E_DEVICE;  // sizing invariant (ws_reserve)
  // 256 workgroups per slot: fewer give longer per-bucket write runs in k_scatter but lose
  // more parallelism than they gain (measured 2.77 / 2.79 / 3.02 / 4.52 ms per proof at
  // 256 / 128 / 64 / 32, tools/gpu_hist_sweep.sh)
  const uint32_t hist_blocks =
      std::max<uint32_t>(1, std::min<uint32_t>(kHistBlocksMax, cdiv(max_len, 512)));

  ReadbackHeader* hdr_dev = static_cast<ReadbackHeader*>(w.out_dev);
  G1xyzz* bits_dev = reinterpret_cast<G1xyzz*>(hdr_dev + 1);
  if (++w.gen == 0xFFFFFFFFu) {  // wrap: clear the stamps once every 2^32 - 1 batches
    std::memset(w.host_out.ptr, 0, sizeof(ReadbackHeader));
    w.gen = 1;
  }
  const uint32_t gen = w.gen;
  // small batches: the whole sort (and the degree check) in one dispatch per batch
  // (the chunk floor stays small_batch's: more scalars than kSortOneMax keep kChunkMin tasks).
  // Round 5: up to kSortOneBig scalars too (the 2^14-size commits at c = 13) instead of
  // k_hist + k_sort_small + k_scatter: 2^14 proofs 16.77 -> 17.33 M, 2^13 / 2^12 within noise
  // (profiles/r05_sort_one_big_c13_ab.jsonl; round 4's single-workgroup form at c = 15 did
  // not pay, profiles/r04_sort_one_big_ab.jsonl)
  const bool sort_one = small_batch || (!wide && B <= kSortSmallMax && max_len <= kSortOneBig);
  const bool hold = max_len <= kSortOneMax;
  if (max_tail && !sort_one) {
    hipLaunchKernelGGL(k_any_nonzero, dim3(cdiv(max_tail, 256), slots), dim3(256), 0, stream,
                       batch, hdr_dev->flag, gen);
  }
  if (wide) {
    if (max_len) {
      PLK_BY_C(s->c, hipLaunchKernelGGL(k_chist<CC>, dim3(hist_blocks, slots), dim3(kHistThreads), 0,
                                        stream, batch, cfg, NC, fb, w.blockhist.as<uint32_t>()))
    } else {
      PLK_HIP_TRY(hipMemsetAsync(w.blockhist.ptr, 0, (size_t)slots * hist_blocks * NC * 4, stream));
    }
    hipLaunchKernelGGL(k_block_scan, dim3(cdiv(NC, 256), slots), dim3(256), 0, stream,
                       w.blockhist.as<uint32_t>(), hist_blocks, NC, w.counts.as<uint32_t>(),
                       w.len_cur.as<uint32_t>(), w.len_fill.as<uint32_t>());
    PLK_BY_C(s->c, hipLaunchKernelGGL(k_cscatter<CC>, dim3(hist_blocks, slots), dim3(kHistThreads),
                                      0, stream, batch, cfg, NC, fb, (uint64_t)s->n,
                                      (const uint32_t*)w.counts.as<uint32_t>(),
                                      (const uint32_t*)w.blockhist.as<uint32_t>(),
                                      w.coarse_off.as<uint32_t>(), w.tmp.as<uint2>(),
                                      (uint64_t)(w.sorted_stride - 1)))
#define PLK_FINE_LAUNCH(FB)                                                                       \
  do {                                                                                            \
    hipLaunchKernelGGL(k_fine<FB>, dim3(NC, slots), dim3(1u << FB), 0, stream, B, NC, chunk,      \
                       (const uint32_t*)w.coarse_off.as<uint32_t>(), (const uint2*)w.tmp.as<uint2>(), \
                       (uint64_t)(w.sorted_stride - 1), w.sorted.as<uint32_t>(),                  \
                       (uint64_t)w.sorted_stride, w.offsets.as<uint32_t>(),                       \
                       w.task_rel.as<uint32_t>(), w.full_off.as<uint32_t>(),                      \
                       w.bin_tot.as<uint32_t>(), w.len_cur.as<uint32_t>());                       \
    hipLaunchKernelGGL(k_make_tasks_wide<FB>, dim3(NC, slots), dim3(1u << FB), 0, stream, B, NC,  \
                       chunk, (const uint32_t*)w.offsets.as<uint32_t>(),                          \
                       (const uint32_t*)w.task_rel.as<uint32_t>(),                                \
                       (const uint32_t*)w.full_off.as<uint32_t>(),                                \
                       (const uint32_t*)w.bin_tot.as<uint32_t>(),                                 \
                       (const uint32_t*)w.len_cur.as<uint32_t>(), w.len_fill.as<uint32_t>(),      \
                       w.task_off.as<uint32_t>(), w.tasks.as<uint2>(), (uint64_t)w.task_stride);  \
  } while (0)
    if (fb == 10) PLK_FINE_LAUNCH(10);
    else if (fb == 9) PLK_FINE_LAUNCH(9);
    else PLK_FINE_LAUNCH(8);
#undef PLK_FINE_LAUNCH
  } else if (sort_one) {
#define PLK_SORT_ONE_LAUNCH(HOLD)                                                                  \
  PLK_BY_C(s->c, hipLaunchKernelGGL((k_sort_one<CC, HOLD>), dim3(std::min(kSortOneParts, B), slots), \
                                    dim3(1024), 0, stream, batch, cfg, (uint64_t)s->n, chunk,        \
                                    w.sorted.as<uint32_t>(), (uint64_t)w.sorted_stride,              \
                                    w.offsets.as<uint32_t>(), w.task_off.as<uint32_t>(),             \
                                    w.tasks.as<uint2>(), (uint64_t)w.task_stride, hdr_dev->flag, gen))
    if (hold) {
      PLK_SORT_ONE_LAUNCH(true);
    } else {
      PLK_SORT_ONE_LAUNCH(false);
    }
#undef PLK_SORT_ONE_LAUNCH
  } else {
    const size_t lds = (size_t)std::min<uint32_t>(B, kLdsBuckets) * 4;
    if (max_len) {
      PLK_BY_C(s->c, hipLaunchKernelGGL(k_hist<CC>, dim3(hist_blocks, slots), dim3(kHistThreads), lds,
                                        stream, batch, cfg, w.blockhist.as<uint32_t>()))
    } else {
      PLK_HIP_TRY(hipMemsetAsync(w.blockhist.ptr, 0, (size_t)slots * hist_blocks * B * 4, stream));
    }
    const bool small_sort = B <= kSortSmallMax;
    if (small_sort) {
      hipLaunchKernelGGL(k_sort_small, dim3(1, slots), dim3(1024), 0, stream,
                         w.blockhist.as<uint32_t>(), hist_blocks, B, chunk, w.offsets.as<uint32_t>(),
                         w.task_off.as<uint32_t>(), w.tasks.as<uint2>(), (uint64_t)w.task_stride);
    } else {
      hipLaunchKernelGGL(k_block_scan, dim3(cdiv(B, 256), slots), dim3(256), 0, stream,
                         w.blockhist.as<uint32_t>(), hist_blocks, B, w.counts.as<uint32_t>(),
                         (uint32_t*)nullptr, (uint32_t*)nullptr);
      hipLaunchKernelGGL(k_scan_buckets, dim3(1, slots), dim3(1024), (size_t)B * 4, stream,
                         w.counts.as<uint32_t>(), B, chunk, w.offsets.as<uint32_t>(),
                         w.task_off.as<uint32_t>(), w.full_off.as<uint32_t>(),
                         w.len_cur.as<uint32_t>());
    }
    if (max_len) {
      PLK_BY_C(s->c, hipLaunchKernelGGL(k_scatter<CC>, dim3(hist_blocks, slots), dim3(kHistThreads),
                                        lds, stream, batch, cfg, (uint64_t)s->n,
                                        w.offsets.as<uint32_t>(), w.blockhist.as<uint32_t>(),
                                        w.sorted.as<uint32_t>(), (uint64_t)w.sorted_stride))
    }
    if (!small_sort) {
      hipLaunchKernelGGL(k_make_tasks, dim3(cdiv(B, 256), slots), dim3(256), 0, stream,
                         w.offsets.as<uint32_t>(), w.task_off.as<uint32_t>(),
                         w.full_off.as<uint32_t>(), w.len_cur.as<uint32_t>(), B, chunk,
                         w.tasks.as<uint2>(), (uint64_t)w.task_stride);
    }
  }
  // 0: single-lane trees, 1: quad trees, 2: quad k_bitsum2 only (its few workgroups are
  // latency-bound at any load); chosen when the workspace is made (msm_common.hpp)
  const int tail = w.tail_quad;
  const bool quad = tail == 1;
  // start / stop events stamped by the dispatch itself (its execution, as rocprofv3 times
  // it), not by the stream: with several lanes on the GPU a stream event would also count
  // the time the kernel waits behind other lanes' kernels
  launch_accumulate(s->has_inf, !w.shared_chip, dim3(cdiv(max_tasks_used, 256), slots), stream, w.ev0, w.ev1,
                    w.tasks.as<uint2>(), w.task_off.as<uint32_t>(), B, (uint64_t)w.task_stride,
                    w.sorted.as<uint32_t>(), (uint64_t)w.sorted_stride, s->table.as<G1Affine>(),
                    s->table_inf.as<uint8_t>(), w.partials.as<G1xyzz>());
  if (wide) {
    hipLaunchKernelGGL(k_runsum1, dim3(cdiv(NR, 256), slots), dim3(256), 0, stream,
                       (const uint32_t*)w.task_off.as<uint32_t>(), B, rb, (uint64_t)w.task_stride,
                       (const G1xyzz*)w.partials.as<G1xyzz>(), w.rsum.as<G1xyzz>());
    hipLaunchKernelGGL(k_runsum2, dim3(cdiv(NR, 256), slots), dim3(256), 0, stream, B, rb,
                       (const G1xyzz*)w.rsum.as<G1xyzz>(), w.ys.as<G1xyzz>(), w.zs.as<G1xyzz>());
  } else {
    // lanes per bucket: until each lane adds ~PLK_LANE_PARTIALS partials (partials per bucket = entries /
    // chunk + 1 tail) or the grid holds 2^17 lanes (the tree levels cost a full addition
    // per lane, so an already full chip gains nothing from more lanes per bucket)
    const size_t per_bucket = cdiv(total_entries, (size_t)chunk * B * slots) + 1;
    uint32_t lp = 0;
    while (lp < 4 && ((size_t)PLK_LANE_PARTIALS << lp) < per_bucket && (((size_t)B * slots) << lp) < 131072) ++lp;
    if (quad) {
      hipLaunchKernelGGL(k_bucket_sum<true>, dim3(cdiv(((size_t)B << lp) * 4, 256), slots), dim3(256), 0, stream,
                         w.task_off.as<uint32_t>(), B, lp, (uint64_t)w.task_stride,
                         w.partials.as<G1xyzz>(), w.bsum.as<G1xyzz>());
    } else {
      hipLaunchKernelGGL(k_bucket_sum<false>, dim3(cdiv((size_t)B << lp, 256), slots), dim3(256), 0, stream,
                         w.task_off.as<uint32_t>(), B, lp, (uint64_t)w.task_stride,
                         w.partials.as<G1xyzz>(), w.bsum.as<G1xyzz>());
    }
  }
  BitsumFold fold{};  // k_bitsum2 folded into k_bitsum1 when the slots have few groups
  if (G <= kFoldMaxGroups) {
    fold.done = w.done.as<uint32_t>();
    fold.out2 = bits_dev;
    fold.offsets = w.offsets.as<uint32_t>();
    fold.entries = hdr_dev->entries;
    fold.B = B;
    fold.nbits = nbits;
    fold.nout = nout;
  }
  if (quad) bitsum_launch<true, true>(wide, G, slots, NR, B, w, fold, nbits, nout, bits_dev, hdr_dev, stream);
  else if (tail == 2) bitsum_launch<false, true>(wide, G, slots, NR, B, w, fold, nbits, nout, bits_dev, hdr_dev, stream);
  else bitsum_launch<false, false>(wide, G, slots, NR, B, w, fold, nbits, nout, bits_dev, hdr_dev, stream);
  PLK_HIP_TRY(hipGetLastError());

  // the readback record (flags, entry counts, then the slots' bit sums) is in host memory
  // once the batch's kernels have completed
  const ReadbackHeader* hdr = w.host_out.as<ReadbackHeader>();
  const G1xyzz* T = reinterpret_cast<const G1xyzz*>(hdr + 1);
  PLK_HIP_TRY(stream_wait(stream));
  const uint32_t* ent = hdr->entries;
  uint32_t flag[kMaxSlots];
  for (uint32_t k = 0; k < slots; ++k) flag[k] = hdr->flag[k] == gen ? 1u : 0u;
  MsmStats& stt = w.stats;
  float ms = 0.f;
  if (hipEventElapsedTime(&ms, w.ev0, w.ev1) == hipSuccess) stt.last_accumulate_ms = ms;
  stt.last_point_adds = 0;
  for (uint32_t k = 0; k < slots; ++k) stt.last_point_adds += ent[k];
  stt.last_slots = slots;
  stt.cum_accumulate_ms += stt.last_accumulate_ms;
  stt.cum_launches += 1;
  stt.cum_point_adds += stt.last_point_adds;
  for (uint32_t k = 0; k < slots; ++k) stt.cum_points += batch.len[k];

  int overall = PLK_OK;
  for (uint32_t k = 0; k < slots; ++k) {
    plk_g1* out = &outs[k];
    if (flag[k]) {
      *out = plk_g1{};
      if (statuses) statuses[k] = PLK_E_DEGREE;
      if (overall == PLK_OK) overall = PLK_E_DEGREE;
      continue;
    }
    // host tail: sum_j 2^j T_j (Horner), then canonical affine. The device stages work in
    // the R' domain (ffr.hpp) with values in [0, 2p): reduce and map back to R first.
    G1xyzz acc = xyzz_infinity();
    // a part (b_lo = part B = part NR K, NR = 2^nbits runs): its buckets weigh b_lo + 1 + b',
    // i.e. + b_lo sum_b S_b = K 2^nbits part sum_r Y_r — part sum_r Y_r seeds the Horner
    // below, whose nbits doublings and the K below scale it
    if (wide && part) {
      const G1xyzz ysum = rx_to_r_domain(T[(size_t)k * nout + nbits + 1]);
      for (int i = 31 - __builtin_clz(part); i >= 0; --i) {
        acc = xyzz_dbl(acc);
        if ((part >> i) & 1u) acc = xyzz_add(acc, ysum);
      }
    }
    for (int j = (int)nbits - 1; j >= 0; --j) {
      acc = xyzz_dbl(acc);
      acc = xyzz_add(acc, rx_to_r_domain(T[(size_t)k * nout + j]));
    }
    if (wide) {  // over the runs: K (sum_r (r + 1) Y_r - sum_r Y_r) + sum_r T_r (k_runsum2)
      G1xyzz a = rx_to_r_domain(T[(size_t)k * nout + nbits + 1]);
      a.Y = fe_neg(a.Y);
      acc = xyzz_add(acc, a);
      for (uint32_t i = 0; i < rb; ++i) acc = xyzz_dbl(acc);
      acc = xyzz_add(acc, rx_to_r_domain(T[(size_t)k * nout + nbits]));
    }
    Fp x, y;
    const bool fin = xyzz_to_affine(acc, x, y);
    for (int i = 0; i < 6; ++i) {
      out->x[i] = (uint64_t)x.v[2 * i] | ((uint64_t)x.v[2 * i + 1] << 32);
      out->y[i] = (uint64_t)y.v[2 * i] | ((uint64_t)y.v[2 * i + 1] << 32);
    }
    out->infinity = fin ? 0 : 1;
    if (statuses) statuses[k] = PLK_OK;
  }
  return overall;
}

int msm_run(plk_srs* s, const Fr* d_scalars, size_t len, size_t check_len, plk_g1* out,
            hipStream_t stream) {
  return msm_run_batch(s, *s->ws, &d_scalars, &len, &check_len, 1, out, nullptr, stream);
}

MsmWorkspace* msm_workspace_new() { return new MsmWorkspace(); }
void msm_workspace_delete(MsmWorkspace* w) { delete w; }
const MsmStats& msm_workspace_stats(const MsmWorkspace& w) { return w.stats; }
MsmStats& msm_workspace_stats(MsmWorkspace& w) { return w.stats; }

}  // namespace plk

plk_srs::plk_srs() = default;
plk_srs::~plk_srs() = default;
