// msm_common.hpp — device load/store helpers and the per-SRS MSM workspace.
#pragma once
#include <cstdlib>

#include "internal.hpp"

namespace plk {

#ifndef PLK_CHUNK_MAX
#define PLK_CHUNK_MAX 64
#endif
#ifndef PLK_CHUNK_MIN
#define PLK_CHUNK_MIN 16
#endif
constexpr uint32_t kChunkMin = PLK_CHUNK_MIN;  // points per accumulation task (bounds)
// small batches (the one-dispatch sort's: B <= 4 096, <= 8 192 scalars per slot) take tasks
// of down to 8 points: their latency-bound accumulation chains halve (round 4: 2^12 proofs
// +7 %; 8 everywhere cost the 2^14 / 2^16 proofs and the lone 2^16 MSM 1-3 %)
#ifndef PLK_CHUNK_SMALL
#define PLK_CHUNK_SMALL 8
#endif
constexpr uint32_t kChunkSmall = PLK_CHUNK_SMALL;
constexpr uint32_t kChunkMax = PLK_CHUNK_MAX;
// task record .y = partial index | (length - 1) << kTaskShift
constexpr uint32_t kTaskShift = 32 - (kChunkMax <= 64 ? 6 : 7);
static_assert(kChunkMax <= 128, "task length field");
constexpr uint32_t kBatchAff = 32;  // points per batch-inversion chunk
constexpr uint32_t kMaxSlots = 16;  // independent MSMs per batch

struct MsmCfg {
  uint32_t c, W, B;
  uint32_t narrow;  // plk_srs::narrow: the top `narrow` windows are c - 1 bits, digits x 2
  // bucket range of a part (msm_run_batch parts > 1: the wide-set sort keeps only digits of
  // buckets [b_lo, b_lo + B), renumbered from 0); b_lo = 0 for a whole MSM
  uint32_t b_lo;
};

// Kernel-argument view of one batch of independent MSMs (slot = blockIdx.y).
struct MsmBatch {
  const Fr* scalars[kMaxSlots];
  uint32_t len[kMaxSlots];
  uint64_t check_len[kMaxSlots];
};

__device__ __forceinline__ void ld_fp(const uint32_t* p, Fp& r) {
  const uint4* q = reinterpret_cast<const uint4*>(p);
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    uint4 a = q[i];
    r.v[4 * i] = a.x; r.v[4 * i + 1] = a.y; r.v[4 * i + 2] = a.z; r.v[4 * i + 3] = a.w;
  }
}

__device__ __forceinline__ void st_fp(uint32_t* p, const Fp& v) {
  uint4* q = reinterpret_cast<uint4*>(p);
#pragma unroll
  for (int i = 0; i < 3; ++i) q[i] = make_uint4(v.v[4 * i], v.v[4 * i + 1], v.v[4 * i + 2], v.v[4 * i + 3]);
}

__device__ __forceinline__ void ld_aff(const G1Affine* p, Fp& x, Fp& y) {
  ld_fp(reinterpret_cast<const uint32_t*>(p), x);
  ld_fp(reinterpret_cast<const uint32_t*>(p) + 12, y);
}

__device__ __forceinline__ void st_aff(G1Affine* p, const Fp& x, const Fp& y) {
  st_fp(reinterpret_cast<uint32_t*>(p), x);
  st_fp(reinterpret_cast<uint32_t*>(p) + 12, y);
}

__device__ __forceinline__ void ld_xyzz(const G1xyzz* p, G1xyzz& r) {
  const uint32_t* q = reinterpret_cast<const uint32_t*>(p);
  ld_fp(q, r.X); ld_fp(q + 12, r.Y); ld_fp(q + 24, r.ZZ); ld_fp(q + 36, r.ZZZ);
}

__device__ __forceinline__ void st_xyzz(G1xyzz* p, const G1xyzz& r) {
  uint32_t* q = reinterpret_cast<uint32_t*>(p);
  st_fp(q, r.X); st_fp(q + 12, r.Y); st_fp(q + 24, r.ZZ); st_fp(q + 36, r.ZZZ);
}

__device__ __forceinline__ Fr ld_fr(const Fr* p) {
  const uint4* q = reinterpret_cast<const uint4*>(p);
  uint4 a = q[0], b = q[1];
  Fr r;
  r.v[0] = a.x; r.v[1] = a.y; r.v[2] = a.z; r.v[3] = a.w;
  r.v[4] = b.x; r.v[5] = b.y; r.v[6] = b.z; r.v[7] = b.w;
  return r;
}


inline uint32_t cdiv(uint64_t a, uint64_t b) { return (uint32_t)((a + b - 1) / b); }

// Head of a batch's readback record (MsmWorkspace::host_out, written by the kernels straight
// into mapped host memory, the bit sums after it): per slot the degree-check flag (stamped
// with the batch's generation number by k_any_nonzero) and the entry count (point
// additions, written by k_bitsum2). 128 bytes, so the G1xyzz records after it stay aligned.
struct ReadbackHeader {
  uint32_t flag[kMaxSlots];
  uint32_t entries[kMaxSlots];
};
static_assert(sizeof(ReadbackHeader) % 16 == 0, "alignment of the bit sums");

struct MsmWorkspace {
  DevBuf counts, blockhist, offsets, task_off, full_off, len_cur, sorted, tasks, partials, bsum, bits1;
  // wide bucket sets only (msm.hip: two-level sort, run-sum reduction)
  DevBuf tmp, task_rel, bin_tot, len_fill, coarse_off, rsum, ys, zs;
  DevBuf done;  // k_bitsum1's per-slot arrival counters (its fold of k_bitsum2)
  // the readback record (ReadbackHeader + bit sums): coherent host memory mapped into the
  // device's address space, written by the kernels themselves (no copy dispatch per batch)
  PinnedBuf host_out;
  void* out_dev = nullptr;  // host_out's device address
  uint32_t gen = 0;    // generation number of the last batch (degree-check flag stamps)
  size_t cap_len = 0, task_stride = 0, sorted_stride = 0;
  uint32_t cap_slots = 0;
  // the SRS shape the buffers and strides were sized for: a workspace moves between SRSs
  // (a prover's key SRS, then a shard slice with another window size), and every size
  // above depends on c and the window count
  uint32_t cap_c = 0, cap_windows = 0;
  uint32_t cap_chunk_min = kChunkMin;  // the task-length floor the buffers were sized for
  // the bit-sum trees' additions: 1 quad-cooperative (g1r_add_quad, lower latency, the lone
  // call's choice), 0 one lane each (fewer issue slots per addition, for prover lanes that
  // share the chip with other proofs), 2 quads in k_bitsum2 only (lane_tail_policy).
  // PLK_TAIL_QUAD (experiments, tests) forces a form for every workspace created while it is
  // set: read once here, never per batch (a getenv in the hot path raced the tests' setenv)
  int tail_quad = 1;
  bool tail_forced = false;
  // the chip is shared with other proofs' kernels (prover lanes): k_accumulate's grouped form
  // at 2 waves per SIMD; otherwise (lone commits, plk_prove) the LONE form (msm_acc.hip)
  bool shared_chip = false;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  MsmStats stats;
  MsmWorkspace() {
    if (const char* e = getenv("PLK_TAIL_QUAD")) {
      const int v = atoi(e);
      if (v >= 0 && v <= 2) {
        tail_quad = v;
        tail_forced = true;
      }
    }
  }
  ~MsmWorkspace() {
    if (ev0) (void)hipEventDestroy(ev0);
    if (ev1) (void)hipEventDestroy(ev1);
  }
};

int ws_reserve(plk_srs* s, MsmWorkspace& w, size_t len, uint32_t slots, hipStream_t stream);

// The reduction trees' form for a prover lane of an n-row circuit (plk_prover_create; lone
// commits and plk_prove's default prover keep 1). A lane shares the chip with other lanes'
// proofs, so issue slots per addition count more than a tree level's latency, except where
// the reduction tails stay latency-bound. Measured, prover lanes at the bench's lane counts,
// interleaved on one box (constraints/s, 0 / 1 / 2):
//   2^12  7.61-7.80 / 8.26-8.65 / —          -> 1 (profiles/r04_tail_quad_ab.jsonl, r04p)
//   2^14  15.1-15.6 / 15.2-15.5 / +3 %        -> 2 (profiles/r04_tail_mode2_ab.jsonl,
//                                                   r04_tail_modes_small_ab.jsonl)
//   2^16  26.2-26.9 / 24.1-26.2 / -3 % vs 0   -> 0
//   2^20  32.5-32.7 / 32.1-32.3 / +0.6 % vs 0 -> 2
// and, round 5 (profiles/r05_small_and_tail_policy_ab.jsonl, two interleaved runs each):
//   2^15  21.2-21.4 / 20.3-20.9 / 21.3-21.5   -> 0 (2 within noise)
//   2^17  29.1-29.2 / 28.5-28.5 / 29.0-29.2   -> 0
//   2^18  29.6-29.8 / 29.0-29.2 / 29.5-29.6   -> 0
// 2^19 and up as 2^20. Re-measured after 2^13 / 2^14 moved to c = 12 / 13 (round 5,
// profiles/r05_tail_forms_new_c_ab.jsonl, three interleaved runs): 2^13 12.71 / 13.17 / 12.74 M
// -> 1 stays, 2^14 16.87 / 16.18 / 17.37 M -> 2 stays.
inline int lane_tail_policy(uint64_t n) {
  if (n <= (1ull << 13)) return 1;
  if (n == (1ull << 14)) return 2;
  if (n >= (1ull << 19)) return 2;
  return 0;
}

// k_accumulate (msm_acc.hip) over grid.x * 256 task lanes per slot (grid.y = slots), stamped
// with the start / stop events ev0 / ev1 by the dispatch itself
void launch_accumulate(bool has_inf, bool lone, dim3 grid, hipStream_t stream, hipEvent_t ev0,
                       hipEvent_t ev1, const uint2* tasks, const uint32_t* task_off, uint32_t B,
                       uint64_t task_stride, const uint32_t* sorted, uint64_t sorted_stride,
                       const G1Affine* table, const uint8_t* table_inf, G1xyzz* partials);

}  // namespace plk
