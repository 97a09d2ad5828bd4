// msm_acc.hip — the MSM's bucket accumulation (k_accumulate), the dominant kernel of a
// proof (≈ 56 % of a 2^20 proof's GPU time). Its own translation unit: msm.hip's sort and
// reduction kernels take minutes to compile, and this kernel is the one tuned most often.
//
// One thread per task of <= 64 same-bucket entries of the sorted digit list (full tasks
// first, tails grouped by length, longest first: the lanes of a wave finish together),
// XYZZ mixed additions in the redundant Fp form (g1r.hpp g1r_madd_lazy_sl), the partial
// written packed. Replaces the bucket accumulation of msm_curve_addition inside zksnarks
// PlonkParams::commit (called at prover.rs:133-136,194,262-265,440,452).
//
// The next entry's point is loaded one addition ahead (round 5): through LDS-DMA (global_load_lds_dwordx4: 6 per 96-B point, no VGPR destination) into a per-wave
// staging slot [6][64] x 16 B (6 KiB per wave), read back with ds_read_b128 when its
// addition starts. The register prefetch of rounds 1-4 held the packed
// point (24 VGPRs) live through the ~4 900-instruction addition: 208 -> 190 VGPRs (grouped
// products), 173 -> 164 (plain chains, which then fit 3 waves per SIMD without spills), and
// 438 instead of 547 s_nop per addition. Measured (round 5, one box, interleaved, A/B against
// the round-4 register prefetch): solo additions/s in the 2^20 proof 5.84-5.87e9 -> 6.83-6.90e9,
// 2^20 proofs 29.7-30.1 -> 31.6 M constraints/s, lone 2^20 MSM 3.08-3.11 -> 2.92 ms (2.84 in the
// LONE form).
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include "internal.hpp"
#include "msm_common.hpp"
#include "g1r.hpp"


namespace plk {

namespace {

constexpr uint32_t kAccThreads = 256;

typedef __attribute__((address_space(3))) void lds_void;

// Issue the 6 LDS-DMA loads of one affine point (96 B) into this wave's staging slot:
// piece i of lane l lands at stage[i][l] (the destination is the wave-uniform base of
// row i plus lane x 16 B).
__device__ __forceinline__ void stage_point(const G1Affine* p, uint4 (*stage)[64]) {
  const uint4* q = reinterpret_cast<const uint4*>(p);
#pragma unroll
  for (int i = 0; i < 6; ++i)
    __builtin_amdgcn_global_load_lds((const void*)(q + i), (lds_void*)&stage[i][0], 16, 0, 0);
}

__device__ __forceinline__ void unstage_point(const uint4 (*stage)[64], uint32_t lane, RFp& x,
                                              RFp& y) {
  Fp px, py;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const uint4 a = stage[i][lane], b = stage[i + 3][lane];
    px.v[4 * i] = a.x; px.v[4 * i + 1] = a.y; px.v[4 * i + 2] = a.z; px.v[4 * i + 3] = a.w;
    py.v[4 * i] = b.x; py.v[4 * i + 1] = b.y; py.v[4 * i + 2] = b.z; py.v[4 * i + 3] = b.w;
  }
  x = rx_unpack(px);
  y = rx_unpack(py);
}

// LONE: the form for a chip the MSM has to itself (lone commits, plk_prove's default
// prover): at 3 waves per SIMD, product PAIRS (168 VGPRs, no spill); otherwise (prover lanes,
// several proofs sharing the chip) the interleaved groups with the (Y3, ZZ3, ZZZ3) triple at 2
// (g1r.hpp g1r_madd_lazy_sl; round 5 A/B, profiles/r05_acc_dma_ab.jsonl). Both with the group
// columns as single asm statements (round 6). The lone form was plain product chains until
// then (4 648 instructions and 311 64-bit merge adds per loop iteration against 4 500 / 114 for
// the asm pairs; lone 2^20 MSM 2.81 -> 2.80 ms, 7.42 -> 7.51e9 solo additions/s over four
// interleaved runs, profiles/r06_lone_asm_pairs_ab.jsonl; the lanes on this form at 3 waves
// measured no better than the triple at 2).
template <bool HAS_INF, bool LONE>
__global__ void __launch_bounds__(kAccThreads)
    __attribute__((amdgpu_waves_per_eu(LONE ? 3 : 2, LONE ? 3 : 2)))
    k_accumulate(const uint2* __restrict__ tasks, const uint32_t* __restrict__ task_off, uint32_t B,
                 uint64_t task_stride, const uint32_t* __restrict__ sorted, uint64_t sorted_stride,
                 const G1Affine* __restrict__ table, const uint8_t* __restrict__ table_inf,
                 G1xyzz* __restrict__ partials) {
  const uint32_t slot = blockIdx.y;
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  __shared__ uint4 s_stage[kAccThreads / 64][6][64];
  uint4 (*stage)[64] = s_stage[threadIdx.x >> 6];
  const uint32_t lane = threadIdx.x & 63;
  if (t >= task_off[(size_t)slot * (B + 1) + B]) return;
  const uint2 tk = tasks[(size_t)slot * task_stride + t];
  const uint2 task = make_uint2(tk.x, (tk.y >> kTaskShift) + 1);  // first entry, length (>= 1)
  const uint32_t pidx = tk.y & ((1u << kTaskShift) - 1);
  sorted += (size_t)slot * sorted_stride;
  // The first entry initialises the accumulator; exceptional additions (accumulator at
  // infinity, equal x) show up as ZZ3 == 0 after the straight-line formula and are
  // finished with the point reloaded (g1r.hpp).
  const uint32_t end = task.x + task.y;
  G1R acc = g1r_infinity();
  {
    const uint32_t c0 = sorted[task.x];
    if (!HAS_INF || !table_inf[c0 & 0x7fffffffu]) {
      ld_g1r_aff(&table[c0 & 0x7fffffffu], acc.X, acc.Y);
      if (c0 & 0x80000000u) acc.Y = rx_neg(acc.Y);
      acc.ZZ = rx_one<FpCfg>();
      acc.ZZZ = rx_one<FpCfg>();
    }
  }
  // entry e's point is in the staging slot when its iteration starts (the compiler waits
  // for the DMA, vmcnt, before the ds_reads); `code` is entry e's index, `next` entry
  // e + 1's, loaded one addition ahead like the point itself; the infinity flag travels
  // with the index so that no ordinary load result is consumed while a DMA is in flight
  // (hipcc would wait vmcnt(0) there and drain it)
  uint32_t code = task.x + 1 < end ? sorted[task.x + 1] : 0u;
  bool inf = HAS_INF && task.x + 1 < end && table_inf[code & 0x7fffffffu];
  if (task.x + 1 < end) stage_point(&table[code & 0x7fffffffu], stage);
  uint32_t next = task.x + 2 < end ? sorted[task.x + 2] : 0u;
  for (uint32_t e = task.x + 1; e < end; ++e) {
    const uint32_t cur = code;
    const bool cur_inf = inf;
    RFp x, y;
    unstage_point(stage, lane, x, y);
    // the ds_reads have returned (their values are unpacked) before the slot is refilled
    __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (e + 1 < end) {
      code = next;
      if (HAS_INF) inf = table_inf[code & 0x7fffffffu];
      stage_point(&table[code & 0x7fffffffu], stage);
      if (e + 2 < end) next = sorted[e + 2];
    }
    if (HAS_INF && cur_inf) continue;
    if (cur & 0x80000000u) y = rx_neg_lazy(y);
    const bool was_inf = g1r_is_inf(acc);
    G1R r = g1r_madd_lazy_sl<true, true, LONE>(acc, x, y);
    if (rx_is_zero(r.ZZ)) {  // rare: reload the point rather than keep it live
      RFp xr, yr;
      ld_g1r_aff(&table[cur & 0x7fffffffu], xr, yr);
      if (cur & 0x80000000u) yr = rx_neg(yr);
      r = g1r_madd_lazy_fix(was_inf, r, xr, yr);
    }
    acc = r;
  }
  st_g1r(&partials[(size_t)slot * task_stride + pidx], g1r_lazy_finish(acc));
}

}  // namespace

void launch_accumulate(bool has_inf, bool lone, dim3 grid, hipStream_t stream, hipEvent_t ev0,
                       hipEvent_t ev1, const uint2* tasks, const uint32_t* task_off, uint32_t B,
                       uint64_t task_stride, const uint32_t* sorted, uint64_t sorted_stride,
                       const G1Affine* table, const uint8_t* table_inf, G1xyzz* partials) {
  const dim3 block(kAccThreads);
#define PLK_ACC_LAUNCH(I, L)                                                                   \
  hipExtLaunchKernelGGL((k_accumulate<I, L>), grid, block, 0, stream, ev0, ev1, 0, tasks, task_off, \
                        B, task_stride, sorted, sorted_stride, table, table_inf, partials)
  if (has_inf) {
    if (lone) PLK_ACC_LAUNCH(true, true);
    else PLK_ACC_LAUNCH(true, false);
  } else {
    if (lone) PLK_ACC_LAUNCH(false, true);
    else PLK_ACC_LAUNCH(false, false);
  }
#undef PLK_ACC_LAUNCH
}

}  // namespace plk
