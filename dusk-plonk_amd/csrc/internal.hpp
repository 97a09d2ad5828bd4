// internal.hpp — shared runtime objects behind the C ABI (include/plk.h).
#pragma once
#include <hip/hip_runtime.h>

#include <map>
#include <memory>
#include <mutex>
#include <vector>

#include "../../include/plk.h"
#include "ff.hpp"
#include "g1.hpp"

namespace plk {

#define PLK_HIP_TRY(expr)                                        \
  do {                                                           \
    hipError_t _e = (expr);                                      \
    if (_e != hipSuccess) {                                      \
      last_hip_error() = _e;                                     \
      return (_e == hipErrorOutOfMemory) ? PLK_E_OOM : PLK_E_DEVICE; \
    }                                                            \
  } while (0)

hipError_t& last_hip_error();

// Device buffer owned by a context object.
struct DevBuf {
  void* ptr = nullptr;
  size_t bytes = 0;
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  DevBuf(DevBuf&& o) noexcept : ptr(o.ptr), bytes(o.bytes) {
    o.ptr = nullptr;
    o.bytes = 0;
  }
  DevBuf& operator=(DevBuf&& o) noexcept {
    if (this != &o) {
      if (ptr) (void)hipFree(ptr);
      ptr = o.ptr;
      bytes = o.bytes;
      o.ptr = nullptr;
      o.bytes = 0;
    }
    return *this;
  }
  ~DevBuf() {
    if (ptr) (void)hipFree(ptr);
  }
  int alloc(size_t b) {
    if (ptr && bytes >= b) return PLK_OK;
    if (ptr) (void)hipFree(ptr);
    ptr = nullptr;
    bytes = 0;
    if (b == 0) return PLK_OK;
    hipError_t e = hipMalloc(&ptr, b);
    if (e != hipSuccess) {
      ptr = nullptr;
      last_hip_error() = e;
      return e == hipErrorOutOfMemory ? PLK_E_OOM : PLK_E_DEVICE;
    }
    bytes = b;
    return PLK_OK;
  }
  template <class T>
  T* as() const {
    return reinterpret_cast<T*>(ptr);
  }
};

struct NttPass {
  uint32_t lp, lr, lt;  // log2 of: sub-transform length so far, radix, columns per block
};

}  // namespace plk

struct plk_domain {
  plk_ctx* ctx = nullptr;
  uint32_t log_n = 0;
  uint64_t n = 0;
  plk::Fr omega, omega_inv, n_inv, g, g_inv;  // Montgomery form (host copies)
  plk::DevBuf tw_fwd;        // w^e, e < n (R domain: the domain elements)
  plk::DevBuf tw_fwd_rx;     // w^e, R' domain (ffr.hpp), read by the NTT passes
  plk::DevBuf tw_inv;        // w^-e, e < n (R' domain)
  plk::DevBuf coset_pow;     // g^e, e < n (R' domain)
  plk::DevBuf icoset_scale;  // n^-1 * g^-e, e < n (R' domain)
  std::vector<plk::DevBuf> pass_tw_fwd, pass_tw_inv;  // per pass q > 0: w_{Rp}^{jk} [j][k] (R')
  // the inverse direction's last pass table times n^-1: a plain idft's scaling rides on the
  // inter-pass twiddle instead of a product per output (multi-pass plans only)
  plk::DevBuf pass_tw_inv_last;
  plk::DevBuf scratch;       // 2n elements (default scratch for plk_ntt_dev)
  plk::DevBuf io;            // n elements (host-buffer entry points stage through it)
  std::vector<plk::NttPass> plan;
  uint32_t le = 10;          // log2 elements per workgroup
};

namespace plk {
struct MsmWorkspace;
// Bucket-accumulation statistics of one MSM workspace (measurement only): the most recent
// batch and the cumulative figures since the last reset — k_accumulate time from
// dispatch-stamped events, launches, point additions and MSM points (scalar counts).
struct MsmStats {
  float last_accumulate_ms = 0.f;
  uint64_t last_point_adds = 0;
  uint32_t last_slots = 0;
  double cum_accumulate_ms = 0.0;
  uint64_t cum_launches = 0, cum_point_adds = 0, cum_points = 0;
  void reset_cum() {
    cum_accumulate_ms = 0.0;
    cum_launches = cum_point_adds = cum_points = 0;
  }
};
}

struct plk_srs {
  plk_ctx* ctx = nullptr;
  size_t n = 0;              // number of SRS points
  uint32_t c = 16;           // window bits
  uint32_t windows = 16;     // ceil(256 / c)
  // balanced windows (round 5): when c does not divide 255, the top `narrow` windows are
  // c - 1 bits wide (narrow = c W - 255) and their digits come scaled by 2, their table rows
  // pre-divided by 2 (msm_prepare_srs, msm.hip digit_at): every window spreads over the whole
  // bucket range, without the short top window whose few digit values piled extra entries
  // onto a few hot buckets
  uint32_t narrow = 0;
  plk::DevBuf points;        // affine, plk::G1Affine (96 B), n entries; inf flags separate
  plk::DevBuf inf;           // uint8 per point
  plk::DevBuf table;         // precomputed 2^(c*w) * P_i, affine, windows * n entries
  plk::DevBuf table_inf;     // uint8, windows * n
  bool has_inf = false;      // any point at infinity in the SRS (slow-path flag checks)
  plk::DevBuf staging;       // host-scalar entry points stage through it
  // the workspace of the SRS's own entry points (plk_msm / plk_commit*: one thread at a
  // time); concurrent provers sharing this SRS each bring their own (plk_prover)
  std::unique_ptr<plk::MsmWorkspace> ws;
  plk_srs();
  ~plk_srs();
};

struct plk_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  std::map<uint32_t, std::unique_ptr<plk_domain>> domains;
  std::mutex mu;
};

namespace plk {
// Page-locked host buffer: the prover's host<->device transfers go through these. A
// pageable hipMemcpy pins and unpins its pages on every call, and the page-table and
// TLB-shootdown work that comes with it slowed a concurrent composer synthesis ~1.6x.
struct PinnedBuf {
  void* ptr = nullptr;
  size_t bytes = 0;
  PinnedBuf() = default;
  PinnedBuf(const PinnedBuf&) = delete;
  PinnedBuf& operator=(const PinnedBuf&) = delete;
  ~PinnedBuf() {
    if (ptr) (void)hipHostFree(ptr);
  }
  int alloc(size_t b, unsigned flags = hipHostMallocDefault) {
    if (ptr && bytes >= b) return PLK_OK;
    if (ptr) (void)hipHostFree(ptr);
    ptr = nullptr;
    bytes = 0;
    if (b == 0) return PLK_OK;
    const hipError_t e = hipHostMalloc(&ptr, b, flags);
    if (e != hipSuccess) {
      ptr = nullptr;
      last_hip_error() = e;
      return e == hipErrorOutOfMemory ? PLK_E_OOM : PLK_E_DEVICE;
    }
    bytes = b;
    return PLK_OK;
  }
  template <class T>
  T* as() const {
    return static_cast<T*>(ptr);
  }
};

// Host wait for all work queued on `s`, blocking in the driver instead of spinning: the
// prover's host thread waits at every commitment, and a spinning wait steals the core a
// concurrent composer synthesis (or any other host work) runs on. One event per thread.
inline hipError_t stream_wait(hipStream_t s) {
  thread_local hipEvent_t ev = nullptr;
  if (!ev) {
    const hipError_t e = hipEventCreateWithFlags(&ev, hipEventBlockingSync | hipEventDisableTiming);
    if (e != hipSuccess) return e;
  }
  const hipError_t e = hipEventRecord(ev, s);
  if (e != hipSuccess) return e;
  return hipEventSynchronize(ev);
}

// RAII device guard
struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    (void)hipGetDevice(&prev);
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    int cur = -1;
    (void)hipGetDevice(&cur);
    if (prev >= 0 && cur != prev) (void)hipSetDevice(prev);
  }
};

int ntt_build_domain(plk_domain* d);
// Per-launch strides of a batch of `count` transforms (vector v: in + v * in_stride, out + v *
// out_stride, pre-scale table pre + v * pre_stride, post-scale table post + v * post_stride;
// a stride of 0 shares one input / table between the vectors). pre / post: R'-domain tables
// replacing the domain's g^j (forward coset) / n^-1 g^-j (inverse coset) tables.
struct NttBatch {
  uint64_t in_stride = 0, out_stride = 0;
  const Fr* pre = nullptr;
  uint64_t pre_stride = 0;
  const Fr* post = nullptr;
  uint64_t post_stride = 0;
  // group > 0: vector v = g * group + m reads in + g * in_group_stride + m * in_stride and its
  // pre / post tables at m * pre_stride / m * post_stride (several polynomials' coset blocks in
  // one launch); outputs stay at v * out_stride
  uint32_t group = 0;
  uint64_t in_group_stride = 0;
};
struct NttStrides {  // kernel-side view
  uint64_t in, out, pre, post, in_group;
  uint32_t group_in, group_post;  // grouping of the first pass' inputs / the last pass' post table
};
int ntt_run_batch(plk_domain* d, const Fr* in, Fr* out, size_t len_in, int dir, int coset,
                  Fr* scratch, hipStream_t stream, uint32_t count, const NttBatch& b);
// pre_table (forward coset transforms only): R'-domain multipliers for the len_in inputs
// in place of the domain's g^j table — a scaled table (c g^j) yields the evaluations of c p
int ntt_run(plk_domain* d, const Fr* in, Fr* out, size_t len_in, int dir, int coset,
            Fr* scratch, hipStream_t stream, uint32_t count, const Fr* pre_table = nullptr);
int msm_prepare_srs(plk_srs* s, hipStream_t stream);
int msm_run(plk_srs* s, const Fr* d_scalars, size_t len, size_t check_len, plk_g1* out,
            hipStream_t stream);
// The SRS (window table) is only read: any number of threads may run batches on one SRS
// concurrently, each with its own workspace `w` and stream.
// part / parts (parts a power of two, 1 = the whole MSM): only the buckets of the part's
// range [part, part + 1) * 2^(c-1) / parts (wide bucket sets, 2^(c-1) / parts >= 2^14); the
// parts' outputs sum to the whole MSM's (one large MSM split over GPUs by bucket
// range, each GPU's reduction over its own buckets only).
int msm_run_batch(plk_srs* s, MsmWorkspace& w, const Fr* const* d_scalars, const size_t* lens,
                  const size_t* check_lens, size_t count, plk_g1* outs, int* statuses,
                  hipStream_t stream, uint32_t part = 0, uint32_t parts = 1);
// whether msm_run_batch accepts `parts` bucket ranges on this SRS (a power of two; for
// parts > 1 a wide bucket set, 2^(c-1) above the LDS histogram's range, and >= 2^14 buckets
// per part)
bool msm_parts_ok(const plk_srs* s, uint32_t parts);
MsmWorkspace* msm_workspace_new();
void msm_workspace_delete(MsmWorkspace* w);
const MsmStats& msm_workspace_stats(const MsmWorkspace& w);
MsmStats& msm_workspace_stats(MsmWorkspace& w);
void fr_root_of_unity(uint32_t log_n, Fr& omega);
int ntt_vanishing(plk_domain* d, uint64_t deg, Fr* d_out, hipStream_t s);
// out[e] = base^e * scale, e < n (R domain; to_rx: converted to the R' domain)
int ntt_power_table(Fr* out, const Fr& base, const Fr& scale, uint64_t n, bool to_rx,
                    hipStream_t s);
int srs_generate(plk_srs* s, const Fr& tau_mont, uint64_t start, hipStream_t stream);
}  // namespace plk
