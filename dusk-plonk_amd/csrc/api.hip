// api.hip — the C ABI (include/plk.h): contexts, Fft domains, NTT entry points, SRS and
// KZG commit. Every entry point catches everything and returns a plk_status, so no C++
// exception or HIP abort crosses the boundary (the reference propagates commit errors
// with `?`, prover.rs:133-452, and treats NTT as infallible).
#include <hip/hip_runtime.h>

#include <cstring>
#include <algorithm>
#include <new>
#include <thread>
#include <vector>

#include "internal.hpp"
#include "msm_common.hpp"

using namespace plk;

namespace plk {
hipError_t& last_hip_error() {
  static thread_local hipError_t e = hipSuccess;
  return e;
}
}  // namespace plk

#define PLK_API_BEGIN try {
#define PLK_API_END                 \
  }                                 \
  catch (const std::bad_alloc&) {   \
    return PLK_E_OOM;               \
  }                                 \
  catch (...) {                     \
    return PLK_E_DEVICE;            \
  }

static inline void fr_to_abi(const Fr& a, plk_fr* out) {
  for (int i = 0; i < 4; ++i) out->l[i] = (uint64_t)a.v[2 * i] | ((uint64_t)a.v[2 * i + 1] << 32);
}

static inline Fr fr_from_abi(const plk_fr* a) {
  Fr r;
  for (int i = 0; i < 4; ++i) {
    r.v[2 * i] = (uint32_t)a->l[i];
    r.v[2 * i + 1] = (uint32_t)(a->l[i] >> 32);
  }
  return r;
}

extern "C" {

int plk_abi_version(void) { return PLK_ABI_VERSION; }

const char* plk_status_str(int s) {
  switch (s) {
    case PLK_OK: return "ok";
    case PLK_E_DEGREE: return "polynomial degree exceeds the SRS (commit)";
    case PLK_E_ARG: return "invalid argument";
    case PLK_E_DEVICE: return "HIP device error";
    case PLK_E_OOM: return "device out of memory";
    case PLK_E_NODEV: return "no GPU available";
    case PLK_E_UNSUPPORTED: return "unsupported feature";
    default: return "unknown status";
  }
}

int plk_device_count(int* out) {
  if (!out) return PLK_E_ARG;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
  *out = n;
  return PLK_OK;
}

int plk_ctx_create(int device, plk_ctx** out) {
  PLK_API_BEGIN
  if (!out) return PLK_E_ARG;
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return PLK_E_NODEV;
  if (device < 0 || device >= n) return PLK_E_ARG;
  DeviceGuard g(device);
  std::unique_ptr<plk_ctx> c(new plk_ctx());
  c->device = device;
  PLK_HIP_TRY(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
  *out = c.release();
  return PLK_OK;
  PLK_API_END
}

int plk_ctx_destroy(plk_ctx* ctx) {
  PLK_API_BEGIN
  if (!ctx) return PLK_E_ARG;
  {
    DeviceGuard g(ctx->device);
    (void)stream_wait(ctx->stream);
    ctx->domains.clear();
    (void)hipStreamDestroy(ctx->stream);
  }
  delete ctx;
  return PLK_OK;
  PLK_API_END
}

int plk_ctx_stream(plk_ctx* ctx, void** stream_out) {
  if (!ctx || !stream_out) return PLK_E_ARG;
  *stream_out = (void*)ctx->stream;
  return PLK_OK;
}

int plk_ctx_synchronize(plk_ctx* ctx) {
  PLK_API_BEGIN
  if (!ctx) return PLK_E_ARG;
  DeviceGuard g(ctx->device);
  PLK_HIP_TRY(stream_wait(ctx->stream));
  return PLK_OK;
  PLK_API_END
}

// ------------------------------------------------------------------------------ domains
int plk_domain_get(plk_ctx* ctx, uint32_t log_n, plk_domain** out) {
  PLK_API_BEGIN
  if (!ctx || !out || log_n > 27) return PLK_E_ARG;
  std::lock_guard<std::mutex> lk(ctx->mu);
  auto it = ctx->domains.find(log_n);
  if (it != ctx->domains.end()) {
    *out = it->second.get();
    return PLK_OK;
  }
  DeviceGuard g(ctx->device);
  std::unique_ptr<plk_domain> d(new plk_domain());
  d->ctx = ctx;
  d->log_n = log_n;
  d->n = 1ull << log_n;
  int st = ntt_build_domain(d.get());
  if (st) return st;
  *out = d.get();
  ctx->domains[log_n] = std::move(d);
  return PLK_OK;
  PLK_API_END
}

int plk_domain_info(const plk_domain* d, uint64_t* size, plk_fr* generator, plk_fr* generator_inv,
                    plk_fr* size_inv, plk_fr* coset, plk_fr* coset_inv) {
  if (!d) return PLK_E_ARG;
  if (size) *size = d->n;
  if (generator) fr_to_abi(d->omega, generator);
  if (generator_inv) fr_to_abi(d->omega_inv, generator_inv);
  if (size_inv) fr_to_abi(d->n_inv, size_inv);
  if (coset) fr_to_abi(d->g, coset);
  if (coset_inv) fr_to_abi(d->g_inv, coset_inv);
  return PLK_OK;
}

int plk_domain_elements(const plk_domain* d, plk_fr* out) {
  PLK_API_BEGIN
  if (!d || !out) return PLK_E_ARG;
  DeviceGuard g(d->ctx->device);
  PLK_HIP_TRY(hipMemcpyAsync(out, d->tw_fwd.ptr, d->n * sizeof(Fr), hipMemcpyDeviceToHost,
                             d->ctx->stream));
  PLK_HIP_TRY(stream_wait(d->ctx->stream));
  return PLK_OK;
  PLK_API_END
}

int plk_domain_vanishing_over_coset(const plk_domain* dc, uint64_t poly_degree, plk_fr* out) {
  PLK_API_BEGIN
  if (!dc || !out) return PLK_E_ARG;
  plk_domain* d = const_cast<plk_domain*>(dc);
  DeviceGuard g(d->ctx->device);
  int st;
  if ((st = d->io.alloc(d->n * sizeof(Fr)))) return st;
  if ((st = ntt_vanishing(d, poly_degree, d->io.as<Fr>(), d->ctx->stream))) return st;
  PLK_HIP_TRY(hipMemcpyAsync(out, d->io.ptr, d->n * sizeof(Fr), hipMemcpyDeviceToHost,
                             d->ctx->stream));
  PLK_HIP_TRY(stream_wait(d->ctx->stream));
  return PLK_OK;
  PLK_API_END
}

// ---------------------------------------------------------------------------------- NTT
int plk_ntt(plk_domain* d, plk_fr* inout, size_t len_in, int dir, int coset) {
  PLK_API_BEGIN
  if (!d || (!inout && len_in) || (dir != 1 && dir != -1) || len_in > d->n) return PLK_E_ARG;
  if (!inout) return PLK_E_ARG;
  DeviceGuard g(d->ctx->device);
  hipStream_t s = d->ctx->stream;
  int st;
  if ((st = d->io.alloc(d->n * sizeof(Fr)))) return st;
  if (len_in)
    PLK_HIP_TRY(hipMemcpyAsync(d->io.ptr, inout, len_in * sizeof(Fr), hipMemcpyHostToDevice, s));
  if ((st = ntt_run(d, d->io.as<Fr>(), d->io.as<Fr>(), len_in, dir, coset, nullptr, s, 1)))
    return st;
  PLK_HIP_TRY(hipMemcpyAsync(inout, d->io.ptr, d->n * sizeof(Fr), hipMemcpyDeviceToHost, s));
  PLK_HIP_TRY(stream_wait(s));
  return PLK_OK;
  PLK_API_END
}

// plk_ntt with the caller's stream (SURVEY §8b's signature): stream-ordered staging buffer
// and scratch of its own (hipMallocAsync), so calls on different streams of one domain do not
// share the domain's io / scratch buffers; returns once `inout` holds the result.
int plk_ntt_stream(plk_domain* d, plk_fr* inout, size_t len_in, int dir, int coset,
                   void* stream) {
  PLK_API_BEGIN
  if (!d || !inout || (dir != 1 && dir != -1) || len_in > d->n) return PLK_E_ARG;
  DeviceGuard g(d->ctx->device);
  hipStream_t s = stream ? (hipStream_t)stream : d->ctx->stream;
  void* buf = nullptr;  // n elements of data + 2n of scratch
  if (hipMallocAsync(&buf, 3 * d->n * sizeof(Fr), s) != hipSuccess) return PLK_E_OOM;
  Fr* io = static_cast<Fr*>(buf);
  int st = PLK_OK;
  hipError_t e = hipSuccess;
  if (len_in) e = hipMemcpyAsync(io, inout, len_in * sizeof(Fr), hipMemcpyHostToDevice, s);
  if (e == hipSuccess) {
    st = ntt_run(d, io, io, len_in, dir, coset, io + d->n, s, 1);
    if (st == PLK_OK)
      e = hipMemcpyAsync(inout, io, d->n * sizeof(Fr), hipMemcpyDeviceToHost, s);
  }
  (void)hipFreeAsync(buf, s);
  if (e == hipSuccess && st == PLK_OK) e = stream_wait(s);
  if (e != hipSuccess) {
    last_hip_error() = e;
    return PLK_E_DEVICE;
  }
  return st;
  PLK_API_END
}

int plk_ntt_dev(plk_domain* d, const plk_fr* d_in, plk_fr* d_out, size_t len_in, int dir,
                int coset, plk_fr* d_scratch, void* stream) {
  PLK_API_BEGIN
  if (!d || !d_out || (!d_in && len_in) || (dir != 1 && dir != -1) || len_in > d->n)
    return PLK_E_ARG;
  DeviceGuard g(d->ctx->device);
  hipStream_t s = stream ? (hipStream_t)stream : d->ctx->stream;
  const Fr* in = d_in ? reinterpret_cast<const Fr*>(d_in) : reinterpret_cast<const Fr*>(d_out);
  return ntt_run(d, in, reinterpret_cast<Fr*>(d_out), len_in, dir, coset,
                 reinterpret_cast<Fr*>(d_scratch), s, 1);
  PLK_API_END
}

int plk_ntt_batch_dev(plk_domain* d, plk_fr* d_inout, size_t count, int dir, int coset,
                      void* stream) {
  PLK_API_BEGIN
  if (!d || !d_inout || count == 0 || count > 65535 || (dir != 1 && dir != -1)) return PLK_E_ARG;
  DeviceGuard g(d->ctx->device);
  hipStream_t s = stream ? (hipStream_t)stream : d->ctx->stream;
  Fr* p = reinterpret_cast<Fr*>(d_inout);
  return ntt_run(d, p, p, d->n, dir, coset, nullptr, s, (uint32_t)count);
  PLK_API_END
}

// ---------------------------------------------------------------------------------- SRS
static int srs_alloc(plk_ctx* ctx, size_t n, std::unique_ptr<plk_srs>& s) {
  s.reset(new plk_srs());
  s->ctx = ctx;
  s->n = n;
  int st;
  if ((st = s->points.alloc(n * sizeof(G1Affine)))) return st;
  if ((st = s->inf.alloc(n))) return st;
  return PLK_OK;
}

static void g1_to_abi(const G1Affine& a, uint8_t inf, plk_g1* out) {
  if (inf) {
    std::memset(out, 0, sizeof(*out));
    out->infinity = 1;
    return;
  }
  for (int i = 0; i < 6; ++i) {
    out->x[i] = (uint64_t)a.x.v[2 * i] | ((uint64_t)a.x.v[2 * i + 1] << 32);
    out->y[i] = (uint64_t)a.y.v[2 * i] | ((uint64_t)a.y.v[2 * i + 1] << 32);
  }
  out->infinity = 0;
}

int plk_srs_points(const plk_srs* s, size_t start, size_t count, plk_g1* out) {
  PLK_API_BEGIN
  if (!s || (!out && count) || start > s->n || count > s->n - start) return PLK_E_ARG;
  if (!count) return PLK_OK;
  DeviceGuard g(s->ctx->device);
  std::vector<G1Affine> pts(count);
  std::vector<uint8_t> inf(count);
  hipStream_t st = s->ctx->stream;
  PLK_HIP_TRY(hipMemcpyAsync(pts.data(), s->points.as<G1Affine>() + start, count * sizeof(G1Affine),
                             hipMemcpyDeviceToHost, st));
  PLK_HIP_TRY(hipMemcpyAsync(inf.data(), s->inf.as<uint8_t>() + start, count, hipMemcpyDeviceToHost, st));
  PLK_HIP_TRY(stream_wait(st));
  for (size_t i = 0; i < count; ++i) g1_to_abi(pts[i], inf[i], &out[i]);
  return PLK_OK;
  PLK_API_END
}

static int srs_finish(plk_srs* s) {
  std::vector<uint8_t> inf(s->n);
  PLK_HIP_TRY(hipMemcpy(inf.data(), s->inf.ptr, s->n, hipMemcpyDeviceToHost));
  s->has_inf = false;
  for (uint8_t f : inf) s->has_inf |= f != 0;
  return msm_prepare_srs(s, s->ctx->stream);
}

int plk_srs_setup(plk_ctx* ctx, const plk_fr* tau, size_t n_points, plk_g1* out_points,
                  plk_srs** out) {
  return plk_srs_setup_range(ctx, tau, 0, n_points, out_points, out);
}

int plk_srs_setup_range(plk_ctx* ctx, const plk_fr* tau, uint64_t start, size_t n_points,
                        plk_g1* out_points, plk_srs** out) {
  PLK_API_BEGIN
  if (!ctx || !tau || !out || n_points == 0 || n_points > (1ull << 26)) return PLK_E_ARG;
  *out = nullptr;
  DeviceGuard g(ctx->device);
  std::unique_ptr<plk_srs> s;
  int st;
  if ((st = srs_alloc(ctx, n_points, s))) return st;
  if ((st = srs_generate(s.get(), fr_from_abi(tau), start, ctx->stream))) return st;
  if ((st = srs_finish(s.get()))) return st;
  if (out_points && (st = plk_srs_points(s.get(), 0, n_points, out_points))) return st;
  *out = s.release();
  return PLK_OK;
  PLK_API_END
}

int plk_srs_load(plk_ctx* ctx, const plk_g1* points, size_t n_points, plk_srs** out) {
  PLK_API_BEGIN
  if (!ctx || !points || !out || n_points == 0 || n_points > (1ull << 26)) return PLK_E_ARG;
  *out = nullptr;
  DeviceGuard g(ctx->device);
  std::unique_ptr<plk_srs> s;
  int st;
  if ((st = srs_alloc(ctx, n_points, s))) return st;
  std::vector<G1Affine> pts(n_points);
  std::vector<uint8_t> inf(n_points);
  for (size_t i = 0; i < n_points; ++i) {
    inf[i] = points[i].infinity ? 1 : 0;
    for (int k = 0; k < 6; ++k) {
      const uint64_t x = inf[i] ? 0 : points[i].x[k], y = inf[i] ? 0 : points[i].y[k];
      pts[i].x.v[2 * k] = (uint32_t)x;
      pts[i].x.v[2 * k + 1] = (uint32_t)(x >> 32);
      pts[i].y.v[2 * k] = (uint32_t)y;
      pts[i].y.v[2 * k + 1] = (uint32_t)(y >> 32);
    }
  }
  PLK_HIP_TRY(hipMemcpy(s->points.ptr, pts.data(), n_points * sizeof(G1Affine), hipMemcpyHostToDevice));
  PLK_HIP_TRY(hipMemcpy(s->inf.ptr, inf.data(), n_points, hipMemcpyHostToDevice));
  if ((st = srs_finish(s.get()))) return st;
  *out = s.release();
  return PLK_OK;
  PLK_API_END
}

int plk_srs_destroy(plk_srs* s) {
  PLK_API_BEGIN
  if (!s) return PLK_E_ARG;
  DeviceGuard g(s->ctx->device);
  (void)stream_wait(s->ctx->stream);
  delete s;
  return PLK_OK;
  PLK_API_END
}

int plk_srs_len(const plk_srs* s, size_t* n) {
  if (!s || !n) return PLK_E_ARG;
  *n = s->n;
  return PLK_OK;
}

// ------------------------------------------------------------------------------ MSM/KZG
static int stage_scalars(plk_srs* s, const plk_fr* scalars, size_t len) {
  int st;
  if ((st = s->staging.alloc((len ? len : 1) * sizeof(Fr)))) return st;
  if (len)
    PLK_HIP_TRY(hipMemcpyAsync(s->staging.ptr, scalars, len * sizeof(Fr), hipMemcpyHostToDevice,
                               s->ctx->stream));
  return PLK_OK;
}

int plk_msm(plk_srs* s, const plk_fr* scalars, size_t len, plk_g1* out) {
  PLK_API_BEGIN
  if (!s || !out || (!scalars && len) || len > s->n) return PLK_E_ARG;
  DeviceGuard g(s->ctx->device);
  int st;
  if ((st = stage_scalars(s, scalars, len))) return st;
  return msm_run(s, s->staging.as<Fr>(), len, len, out, s->ctx->stream);
  PLK_API_END
}

int plk_commit(plk_srs* s, const plk_fr* coeffs, size_t len, plk_g1* out) {
  PLK_API_BEGIN
  if (!s || !out || (!coeffs && len)) return PLK_E_ARG;
  // Coefficients::degree() ignores trailing zeros; commit errs past the SRS length
  size_t eff = len;
  while (eff > 0) {
    const plk_fr& c = coeffs[eff - 1];
    if (c.l[0] | c.l[1] | c.l[2] | c.l[3]) break;
    --eff;
  }
  if (eff > s->n) return PLK_E_DEGREE;
  DeviceGuard g(s->ctx->device);
  int st;
  if ((st = stage_scalars(s, coeffs, eff))) return st;
  return msm_run(s, s->staging.as<Fr>(), eff, eff, out, s->ctx->stream);
  PLK_API_END
}

int plk_commit_dev(plk_srs* s, const plk_fr* d_coeffs, size_t len, plk_g1* out, void* stream) {
  PLK_API_BEGIN
  if (!s || !out || (!d_coeffs && len)) return PLK_E_ARG;
  DeviceGuard g(s->ctx->device);
  hipStream_t st = stream ? (hipStream_t)stream : s->ctx->stream;
  const size_t m = len < s->n ? len : s->n;
  return msm_run(s, reinterpret_cast<const Fr*>(d_coeffs), m, len, out, st);
  PLK_API_END
}

int plk_commit_batch_dev(plk_srs* s, const plk_fr* const* d_coeffs, const size_t* lens,
                         size_t count, plk_g1* outs, int* statuses, void* stream) {
  return plk_commit_batch_dev_part(s, d_coeffs, lens, count, 0, 1, outs, statuses, stream);
}

int plk_commit_batch_dev_part(plk_srs* s, const plk_fr* const* d_coeffs, const size_t* lens,
                              size_t count, uint32_t part, uint32_t parts, plk_g1* outs,
                              int* statuses, void* stream) {
  PLK_API_BEGIN
  if (!s || !outs || (count && (!d_coeffs || !lens))) return PLK_E_ARG;
  for (size_t k = 0; k < count; ++k)
    if (!d_coeffs[k] && lens[k]) return PLK_E_ARG;
  DeviceGuard g(s->ctx->device);
  hipStream_t st = stream ? (hipStream_t)stream : s->ctx->stream;
  int overall = PLK_OK;
  for (size_t base = 0; base < count; base += kMaxSlots) {
    const size_t m = count - base < kMaxSlots ? count - base : kMaxSlots;
    const Fr* ptrs[kMaxSlots];
    size_t use[kMaxSlots], chk[kMaxSlots];
    for (size_t k = 0; k < m; ++k) {
      ptrs[k] = reinterpret_cast<const Fr*>(d_coeffs[base + k]);
      chk[k] = lens[base + k];
      use[k] = chk[k] < s->n ? chk[k] : s->n;
    }
    const int r = msm_run_batch(s, *s->ws, ptrs, use, chk, m, outs + base,
                                statuses ? statuses + base : nullptr, st, part, parts);
    if (r != PLK_OK && r != PLK_E_DEGREE) return r;
    if (r != PLK_OK && overall == PLK_OK) overall = r;
  }
  return overall;
  PLK_API_END
}

int plk_g1_sum(const plk_g1* points, size_t n, plk_g1* out) {
  PLK_API_BEGIN
  if (!out || (!points && n)) return PLK_E_ARG;
  G1xyzz acc = xyzz_infinity();
  for (size_t i = 0; i < n; ++i) {
    if (points[i].infinity) continue;
    Fp x, y;
    for (int k = 0; k < 6; ++k) {
      x.v[2 * k] = (uint32_t)points[i].x[k];
      x.v[2 * k + 1] = (uint32_t)(points[i].x[k] >> 32);
      y.v[2 * k] = (uint32_t)points[i].y[k];
      y.v[2 * k + 1] = (uint32_t)(points[i].y[k] >> 32);
    }
    acc = xyzz_add_affine(acc, x, y);
  }
  G1Affine r;
  const bool fin = xyzz_to_affine(acc, r.x, r.y);
  g1_to_abi(r, fin ? 0 : 1, out);
  return PLK_OK;
  PLK_API_END
}

int plk_msm_sharded(plk_srs* const* per_gpu, int n_gpu, const plk_fr* scalars, size_t len,
                    plk_g1* out) {
  PLK_API_BEGIN
  if (!per_gpu || n_gpu <= 0 || !out || (!scalars && len)) return PLK_E_ARG;
  size_t total = 0;
  for (int i = 0; i < n_gpu; ++i) {
    if (!per_gpu[i]) return PLK_E_ARG;
    total += per_gpu[i]->n;
  }
  if (len > total) return PLK_E_ARG;
  std::vector<plk_g1> part((size_t)n_gpu, plk_g1{});
  std::vector<int> status((size_t)n_gpu, PLK_OK);
  std::vector<std::thread> workers;
  workers.reserve((size_t)n_gpu);
  size_t off = 0;
  try {
    for (int i = 0; i < n_gpu; ++i) {
      plk_srs* s = per_gpu[i];
      const size_t cnt = off < len ? std::min(s->n, len - off) : 0;
      part[i].infinity = 1;
      if (cnt)
        workers.emplace_back([&part, &status, s, i, cnt, p = scalars + off]() {
          status[i] = plk_msm(s, p, cnt, &part[i]);
        });
      off += s->n;
    }
  } catch (...) {  // a thread that failed to start: drain the started ones, then report
    for (auto& t : workers) t.join();
    throw;
  }
  for (auto& t : workers) t.join();
  for (int i = 0; i < n_gpu; ++i)
    if (status[i] != PLK_OK) return status[i];
  return plk_g1_sum(part.data(), (size_t)n_gpu, out);
  PLK_API_END
}

int plk_srs_msm_stats_reset(plk_srs* s) {
  if (!s) return PLK_E_ARG;
  s->ws->stats.reset_cum();
  return PLK_OK;
}

int plk_srs_cum_msm_stats(const plk_srs* s, double* accumulate_ms, uint64_t* launches,
                          uint64_t* point_adds, uint64_t* points) {
  if (!s) return PLK_E_ARG;
  const MsmStats& st = s->ws->stats;
  if (accumulate_ms) *accumulate_ms = st.cum_accumulate_ms;
  if (launches) *launches = st.cum_launches;
  if (point_adds) *point_adds = st.cum_point_adds;
  if (points) *points = st.cum_points;
  return PLK_OK;
}

int plk_srs_last_msm_stats(const plk_srs* s, float* accumulate_ms, uint64_t* point_adds,
                           uint32_t* window_bits) {
  if (!s) return PLK_E_ARG;
  if (accumulate_ms) *accumulate_ms = s->ws->stats.last_accumulate_ms;
  if (point_adds) *point_adds = s->ws->stats.last_point_adds;
  if (window_bits) *window_bits = s->c;
  return PLK_OK;
}

}  // extern "C"
