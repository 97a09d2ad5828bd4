// opening.hip — PlonkParams::compute_aggregate_witness as a primitive C-ABI entry point.
//
// The reference opens its polynomials with
//   keypair.compute_aggregate_witness(&[p_0, .., p_{k-1}], &point, &v)
// (/root/reference/src/prover.rs:422-438 at z, :444-450 at z·ω), i.e.
//   W(X) = (sum_i v^i p_i(X)) / (X - point)        (Ruffini; the remainder is dropped)
// in the un-vendored zksnarks crate. plk_prove does the same inside the prover (k_lincomb +
// pk_ruffini, prover.hip); these entries expose it on its own so a patched zksnarks can
// route the call to the GPU at the primitive level, like plk_commit.
//
// Device work: ceil(k / 23) k_lincomb passes (a linear combination of up to kMaxTerms
// polynomials per pass, the running sum carried as the first term of the next pass), then
// the Ruffini division (scaled powers, a suffix scan, scaled powers). Scratch is allocated
// stream-ordered (hipMallocAsync / hipFreeAsync), so calls on different streams of one
// context do not share buffers.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <new>
#include <vector>

#include "ffr.hpp"
#include "internal.hpp"
#include "prover.hpp"

using namespace plk;

#define PLK_API_BEGIN try {
#define PLK_API_END               \
  }                               \
  catch (const std::bad_alloc&) { \
    return PLK_E_OOM;             \
  }                               \
  catch (...) {                   \
    return PLK_E_DEVICE;          \
  }

namespace {

Fr fr_of(const plk_fr& a) {
  Fr r;
  for (int i = 0; i < 4; ++i) {
    r.v[2 * i] = (uint32_t)a.l[i];
    r.v[2 * i + 1] = (uint32_t)(a.l[i] >> 32);
  }
  return r;
}

// limbs < r (the ABI takes canonical Montgomery values)
bool fr_canonical(const plk_fr& a) {
  for (int i = FrCfg::N - 1; i >= 0; --i) {
    const uint32_t w = (uint32_t)(a.l[i / 2] >> (32 * (i % 2)));
    if (w != FrCfg::P[i]) return w < FrCfg::P[i];
  }
  return false;
}

// Stream-ordered scratch freed on the same stream when the scope ends.
struct AsyncBuf {
  void* ptr = nullptr;
  hipStream_t s = nullptr;
  int alloc(size_t bytes, hipStream_t st) {
    s = st;
    if (hipMallocAsync(&ptr, std::max<size_t>(bytes, 32), st) != hipSuccess) {
      ptr = nullptr;
      return PLK_E_OOM;
    }
    return PLK_OK;
  }
  ~AsyncBuf() {
    if (ptr) (void)hipFreeAsync(ptr, s);
  }
  Fr* fr() const { return static_cast<Fr*>(ptr); }
};

// W = (sum_i v^i p_i) / (X - point) on `s`; out receives max(lens) - 1 coefficients.
int aggregate_witness(const Fr* const* polys, const size_t* lens, size_t count, const Fr& point,
                      const Fr& v, Fr* out, uint64_t max_len, hipStream_t s) {
  AsyncBuf sum[2], tmp, scan;
  int st;
  if ((st = sum[0].alloc(max_len * sizeof(Fr), s))) return st;
  if (count > (size_t)kMaxTerms && (st = sum[1].alloc(max_len * sizeof(Fr), s))) return st;
  // sum_i v^i p_i in passes of kMaxTerms terms (after the first pass, term 0 is the sum so far)
  Fr vp = fe_one<FrCfg>();
  size_t i = 0;
  int cur = -1;
  while (i < count) {
    LinComb lc{};
    if (cur >= 0) {
      lc.p[0] = sum[cur].fr();
      lc.len[0] = max_len;
      lc.s[0] = fe_one<FrCfg>();
      lc.terms = 1;
    }
    while (i < count && lc.terms < (uint32_t)kMaxTerms) {
      lc.p[lc.terms] = polys[i];
      lc.len[lc.terms] = lens[i];
      lc.s[lc.terms] = vp;
      ++lc.terms;
      vp = fe_mul(vp, v);
      ++i;
    }
    const int nxt = cur < 0 ? 0 : 1 - cur;
    if ((st = pk_lincomb(lc, sum[nxt].fr(), max_len, s))) return st;
    cur = nxt;
  }
  if (max_len <= 1) return PLK_OK;
  if (fe_is_zero(point)) {  // division by X: q_k = c_(k+1)
    PLK_HIP_TRY(hipMemcpyAsync(out, sum[cur].fr() + 1, (max_len - 1) * sizeof(Fr),
                               hipMemcpyDeviceToDevice, s));
    return PLK_OK;
  }
  if ((st = tmp.alloc(max_len * sizeof(Fr), s))) return st;
  if ((st = scan.alloc(pk_scan_tmp_elems(max_len) * sizeof(Fr), s))) return st;
  return pk_ruffini(sum[cur].fr(), max_len, point, out, tmp.fr(), scan.fr(), s);
}

int check_args(const size_t* lens, size_t count, const plk_fr* point, const plk_fr* challenge,
               size_t* out_len, uint64_t* max_len) {
  if ((count && !lens) || !point || !challenge || !out_len) return PLK_E_ARG;
  if (!fr_canonical(*point) || !fr_canonical(*challenge)) return PLK_E_ARG;
  uint64_t m = 0;
  for (size_t i = 0; i < count; ++i) m = std::max<uint64_t>(m, lens[i]);
  *max_len = m;
  *out_len = m > 1 ? (size_t)(m - 1) : 0;
  return PLK_OK;
}

}  // namespace

extern "C" {

int plk_aggregate_witness_dev(plk_ctx* ctx, const plk_fr* const* d_polys, const size_t* lens,
                              size_t count, const plk_fr* point, const plk_fr* challenge,
                              plk_fr* d_out, size_t* out_len, void* stream) {
  PLK_API_BEGIN
  if (!ctx || (count && !d_polys)) return PLK_E_ARG;
  uint64_t max_len = 0;
  int st;
  if ((st = check_args(lens, count, point, challenge, out_len, &max_len))) return st;
  if (*out_len == 0) return PLK_OK;
  if (!d_out) return PLK_E_ARG;
  for (size_t i = 0; i < count; ++i)
    if (lens[i] && !d_polys[i]) return PLK_E_ARG;
  DeviceGuard g(ctx->device);
  hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
  return aggregate_witness(reinterpret_cast<const Fr* const*>(d_polys), lens, count,
                           fr_of(*point), fr_of(*challenge), reinterpret_cast<Fr*>(d_out),
                           max_len, s);
  PLK_API_END
}

int plk_aggregate_witness(plk_ctx* ctx, const plk_fr* const* polys, const size_t* lens,
                          size_t count, const plk_fr* point, const plk_fr* challenge,
                          plk_fr* out, size_t* out_len) {
  PLK_API_BEGIN
  if (!ctx || (count && !polys)) return PLK_E_ARG;
  uint64_t max_len = 0;
  int st;
  if ((st = check_args(lens, count, point, challenge, out_len, &max_len))) return st;
  if (*out_len == 0) return PLK_OK;
  if (!out) return PLK_E_ARG;
  uint64_t total = 0;
  for (size_t i = 0; i < count; ++i) {
    if (lens[i] && !polys[i]) return PLK_E_ARG;
    total += lens[i];
  }
  DeviceGuard g(ctx->device);
  hipStream_t s = ctx->stream;
  AsyncBuf in, res;
  if ((st = in.alloc(total * sizeof(Fr), s))) return st;
  if ((st = res.alloc(*out_len * sizeof(Fr), s))) return st;
  std::vector<const Fr*> dp(count);
  uint64_t off = 0;
  for (size_t i = 0; i < count; ++i) {
    dp[i] = in.fr() + off;
    if (lens[i])
      PLK_HIP_TRY(hipMemcpyAsync(in.fr() + off, polys[i], lens[i] * sizeof(Fr),
                                 hipMemcpyHostToDevice, s));
    off += lens[i];
  }
  if ((st = aggregate_witness(dp.data(), lens, count, fr_of(*point), fr_of(*challenge), res.fr(),
                              max_len, s)))
    return st;
  PLK_HIP_TRY(hipMemcpyAsync(out, res.fr(), *out_len * sizeof(Fr), hipMemcpyDeviceToHost, s));
  PLK_HIP_TRY(stream_wait(s));
  return PLK_OK;
  PLK_API_END
}

}  // extern "C"
