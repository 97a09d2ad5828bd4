// debug.hip — plk_debug_field_op: elementwise device field arithmetic for parity tests.
#include <hip/hip_runtime.h>

#include "internal.hpp"

namespace plk {
namespace {

template <class C>
__global__ void k_field_op(int op, const Fe<C>* __restrict__ a, const Fe<C>* __restrict__ b,
                           Fe<C>* __restrict__ out, uint64_t n) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const Fe<C> x = a[i], y = b[i];
  Fe<C> r;
  switch (op) {
    case 0: r = fe_mul(x, y); break;
    case 1: r = fe_add(x, y); break;
    case 2: r = fe_sub(x, y); break;
    case 3: r = fe_sqr(x); break;
    default: r = fe_inv(x); break;
  }
  out[i] = r;
}

template <class C>
int run(plk_ctx* ctx, int op, const uint64_t* a, const uint64_t* b, uint64_t* out, size_t n) {
  const size_t bytes = n * sizeof(Fe<C>);
  DevBuf da, db, dout;
  int st;
  if ((st = da.alloc(bytes)) || (st = db.alloc(bytes)) || (st = dout.alloc(bytes))) return st;
  hipStream_t s = ctx->stream;
  PLK_HIP_TRY(hipMemcpyAsync(da.ptr, a, bytes, hipMemcpyHostToDevice, s));
  PLK_HIP_TRY(hipMemcpyAsync(db.ptr, b ? b : a, bytes, hipMemcpyHostToDevice, s));
  hipLaunchKernelGGL(k_field_op<C>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, op,
                     da.as<Fe<C>>(), db.as<Fe<C>>(), dout.as<Fe<C>>(), (uint64_t)n);
  PLK_HIP_TRY(hipGetLastError());
  PLK_HIP_TRY(hipMemcpyAsync(out, dout.ptr, bytes, hipMemcpyDeviceToHost, s));
  PLK_HIP_TRY(stream_wait(s));
  return PLK_OK;
}

}  // namespace
}  // namespace plk

extern "C" int plk_debug_field_op(plk_ctx* ctx, int field, int op, const uint64_t* a,
                                  const uint64_t* b, uint64_t* out, size_t n) {
  try {
    if (!ctx || !a || !out || op < 0 || op > 4 || (field != 0 && field != 1)) return PLK_E_ARG;
    if (n == 0) return PLK_OK;
    plk::DeviceGuard g(ctx->device);
    return field == 0 ? plk::run<plk::FrCfg>(ctx, op, a, b, out, n)
                      : plk::run<plk::FpCfg>(ctx, op, a, b, out, n);
  } catch (...) {
    return PLK_E_DEVICE;
  }
}
