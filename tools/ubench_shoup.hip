// ubench_shoup.hip — the constant-twiddle (Shoup) Fr product of ntt.hip (fr_shoup, ffr.hpp)
// against the Montgomery product it replaces (rx_mul by an R'-domain twiddle):
//   * check: for random x (canonical, and unnormalised NTT-style multiplicands a + 6r - b)
//     and random twiddles w, fr_shoup(x, w, w') == rx_mul(x, w R' mod r) mod r;
//   * throughput: chains of products by 4 constants, whole chip, both forms.
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/ubench_shoup.hip -o tools/ubench_shoup
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <vector>

#include "../dusk-plonk_amd/csrc/ffr.hpp"

using namespace plk;
using RFr = Rx<FrCfg>;

#define CHECK(x)                                                                    \
  do {                                                                              \
    hipError_t e = (x);                                                             \
    if (e != hipSuccess) {                                                          \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      return 1;                                                                     \
    }                                                                               \
  } while (0)

// (w, w') of a canonical R'-domain twiddle rho = w R' mod r, kept as raw limbs (w' is a
// 261-bit value: it does not fit the packed 256-bit layout)
__global__ void k_prep(const Fr* rho, RFr* w, RFr* wp, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  fr_shoup_prep(rx_unpack(rho[i]), w[i], wp[i]);
}

// out = x * w mod r (canonical) both ways; mode 1: x -> x + 6r - y (unnormalised limbs)
__global__ void k_check(const Fr* x, const Fr* y, const Fr* rho, const RFr* w, const RFr* wp,
                        uint32_t n, int mode, uint32_t* bad) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  RFr a = rx_unpack(x[i]);
  if (mode == 1) a = rx_sub_u<FrCfg, 6>(a, rx_unpack(y[i]));
  const Fr m = rx_pack_canonical(rx_mul(a, rx_unpack(rho[i])));
  Fr s = rx_pack(fr_shoup(a, w[i], wp[i]));  // [0, 3r)
  fe_reduce_once(s);
  fe_reduce_once(s);
  for (int k = 0; k < 8; ++k)
    if (m.v[k] != s.v[k]) {
      atomicAdd(bad, 1u);
      break;
    }
}

template <int FORM>
__global__ void __launch_bounds__(256) k_thr(Fr* io, const Fr* rho, const RFr* w, const RFr* wp,
                                             uint32_t iters) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  RFr x0 = rx_unpack(io[2 * i]), x1 = rx_unpack(io[2 * i + 1]);
  RFr c[4], cp[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    c[k] = FORM == 0 ? rx_unpack(rho[k]) : w[k];
    cp[k] = wp[k];
  }
  for (uint32_t it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (FORM == 0) {
        x0 = rx_mul(x0, c[k]);
        x1 = rx_mul(x1, c[(k + 1) & 3]);
      } else {
        x0 = fr_shoup(x0, c[k], cp[k]);
        x1 = fr_shoup(x1, c[(k + 1) & 3], cp[(k + 1) & 3]);
      }
    }
  }
  io[2 * i] = rx_pack(x0);
  io[2 * i + 1] = rx_pack(x1);
}

static uint64_t g_s = 0x5eed;
static uint32_t rnd() {
  g_s += 0x9E3779B97F4A7C15ull;
  uint64_t z = g_s;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return (uint32_t)(z ^ (z >> 31));
}
static Fr rnd_fr() {  // canonical (top word < r's top word)
  Fr x;
  for (int k = 0; k < 8; ++k) x.v[k] = rnd();
  x.v[7] &= 0x3fffffffu;
  if (x.v[7] >= FrCfg::P[7]) x.v[7] -= FrCfg::P[7];
  return x;
}

int main() {
  const uint32_t n = 1u << 20;
  std::vector<Fr> hx(n), hy(n), hrho(n);
  for (uint32_t i = 0; i < n; ++i) {
    hx[i] = rnd_fr();
    hy[i] = rnd_fr();
    hrho[i] = rnd_fr();
  }
  // edge cases: 0, r - 1, twiddle 1 and r - 1 (R'-domain values are arbitrary canonical)
  for (int k = 0; k < 8; ++k) {
    hx[0].v[k] = 0;
    hx[1].v[k] = FrCfg::P[k];
  }
  hx[1].v[0] -= 1;
  Fr *dx, *dy, *drho;
  RFr *dw, *dwp;
  uint32_t* dbad;
  CHECK(hipMalloc(&dx, n * sizeof(Fr)));
  CHECK(hipMalloc(&dy, n * sizeof(Fr)));
  CHECK(hipMalloc(&drho, n * sizeof(Fr)));
  CHECK(hipMalloc(&dw, n * sizeof(RFr)));
  CHECK(hipMalloc(&dwp, n * sizeof(RFr)));
  CHECK(hipMalloc(&dbad, 4));
  CHECK(hipMemcpy(dx, hx.data(), n * sizeof(Fr), hipMemcpyHostToDevice));
  CHECK(hipMemcpy(dy, hy.data(), n * sizeof(Fr), hipMemcpyHostToDevice));
  CHECK(hipMemcpy(drho, hrho.data(), n * sizeof(Fr), hipMemcpyHostToDevice));
  hipLaunchKernelGGL(k_prep, dim3(n / 256), dim3(256), 0, 0, drho, dw, dwp, n);
  for (int mode = 0; mode < 2; ++mode) {
    CHECK(hipMemset(dbad, 0, 4));
    hipLaunchKernelGGL(k_check, dim3(n / 256), dim3(256), 0, 0, dx, dy, drho, dw, dwp, n, mode, dbad);
    uint32_t bad = 0;
    CHECK(hipMemcpy(&bad, dbad, 4, hipMemcpyDeviceToHost));
    std::printf("{\"test\":\"shoup_check_mode%d\",\"cases\":%u,\"mismatches\":%u}\n", mode, n, bad);
  }
  const uint32_t threads = 1u << 18, iters = 256;
  Fr* dio;
  CHECK(hipMalloc(&dio, 2 * threads * sizeof(Fr)));
  CHECK(hipMemcpy(dio, hx.data(), 2 * threads * sizeof(Fr), hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int rep = 0; rep < 2; ++rep)
    for (int form = 0; form < 2; ++form) {
      auto kern = form == 0 ? k_thr<0> : k_thr<1>;
      hipLaunchKernelGGL(kern, dim3(threads / 256), dim3(256), 0, 0, dio, drho, dw, dwp, 8u);
      CHECK(hipDeviceSynchronize());
      CHECK(hipEventRecord(e0));
      hipLaunchKernelGGL(kern, dim3(threads / 256), dim3(256), 0, 0, dio, drho, dw, dwp, iters);
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float ms;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      const double muls = (double)threads * iters * 8;
      std::printf("{\"test\":\"%s\",\"mul_per_s\":%.4e}\n", form == 0 ? "montgomery_rx_mul" : "shoup",
                  muls / (ms * 1e-3));
    }
  return 0;
}
