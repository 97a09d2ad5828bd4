// ubench_quad.hip — latency of one dependent XYZZ full addition on a lone wave: the
// single-lane lazy addition (g1r_add_lazy) against the quad-cooperative one (g1r_add_quad,
// g1r.hpp), and a bit-identity check of the two on the same chains. (Round 4 also measured the
// quad's products with their column terms in 2 / 4 pinned accumulator chains: 6.6 / 7.2 us
// against 6.1 us — a lone wave's addition is issue-bound, not chain-bound; not kept.)
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/ubench_quad.hip -o tools/ubench_quad
#include <hip/hip_runtime.h>

#include <cstdio>
#include <random>
#include <vector>

#include "../dusk-plonk_amd/csrc/g1r.hpp"

using namespace plk;

#define CHECK(x)                                                                    \
  do {                                                                              \
    hipError_t e = (x);                                                             \
    if (e != hipSuccess) {                                                          \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      return 1;                                                                     \
    }                                                                               \
  } while (0)

constexpr int kPts = 4096;

// thread t: acc = in[t], then acc += in[(t + 7 i + 1) % kPts], n times
__global__ void __launch_bounds__(64) k_chain(const G1xyzz* __restrict__ in, G1xyzz* __restrict__ out, int n) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  G1R acc = ld_g1r(&in[t % kPts]);
  for (int i = 0; i < n; ++i) acc = g1r_add_lazy(acc, ld_g1r(&in[(t + 7 * i + 1) % kPts]));
  st_g1r(&out[t], g1r_lazy_finish(acc));
}

// quad t (lanes 4t .. 4t + 3) runs thread t's chain
__global__ void __launch_bounds__(256) k_chain_quad(const G1xyzz* __restrict__ in, G1xyzz* __restrict__ out, int n) {
  const uint32_t t = (blockIdx.x * blockDim.x + threadIdx.x) >> 2, l = threadIdx.x & 3;
  G1R acc = ld_g1r(&in[t % kPts]);
  for (int i = 0; i < n; ++i) acc = g1r_add_quad(acc, ld_g1r(&in[(t + 7 * i + 1) % kPts]), l);
  if (l == 0) st_g1r(&out[t], g1r_lazy_finish(acc));
}

int main() {
  // random XYZZ-shaped values (the instruction stream is that of real points); canonical limbs
  std::mt19937_64 g(5);
  std::vector<uint32_t> h(kPts * 48);
  for (int i = 0; i < kPts; ++i)
    for (int c = 0; c < 4; ++c)
      for (int w = 0; w < 12; ++w) h[i * 48 + c * 12 + w] = w == 11 ? (uint32_t)(g() & 0x0fffffffu) : (uint32_t)g();
  G1xyzz *din, *d1, *d2;
  CHECK(hipMalloc(&din, kPts * sizeof(G1xyzz)));
  CHECK(hipMalloc(&d1, kPts * sizeof(G1xyzz)));
  CHECK(hipMalloc(&d2, kPts * sizeof(G1xyzz)));
  CHECK(hipMemcpy(din, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  auto timeit = [&](auto launch) {
    launch();
    (void)hipDeviceSynchronize();
    float best = 1e30f;
    for (int r = 0; r < 3; ++r) {
      (void)hipEventRecord(a);
      launch();
      (void)hipEventRecord(b);
      (void)hipEventSynchronize(b);
      float ms;
      (void)hipEventElapsedTime(&ms, a, b);
      best = ms < best ? ms : best;
    }
    return best;
  };
  const int n = 64;
  const float ms1 = timeit([&] { hipLaunchKernelGGL(k_chain, dim3(1), dim3(64), 0, 0, din, d1, n); });
  const float msq = timeit([&] { hipLaunchKernelGGL(k_chain_quad, dim3(1), dim3(256), 0, 0, din, d2, n); });
  std::vector<uint32_t> r1(64 * 48), r2(64 * 48);
  CHECK(hipMemcpy(r1.data(), d1, r1.size() * 4, hipMemcpyDeviceToHost));
  CHECK(hipMemcpy(r2.data(), d2, r2.size() * 4, hipMemcpyDeviceToHost));
  hipFuncAttributes fa;
  CHECK(hipFuncGetAttributes(&fa, (const void*)k_chain_quad));
  std::printf("{\"lone_wave_lazy_us_per_add\":%.2f,\"quad_us_per_add\":%.2f,\"quad_vgprs\":%d,\"quad_spill_bytes\":%d,\"bit_identical\":%s}\n",
              1e3 * ms1 / n, 1e3 * msq / n, fa.numRegs, (int)fa.localSizeBytes,
              r1 == r2 ? "true" : "false");
  return 0;
}
