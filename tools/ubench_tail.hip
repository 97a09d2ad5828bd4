// ubench_tail.hip — cost of one XYZZ full addition (g1r.hpp) on a lone wave versus a full
// chip: the MSM's bucket-reduction tail (k_runsum*, k_bitsum*) is a tree of dependent full
// additions whose narrow levels run one wave per SIMD or less.
//   chain: each lane adds n points in sequence (acc = acc + q_i), grids of 1, 1024, 4096 waves
//   tree:  one workgroup of 256 lanes runs the k_bitsum2-shaped shuffle tree (6 levels over a
//          wave, then the wave totals through LDS) r times
// for g1r_add (branching full addition) and g1r_add_lazy (straight-line, repaired after).
// Random field values stand in for points: the instruction stream is the same.
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/ubench_tail.hip -o tools/ubench_tail
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

template <int V>
__device__ __forceinline__ G1R add(const G1R& a, const G1R& b) {
  if (V == 0) return g1r_add(a, b);
  return g1r_add_lazy(a, b);
}

template <int V, int W>
__global__ void __launch_bounds__(256, W) k_chain(const G1xyzz* __restrict__ in, G1xyzz* __restrict__ out, int n) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  G1R acc = ld_g1r(&in[t % kPts]);
  for (int i = 0; i < n; ++i) acc = add<V>(acc, ld_g1r(&in[(t + 7 * i + 1) % kPts]));
  st_g1r(&out[t], acc);
}

__device__ __forceinline__ RFp shfl_rfp(const RFp& v, uint32_t h) {
  Fp x = rx_pack(v);
#pragma unroll
  for (int i = 0; i < 12; ++i) x.v[i] = __shfl_down(x.v[i], h, 64);
  return rx_unpack(x);
}

template <int V, int W>
__global__ void __launch_bounds__(256, W) k_tree(const G1xyzz* __restrict__ in, G1xyzz* __restrict__ out, int r) {
  __shared__ G1xyzz sh[4];
  const uint32_t tid = threadIdx.x;
  G1R acc = ld_g1r(&in[tid]);
  for (int it = 0; it < r; ++it) {
    for (uint32_t h = 32; h >= 1; h >>= 1) {
      G1R o;
      o.X = shfl_rfp(acc.X, h);
      o.Y = shfl_rfp(acc.Y, h);
      o.ZZ = shfl_rfp(acc.ZZ, h);
      o.ZZZ = shfl_rfp(acc.ZZZ, h);
      if ((tid & 63) < h) acc = add<V>(acc, o);
    }
    if ((tid & 63) == 0) st_g1r(&sh[tid >> 6], acc);
    __syncthreads();
    if (tid < 2) acc = add<V>(ld_g1r(&sh[2 * tid]), ld_g1r(&sh[2 * tid + 1]));
    if (tid < 64) {
      G1R o;
      o.X = shfl_rfp(acc.X, 1);
      o.Y = shfl_rfp(acc.Y, 1);
      o.ZZ = shfl_rfp(acc.ZZ, 1);
      o.ZZZ = shfl_rfp(acc.ZZZ, 1);
      if (tid == 0) acc = add<V>(acc, o);
    }
    __syncthreads();
    acc = add<V>(acc, ld_g1r(&in[(tid + it) % kPts]));  // next round's values (one more level)
  }
  if (tid == 0) st_g1r(&out[0], acc);
}

int main() {
  // random R'-domain values below p with the top word small (normalised limbs after unpack)
  std::mt19937_64 rng(7);
  std::vector<uint32_t> h((size_t)kPts * 48);
  for (auto& w : h) w = (uint32_t)rng();
  for (size_t i = 0; i < (size_t)kPts * 4; ++i) h[i * 12 + 11] &= 0x0fffffffu;
  G1xyzz *din, *dout;
  CHECK(hipMalloc(&din, sizeof(G1xyzz) * kPts));
  CHECK(hipMalloc(&dout, sizeof(G1xyzz) * 4096 * 64));
  CHECK(hipMemcpy(din, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  auto timeit = [&](auto launch) -> float {
    launch();
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(e0));
    launch();
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    return ms;
  };
  hipFuncAttributes fa;
  auto run = [&](const char* nm, auto kchain, auto ktree) -> int {
    CHECK(hipFuncGetAttributes(&fa, (const void*)kchain));
    std::printf("%s: chain kernel %d VGPRs (%d spill bytes)\n", nm, fa.numRegs, (int)fa.localSizeBytes);
    for (int waves : {1, 1024, 4096}) {
      const int n = 64;
      float ms = timeit([&] { hipLaunchKernelGGL(kchain, dim3(waves), dim3(64), 0, 0, din, dout, n); });
      const double adds = (double)waves * 64 * n;
      std::printf("  chain %5d waves x %d adds: %8.3f ms  %7.2f us per dependent add  %.3g adds/s\n", waves, n,
                  ms, 1e3 * ms / n, adds / (ms * 1e-3));
    }
    const int r = 8;
    float ms = timeit([&] { hipLaunchKernelGGL(ktree, dim3(1), dim3(256), 0, 0, din, dout, r); });
    std::printf("  tree: %d rounds of 9 levels in %.3f ms: %.2f us per level\n", r, ms, 1e3 * ms / (9 * r));
    ms = timeit([&] { hipLaunchKernelGGL(ktree, dim3(512), dim3(256), 0, 0, din, dout, r); });
    std::printf("  tree x512 workgroups: %.3f ms: %.2f us per level\n", ms, 1e3 * ms / (9 * r));
    return 0;
  };
  if (run("g1r_add", k_chain<0, 1>, k_tree<0, 1>)) return 1;
  if (run("g1r_add_lazy", k_chain<1, 1>, k_tree<1, 1>)) return 1;
  if (run("g1r_add_lazy, 2 waves/SIMD cap", k_chain<1, 2>, k_tree<1, 2>)) return 1;
  if (run("g1r_add, 2 waves/SIMD cap", k_chain<0, 2>, k_tree<0, 2>)) return 1;
  return 0;
}
