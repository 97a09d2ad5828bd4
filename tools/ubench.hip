// ubench.hip — integer-VALU ceilings on MI355X for the roofline of the hot path:
// raw v_mad_u64_u32 issue rate, Fr/Fp Montgomery multiply throughput and the XYZZ mixed
// addition throughput, measured chip-wide with every CU busy and independent chains.
// Build: hipcc -O3 --offload-arch=gfx950 -I../dusk-plonk_amd/csrc tools/ubench.hip -o tools/ubench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#include "../dusk-plonk_amd/csrc/g1.hpp"

using namespace plk;

#define CHECK(x)                                                        \
  do {                                                                  \
    hipError_t e = (x);                                                 \
    if (e != hipSuccess) {                                              \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      return 1;                                                         \
    }                                                                   \
  } while (0)

// 8 independent 64-bit accumulation chains of v_mad_u64_u32
__global__ void __launch_bounds__(256) k_mad(uint64_t* out, uint32_t iters, uint32_t seed) {
  uint32_t a = threadIdx.x ^ seed, b = blockIdx.x * 7 + 3;
  uint64_t acc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) acc[i] = i;
  for (uint32_t it = 0; it < iters; ++it) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        uint64_t cy;
        asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc[i]), "=s"(cy) : "v"(a), "v"(b + i));
      }
    }
  }
  uint64_t s = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) s ^= acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <class C, int CHAINS>
__global__ void __launch_bounds__(256) k_modmul(Fe<C>* io, uint32_t iters) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  Fe<C> x[CHAINS], y = io[t];
#pragma unroll
  for (int i = 0; i < CHAINS; ++i) {
    x[i] = y;
    x[i].v[0] ^= i;
  }
  for (uint32_t it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < CHAINS; ++i) x[i] = fe_mul(x[i], y);
  }
  Fe<C> s = x[0];
#pragma unroll
  for (int i = 1; i < CHAINS; ++i) s = fe_add(s, x[i]);
  io[t] = s;
}

__global__ void __launch_bounds__(256) k_madd(G1xyzz* io, const G1Affine* pts, uint32_t iters,
                                              uint32_t npts) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  G1xyzz acc = io[t];
  for (uint32_t it = 0; it < iters; ++it) {
    const G1Affine p = pts[(t + it * 977u) % npts];
    acc = xyzz_add_affine(acc, p.x, p.y);
  }
  io[t] = acc;
}

int main() {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const uint32_t blocks = cus * 8, threads = 256, total = blocks * threads;
  float ms;
  // raw mad
  {
    uint64_t* out;
    CHECK(hipMalloc(&out, total * 8));
    const uint32_t iters = 256;
    hipLaunchKernelGGL(k_mad, dim3(blocks), dim3(threads), 0, 0, out, 4, 1u);
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL(k_mad, dim3(blocks), dim3(threads), 0, 0, out, iters, 1u);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    const double mads = (double)total * iters * 16 * 8;
    std::printf("{\"test\":\"v_mad_u64_u32\",\"per_s\":%.4e,\"per_cu_per_clk_at_2.4GHz\":%.3f}\n",
                mads / (ms * 1e-3), mads / (ms * 1e-3) / cus / 2.4e9);
    CHECK(hipFree(out));
  }
  // Fr / Fp modmul
  {
    Fr* io;
    CHECK(hipMalloc(&io, total * sizeof(Fr)));
    CHECK(hipMemset(io, 0x11, total * sizeof(Fr)));
    const uint32_t iters = 512;
    hipLaunchKernelGGL((k_modmul<FrCfg, 4>), dim3(blocks), dim3(threads), 0, 0, io, 4);
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL((k_modmul<FrCfg, 4>), dim3(blocks), dim3(threads), 0, 0, io, iters);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    std::printf("{\"test\":\"fr_mul\",\"per_s\":%.4e}\n", (double)total * iters * 4 / (ms * 1e-3));
    CHECK(hipFree(io));
  }
  {
    Fp* io;
    CHECK(hipMalloc(&io, total * sizeof(Fp)));
    CHECK(hipMemset(io, 0x11, total * sizeof(Fp)));
    const uint32_t iters = 256;
    hipLaunchKernelGGL((k_modmul<FpCfg, 2>), dim3(blocks), dim3(threads), 0, 0, io, 4);
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL((k_modmul<FpCfg, 2>), dim3(blocks), dim3(threads), 0, 0, io, iters);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    std::printf("{\"test\":\"fp_mul\",\"per_s\":%.4e}\n", (double)total * iters * 2 / (ms * 1e-3));
    CHECK(hipFree(io));
  }
  // XYZZ mixed add (the MSM accumulation step), points from a small table (L2-resident)
  {
    const uint32_t npts = 4096, iters = 128;
    std::vector<G1Affine> h(npts);
    // any field elements exercise the same instruction stream; use Montgomery(1), (2)...
    for (uint32_t i = 0; i < npts; ++i) {
      for (int k = 0; k < 12; ++k) {
        h[i].x.v[k] = (i * 2654435761u + k) & 0x0fffffffu;
        h[i].y.v[k] = (i * 40503u + 7 * k) & 0x0fffffffu;
      }
    }
    G1Affine* pts;
    G1xyzz* io;
    CHECK(hipMalloc(&pts, npts * sizeof(G1Affine)));
    CHECK(hipMalloc(&io, total * sizeof(G1xyzz)));
    CHECK(hipMemcpy(pts, h.data(), npts * sizeof(G1Affine), hipMemcpyHostToDevice));
    CHECK(hipMemset(io, 0x01, total * sizeof(G1xyzz)));
    hipLaunchKernelGGL(k_madd, dim3(blocks), dim3(threads), 0, 0, io, pts, 2, npts);
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL(k_madd, dim3(blocks), dim3(threads), 0, 0, io, pts, iters, npts);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    std::printf("{\"test\":\"g1_xyzz_madd\",\"per_s\":%.4e}\n", (double)total * iters / (ms * 1e-3));
    CHECK(hipFree(pts));
    CHECK(hipFree(io));
  }
  return 0;
}
