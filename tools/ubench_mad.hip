// ubench_mad.hip — v_mad_u64_u32 issue cost vs dependent latency on gfx950: NCH independent
// 64-bit accumulator chains per lane, WPS waves per SIMD (256 CUs x 4 SIMDs x WPS waves).
// Reports cycles per mad per wave (clock from hipDeviceAttributeClockRate).
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/ubench_mad.hip -o tools/ubench_mad
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

template <int NCH>
__global__ void __launch_bounds__(256) k_mad(uint64_t* out, uint32_t a0, uint32_t b0, int iters) {
  uint64_t acc[NCH];
  uint32_t b = b0 ^ blockIdx.x;
#pragma unroll
  for (int c = 0; c < NCH; ++c) acc[c] = a0 + c + threadIdx.x;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int u = 0; u < 64 / NCH; ++u)
#pragma unroll
      for (int c = 0; c < NCH; ++c) acc[c] = (uint64_t)(uint32_t)acc[c] * (b + u) + acc[c];
  }
  uint64_t s = 0;
#pragma unroll
  for (int c = 0; c < NCH; ++c) s ^= acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
  int clk_khz = 0;
  hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, 0);
  int ncu = 0;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  uint64_t* out;
  hipMalloc(&out, (size_t)ncu * 8 * 256 * 8);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int iters = 4000;
  for (int wps : {1, 2, 4}) {
    for (int nch : {1, 2, 4}) {
      // blocks of 256 threads = 4 waves = one wave per SIMD of one CU
      const int blocks = ncu * wps;
      auto launch = [&]() {
        if (nch == 1) hipLaunchKernelGGL(k_mad<1>, dim3(blocks), dim3(256), 0, 0, out, 3u, 5u, iters);
        if (nch == 2) hipLaunchKernelGGL(k_mad<2>, dim3(blocks), dim3(256), 0, 0, out, 3u, 5u, iters);
        if (nch == 4) hipLaunchKernelGGL(k_mad<4>, dim3(blocks), dim3(256), 0, 0, out, 3u, 5u, iters);
      };
      launch();
      hipDeviceSynchronize();
      hipEventRecord(e0);
      launch();
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      const double mads_per_wave = 64.0 * iters;
      const double cyc = ms * 1e-3 * clk_khz * 1e3;
      // per SIMD: wps waves each issuing mads_per_wave
      std::printf("{\"waves_per_simd\":%d,\"chains\":%d,\"cycles_per_mad_per_simd\":%.2f,\"cycles_per_mad_per_wave\":%.2f,\"chip_mads_per_s\":%.3e}\n",
                  wps, nch, cyc / (mads_per_wave * wps), cyc / mads_per_wave,
                  mads_per_wave * blocks * 4 * 64 / (ms * 1e-3));
    }
  }
  return 0;
}
