// ubench_issue.hip — chip-wide issue cost of the VALU instructions that make up the MSM's
// mixed addition (tools/isa_count.py mix): v_mad_u64_u32, v_lshrrev_b64, v_lshl_add_u64,
// v_and_b32, v_add_u32, v_mul_lo_u32, v_ashrrev_i32. Each kernel runs 8 independent chains
// of ONE instruction per lane (inline asm, so the instruction is exactly the named one), at
// 4 waves per SIMD on every CU; cycles per wave-instruction per SIMD at the reported clock.
// (The mad chains are plain C like ffr.hpp's: as inline asm the compiler pads each one with
// an s_nop.)
// bench.py prices the compiled loop body with these costs (the VALU issue-cycle roofline).
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/ubench_issue.hip -o tools/ubench_issue
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

constexpr int kChains = 8, kUnroll = 32;

template <int OP>
__global__ void __launch_bounds__(256) k_issue(uint64_t* out, uint32_t seed, int iters) {
  uint64_t x[kChains];
  uint32_t y[kChains];
#pragma unroll
  for (int c = 0; c < kChains; ++c) {
    x[c] = ((uint64_t)(seed + c) << 32) | (threadIdx.x * 7u + c);
    y[c] = seed * 3u + c + threadIdx.x;
  }
  const uint32_t k = seed | 1u;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
#pragma unroll
      for (int c = 0; c < kChains; ++c) {
        if constexpr (OP == 0) {
          // plain C (as ffr.hpp writes it): inline asm would add s_nop hazard padding
          x[c] = (uint64_t)(uint32_t)x[c] * (k + u) + x[c];
        } else if constexpr (OP == 1) {
          asm volatile("v_lshrrev_b64 %0, 3, %0" : "+v"(x[c]));
        } else if constexpr (OP == 2) {
          asm volatile("v_lshl_add_u64 %0, %0, 2, %0" : "+v"(x[c]));
        } else if constexpr (OP == 3) {
          asm volatile("v_and_b32 %0, %1, %0" : "+v"(y[c]) : "v"(k));
        } else if constexpr (OP == 4) {
          asm volatile("v_add_u32 %0, %1, %0" : "+v"(y[c]) : "v"(k));
        } else if constexpr (OP == 5) {
          asm volatile("v_mul_lo_u32 %0, %1, %0" : "+v"(y[c]) : "v"(k));
        } else {
          asm volatile("v_ashrrev_i32 %0, 1, %0" : "+v"(y[c]));
        }
      }
    }
  }
  uint64_t s = 0;
#pragma unroll
  for (int c = 0; c < kChains; ++c) s ^= x[c] ^ y[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int OP>
void run(const char* name, int ncu, int clk_khz, uint64_t* out, hipEvent_t e0, hipEvent_t e1) {
  const int iters = 2000, wps = 4, blocks = ncu * wps;
  hipLaunchKernelGGL(k_issue<OP>, dim3(blocks), dim3(256), 0, 0, out, 5u, iters);
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(e0);
  hipLaunchKernelGGL(k_issue<OP>, dim3(blocks), dim3(256), 0, 0, out, 5u, iters);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double per_wave = (double)iters * kUnroll * kChains;  // instructions per wave
  const double cyc = ms * 1e-3 * clk_khz * 1e3;
  std::printf("{\"op\":\"%s\",\"cycles_per_wave_instr_per_simd\":%.3f,\"chip_wave_instr_per_s\":%.4e,\"clock_khz\":%d}\n",
              name, cyc / (per_wave * wps), per_wave * blocks * 4 / (ms * 1e-3), clk_khz);
}

int main() {
  int clk_khz = 0, ncu = 0;
  (void)hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, 0);
  (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  uint64_t* out = nullptr;
  if (hipMalloc(&out, (size_t)ncu * 4 * 256 * 8) != hipSuccess) return 1;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  run<0>("v_mad_u64_u32", ncu, clk_khz, out, e0, e1);
  run<1>("v_lshrrev_b64", ncu, clk_khz, out, e0, e1);
  run<2>("v_lshl_add_u64", ncu, clk_khz, out, e0, e1);
  run<3>("v_and_b32", ncu, clk_khz, out, e0, e1);
  run<4>("v_add_u32", ncu, clk_khz, out, e0, e1);
  run<5>("v_mul_lo_u32", ncu, clk_khz, out, e0, e1);
  run<6>("v_ashrrev_i32", ncu, clk_khz, out, e0, e1);
  return 0;
}
