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

// ---- experiment: one lazy full addition on the 4 lanes of a quad ----------------------
// Lanes 4i .. 4i + 3 hold the same operands and end with the same result; each round every
// lane forms ONE of the independent products of g1r_add_lazy_sl (operands picked per lane)
// and the results are broadcast through DPP quad permutations: 4 rounds (the 4th a fused
// product pair) instead of 13 products. Bit-identical to g1r_add_lazy, but a lone wave
// gains only 12.4 -> 9.8 us per dependent addition: one product alone in a round is
// latency-bound (~2.4 us, ~3x its issue cost), and the serial formula's critical path is
// itself ~5 dependent products. Kept here, not in the product (round-3 DESIGN §3).
template <int K>
__device__ __forceinline__ RFp rx_quad_bcast(const RFp& v) {  // lane K of the quad, to all 4
  constexpr int kCtrl = K | (K << 2) | (K << 4) | (K << 6);       // quad_perm [K, K, K, K]
  RFp r;
#pragma unroll
  for (int i = 0; i < RxShape<FpCfg>::L; ++i)
    r.v[i] = (uint32_t)__builtin_amdgcn_mov_dpp((int)v.v[i], kCtrl, 0xF, 0xF, false);
  return r;
}

__device__ __forceinline__ RFp rx_sel4(uint32_t k, const RFp& a0, const RFp& a1, const RFp& a2,
                                       const RFp& a3) {
  RFp r;
#pragma unroll
  for (int i = 0; i < RxShape<FpCfg>::L; ++i)
    r.v[i] = k == 0 ? a0.v[i] : k == 1 ? a1.v[i] : k == 2 ? a2.v[i] : a3.v[i];
  return r;
}

__device__ __forceinline__ G1R g1r_add_lazy_quad(const G1R& p, const G1R& q) {
  const uint32_t k = __lane_id() & 3;
  // round 1: U1 = X1 ZZ2, U2 = X2 ZZ1, S1 = Y1 ZZZ2, S2 = Y2 ZZZ1
  const RFp m1 = rx_mul(rx_sel4(k, p.X, q.X, p.Y, q.Y), rx_sel4(k, q.ZZ, p.ZZ, q.ZZZ, p.ZZZ));
  const RFp U1 = rx_quad_bcast<0>(m1), S1 = rx_quad_bcast<2>(m1);
  const RFp P = rx_sub_u<FpCfg, 3>(rx_quad_bcast<1>(m1), U1);  // U2 - U1 + 3p in (p, 5p)
  const RFp R = rx_sub_u<FpCfg, 3>(rx_quad_bcast<3>(m1), S1);  // S2 - S1 + 3p in (p, 5p)
  // round 2: PP = P^2, RR = R^2, ZZ12 = ZZ1 ZZ2, ZZZ12 = ZZZ1 ZZZ2
  const RFp m2 = rx_mul(rx_sel4(k, P, R, p.ZZ, p.ZZZ), rx_sel4(k, P, R, q.ZZ, q.ZZZ));
  const RFp PP = rx_quad_bcast<0>(m2), ZZ12 = rx_quad_bcast<2>(m2);
  // round 3: PPP = P PP, Q = U1 PP, ZZ3 = ZZ12 PP (lane 3 repeats lane 2's product)
  const RFp m3 = rx_mul(rx_sel4(k, P, U1, ZZ12, ZZ12), PP);
  const RFp PPP = rx_quad_bcast<0>(m3), Q = rx_quad_bcast<1>(m3);
  G1R r;
  r.ZZ = rx_quad_bcast<2>(m3);
  r.X = rx_sub2_n<FpCfg, 6>(rx_quad_bcast<1>(m2), PPP, Q);  // RR + 6p - PPP - 2Q in (0, 8p)
  // round 4: lane 0 ZZZ3 = ZZZ12 PPP (+ 0 PPP); lane 1 Y3 = R (Q - X3 + 10p) + (5p - S1) PPP
  const RFp zero = rx_zero<FpCfg>();
  const RFp m4 = rx_mul_add(rx_sel4(k, rx_quad_bcast<3>(m2), R, R, R),
                            rx_sel4(k, PPP, rx_sub_u<FpCfg, 10>(Q, r.X), zero, zero),
                            rx_sel4(k, zero, rx_sub_u<FpCfg, 5>(zero, S1), zero, zero), PPP);
  r.ZZZ = rx_quad_bcast<0>(m4);
  r.Y = rx_quad_bcast<1>(m4);
  return rx_is_zero(r.ZZ) ? g1r_add_lazy_fix(p, q, r.X) : r;  // rare branch (uniform per quad)
}

// quad-cooperative chains: quad i (lanes 4i .. 4i + 3) runs the chain of thread i of k_chain
__global__ void __launch_bounds__(256, 1) k_chain_quad(const G1xyzz* __restrict__ in, G1xyzz* __restrict__ out, int n) {
  const uint32_t t = (blockIdx.x * blockDim.x + threadIdx.x) >> 2;
  G1R acc = ld_g1r(&in[t % kPts]);
  for (int i = 0; i < n; ++i) acc = g1r_add_lazy_quad(acc, ld_g1r(&in[(t + 7 * i + 1) % kPts]));
  if ((threadIdx.x & 3) == 0) st_g1r(&out[t], acc);
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
  CHECK(hipMalloc(&dout, sizeof(G1xyzz) * 16384 * 64));  // one record per thread of the largest grid
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
  // the same lone-wave chain right after a heavy full-chip kernel (as the MSM's tail runs
  // right after k_accumulate): does the clock the heavy kernel left behind slow it down?
  for (int rep = 0; rep < 3; ++rep) {
    hipEvent_t a, b, c;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    CHECK(hipEventCreate(&c));
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(a));
    hipLaunchKernelGGL((k_chain<1, 1>), dim3(16384), dim3(64), 0, 0, din, dout, 64);
    CHECK(hipEventRecord(b));
    hipLaunchKernelGGL((k_chain<1, 1>), dim3(1), dim3(64), 0, 0, din, dout, 64);
    CHECK(hipEventRecord(c));
    CHECK(hipEventSynchronize(c));
    float hot = 0, lone = 0;
    CHECK(hipEventElapsedTime(&hot, a, b));
    CHECK(hipEventElapsedTime(&lone, b, c));
    std::printf("after a %.2f ms full-chip chain: lone-wave chain %.2f us per dependent add\n", hot,
                1e3 * lone / 64);
  }
  {  // quad-cooperative lazy addition: same values as g1r_add_lazy, time per dependent add
    const int n = 64;
    float ms = timeit([&] { hipLaunchKernelGGL((k_chain<1, 1>), dim3(4), dim3(64), 0, 0, din, dout, n); });
    std::vector<uint32_t> ref(256 * 48), got(256 * 48);
    CHECK(hipMemcpy(ref.data(), dout, ref.size() * 4, hipMemcpyDeviceToHost));
    float mq = timeit([&] { hipLaunchKernelGGL(k_chain_quad, dim3(16), dim3(64), 0, 0, din, dout, n); });
    CHECK(hipMemcpy(got.data(), dout, got.size() * 4, hipMemcpyDeviceToHost));
    std::printf("quad add: %s vs g1r_add_lazy on 256 chains; lone wave %.2f us (quads) vs %.2f us per dependent add\n",
                ref == got ? "bit-identical" : "MISMATCH", 1e3 * mq / n, 1e3 * ms / n);
    CHECK(hipFuncGetAttributes(&fa, (const void*)k_chain_quad));
    std::printf("  quad chain kernel %d VGPRs (%d spill bytes)\n", fa.numRegs, (int)fa.localSizeBytes);
  }
  if (run("g1r_add", k_chain<0, 1>, k_tree<0, 1>)) return 1;
  if (run("g1r_add_lazy", k_chain<1, 1>, k_tree<1, 1>)) return 1;
  if (run("g1r_add_lazy, 2 waves/SIMD cap", k_chain<1, 2>, k_tree<1, 2>)) return 1;
  if (run("g1r_add, 2 waves/SIMD cap", k_chain<0, 2>, k_tree<0, 2>)) return 1;
  return 0;
}
