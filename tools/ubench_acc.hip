// ubench_acc.hip — variants of the MSM accumulation loop (msm.hip k_accumulate) on a
// synthetic workload of the bench's shape: a 16M-entry affine table (R' domain values,
// random coordinates: the instruction stream is the same as for curve points), tasks of
// CH consecutive sorted entries with random table indices. Reports point adds/s for
//   v0: the production loop (index load -> point load -> madd)
//   v1: software-pipelined: the next index and point are loaded before the current madd
//   v2: v0 with a 3-waves/SIMD register budget
//   v3: v1 with a 3-waves/SIMD register budget
//   v4: the production loop (msm.hip): lazy straight-line mixed addition with the
//       exceptional cases repaired after (g1r_madd_lazy_sl/_fix); compared with v0 mod p
//   v5: v4 with a 3-waves/SIMD register budget
//   (tried: ordering the products for short operand lifetimes — no change, the scheduler
//   reorders anyway)
//   (a variant with a two-chain multiply — column k+1's products in a second accumulator — ran
//   5% slower than v4: v_mad_u64_u32's dependent latency equals its issue cost, see
//   tools/ubench_mad.hip)
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/ubench_acc.hip -o tools/ubench_acc
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
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

__device__ __forceinline__ void ld_fp(const uint32_t* p, Fp& r) {
  const uint4* q = reinterpret_cast<const uint4*>(p);
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const uint4 a = q[i];
    r.v[4 * i] = a.x;
    r.v[4 * i + 1] = a.y;
    r.v[4 * i + 2] = a.z;
    r.v[4 * i + 3] = a.w;
  }
}

__device__ __forceinline__ void acc_plain(const uint2 task, const uint32_t* __restrict__ sorted,
                                          const G1Affine* __restrict__ table, G1xyzz* out) {
  G1R acc = g1r_infinity();
  for (uint32_t e = task.x; e < task.x + task.y; ++e) {
    const uint32_t code = sorted[e];
    RFp x, y;
    ld_g1r_aff(&table[code & 0x7fffffffu], x, y);
    if (code & 0x80000000u) y = rx_neg(y);
    acc = g1r_add_affine(acc, x, y);
  }
  st_g1r(out, acc);
}

__device__ __forceinline__ void acc_pipe(const uint2 task, const uint32_t* __restrict__ sorted,
                                         const G1Affine* __restrict__ table, G1xyzz* out) {
  G1R acc = g1r_infinity();
  const uint32_t end = task.x + task.y;
  uint32_t code = sorted[task.x];
  Fp px, py;
  {
    const uint32_t* q = reinterpret_cast<const uint32_t*>(&table[code & 0x7fffffffu]);
    ld_fp(q, px);
    ld_fp(q + 12, py);
  }
  for (uint32_t e = task.x; e < end; ++e) {
    RFp x = rx_unpack(px), y = rx_unpack(py);
    if (code & 0x80000000u) y = rx_neg(y);
    if (e + 1 < end) {  // issue the next loads before the madd
      code = sorted[e + 1];
      const uint32_t* q = reinterpret_cast<const uint32_t*>(&table[code & 0x7fffffffu]);
      ld_fp(q, px);
      ld_fp(q + 12, py);
    }
    acc = g1r_add_affine(acc, x, y);
  }
  st_g1r(out, acc);
}

__device__ __forceinline__ void acc_lazy(const uint2 task, const uint32_t* __restrict__ sorted,
                                         const G1Affine* __restrict__ table, G1xyzz* out) {
  // msm.hip k_accumulate's loop: first entry initialises, straight-line lazy madd, rare
  // ZZ3 == 0 repair with the point reloaded
  const uint32_t end = task.x + task.y;
  G1R acc;
  {
    const uint32_t c0 = sorted[task.x];
    ld_g1r_aff(&table[c0 & 0x7fffffffu], acc.X, acc.Y);
    if (c0 & 0x80000000u) acc.Y = rx_neg(acc.Y);
    acc.ZZ = rx_one<FpCfg>();
    acc.ZZZ = rx_one<FpCfg>();
  }
  uint32_t code = task.x + 1 < end ? sorted[task.x + 1] : 0u;
  Fp px, py;
  {
    const uint32_t* q = reinterpret_cast<const uint32_t*>(&table[code & 0x7fffffffu]);
    ld_fp(q, px);
    ld_fp(q + 12, py);
  }
  for (uint32_t e = task.x + 1; e < end; ++e) {
    const uint32_t cur = code;
    const RFp x = rx_unpack(px);
    RFp y = rx_unpack(py);
    if (e + 1 < end) {
      code = sorted[e + 1];
      const uint32_t* q = reinterpret_cast<const uint32_t*>(&table[code & 0x7fffffffu]);
      ld_fp(q, px);
      ld_fp(q + 12, py);
    }
    if (cur & 0x80000000u) y = rx_neg_lazy(y);
    const bool was_inf = g1r_is_inf(acc);
    G1R r = g1r_madd_lazy_sl(acc, x, y);
    if (rx_is_zero(r.ZZ)) {
      RFp xr, yr;
      ld_g1r_aff(&table[cur & 0x7fffffffu], xr, yr);
      if (cur & 0x80000000u) yr = rx_neg(yr);
      r = g1r_madd_lazy_fix(was_inf, r, xr, yr);
    }
    acc = r;
  }
  st_g1r(out, g1r_lazy_finish(acc));
}

__global__ void __launch_bounds__(256) k_v0(const uint2* tasks, uint32_t ntasks,
                                            const uint32_t* sorted, const G1Affine* table,
                                            G1xyzz* out) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t < ntasks) acc_plain(tasks[t], sorted, table, &out[t]);
}
__global__ void __launch_bounds__(256) k_v1(const uint2* tasks, uint32_t ntasks,
                                            const uint32_t* sorted, const G1Affine* table,
                                            G1xyzz* out) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t < ntasks) acc_pipe(tasks[t], sorted, table, &out[t]);
}
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3, 3)))
k_v2(const uint2* tasks, uint32_t ntasks, const uint32_t* sorted, const G1Affine* table,
     G1xyzz* out) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t < ntasks) acc_plain(tasks[t], sorted, table, &out[t]);
}
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3, 3)))
k_v3(const uint2* tasks, uint32_t ntasks, const uint32_t* sorted, const G1Affine* table,
     G1xyzz* out) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t < ntasks) acc_pipe(tasks[t], sorted, table, &out[t]);
}

__global__ void __launch_bounds__(256) k_v4(const uint2* tasks, uint32_t ntasks,
                                            const uint32_t* sorted, const G1Affine* table,
                                            G1xyzz* out) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t < ntasks) acc_lazy(tasks[t], sorted, table, &out[t]);
}
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3, 3)))
k_v5(const uint2* tasks, uint32_t ntasks, const uint32_t* sorted, const G1Affine* table,
     G1xyzz* out) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t < ntasks) acc_lazy(tasks[t], sorted, table, &out[t]);
}

// a, b in [0, 2p) as 12 words: equal mod p
static bool eq_mod_p(const uint32_t* a, const uint32_t* b) {
  if (!memcmp(a, b, 48)) return true;
  uint32_t d[12];
  uint64_t br = 0;
  const uint32_t *hi = a, *lo = b;
  for (int i = 11; i >= 0; --i)
    if (a[i] != b[i]) {
      if (a[i] < b[i]) hi = b, lo = a;
      break;
    }
  for (int i = 0; i < 12; ++i) {
    const uint64_t t = (uint64_t)hi[i] - lo[i] - br;
    d[i] = (uint32_t)t;
    br = (t >> 63) & 1;
  }
  return !memcmp(d, FpCfg::P, 48);
}

static uint64_t g_s = 0x9e37;
static uint32_t rnd() {
  g_s += 0x9E3779B97F4A7C15ull;
  uint64_t z = g_s;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return (uint32_t)(z ^ (z >> 31));
}

int main() {
  const uint32_t npts = 16u << 20;   // 2^20 points x 16 windows
  const uint32_t entries = 16u << 20;  // one MSM of 2^20 scalars x 16 windows
  const uint32_t CH = 32, ntasks = entries / CH;
  std::vector<G1Affine> tab(npts);
  for (auto& p : tab) {
    for (int k = 0; k < 12; ++k) {
      p.x.v[k] = rnd();
      p.y.v[k] = rnd();
    }
    p.x.v[11] &= 0x0fffffffu;  // < p
    p.y.v[11] &= 0x0fffffffu;
  }
  std::vector<uint32_t> sorted(entries);
  for (auto& s : sorted) s = (rnd() % npts) | (rnd() & 0x80000000u);
  std::vector<uint2> tasks(ntasks);
  for (uint32_t t = 0; t < ntasks; ++t) tasks[t] = make_uint2(t * CH, CH);
  G1Affine* dtab;
  uint32_t* dsorted;
  uint2* dtasks;
  G1xyzz* dout;
  CHECK(hipMalloc(&dtab, (size_t)npts * sizeof(G1Affine)));
  CHECK(hipMalloc(&dsorted, (size_t)entries * 4));
  CHECK(hipMalloc(&dtasks, (size_t)ntasks * 8));
  CHECK(hipMalloc(&dout, (size_t)ntasks * sizeof(G1xyzz)));
  CHECK(hipMemcpy(dtab, tab.data(), (size_t)npts * sizeof(G1Affine), hipMemcpyHostToDevice));
  CHECK(hipMemcpy(dsorted, sorted.data(), (size_t)entries * 4, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(dtasks, tasks.data(), (size_t)ntasks * 8, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  void (*ks[6])(const uint2*, uint32_t, const uint32_t*, const G1Affine*, G1xyzz*) = {k_v0, k_v1, k_v2, k_v3, k_v4, k_v5};
  const char* names[6] = {"v0_plain", "v1_pipelined", "v2_plain_w3", "v3_pipelined_w3", "v4_lazy", "v5_lazy_w3"};
  std::vector<G1xyzz> ref(ntasks), got(ntasks);
  for (int v = 0; v < 6; ++v) {
    const dim3 grid((ntasks + 255) / 256);
    hipLaunchKernelGGL(ks[v], grid, dim3(256), 0, 0, dtasks, ntasks, dsorted, dtab, dout);
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(e0));
    const int reps = 3;
    for (int r = 0; r < reps; ++r)
      hipLaunchKernelGGL(ks[v], grid, dim3(256), 0, 0, dtasks, ntasks, dsorted, dtab, dout);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    CHECK(hipMemcpy(v == 0 ? ref.data() : got.data(), dout, (size_t)ntasks * sizeof(G1xyzz),
                    hipMemcpyDeviceToHost));
    bool same = true;
    if (v) same = memcmp(ref.data(), got.data(), (size_t)ntasks * sizeof(G1xyzz)) == 0;
    if (v >= 4) {  // projective coordinates agree mod p (both in [0, 2p))
      same = true;
      for (uint32_t t = 0; t < ntasks && same; ++t) {
        const uint32_t* a = reinterpret_cast<const uint32_t*>(&ref[t]);
        const uint32_t* b = reinterpret_cast<const uint32_t*>(&got[t]);
        for (int c = 0; c < 4 && same; ++c) same = eq_mod_p(a + 12 * c, b + 12 * c);
      }
    }
    std::printf("{\"test\":\"%s\",\"ms_per_msm\":%.3f,\"adds_per_s\":%.4e,\"same_as_v0\":%s}\n",
                names[v], ms / reps, (double)entries * reps / (ms * 1e-3), same ? "true" : "false");
  }
  return 0;
}
