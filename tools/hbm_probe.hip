// hbm_probe.hip -- measured HBM streaming ceilings on MI355X for the RS traffic mix.
// Standalone (tools/, not product).  Build: hipcc --offload-arch=gfx950 -O3 -o hbm_probe hbm_probe.hip
// Each variant streams >= 2 GiB (beyond the 256 MiB Infinity Cache), timed by hipEvents.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ u32x4 ld(const u32x4* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}
template <bool NT>
__device__ __forceinline__ void st(u32x4* p, u32x4 v) {
  if constexpr (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

// copy: U independent 16-B loads per lane per iteration
template <bool NTL, bool NTS, int U>
__global__ __launch_bounds__(256) void copy_k(const u32x4* __restrict__ s, u32x4* __restrict__ d, size_t n) {
  const size_t stride = (size_t)gridDim.x * 256 * U;
  for (size_t base = (size_t)blockIdx.x * 256 * U + threadIdx.x; base < n; base += stride) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (base + u * 256 < n) v[u] = ld<NTL>(s + base + u * 256);
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (base + u * 256 < n) st<NTS>(d + base + u * 256, v[u]);
  }
}

// RS-shaped mix: per stripe 4 input rows and 2 output rows of R 16-B columns,
// wave per (stripe, 1 KiB block) like apply_kernel; XOR instead of GF math.
template <bool NTL, bool NTS>
__global__ __launch_bounds__(256) void mix42_k(const u32x4* __restrict__ in, u32x4* __restrict__ out, uint32_t N,
                                               uint32_t cols /*per shard*/) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
  const uint32_t nw = gridDim.x * 4;
  const uint32_t bps = cols / 64;
  const uint64_t tasks = (uint64_t)N * bps;
  for (uint64_t t = wave; t < tasks; t += nw) {
    const uint32_t s = t / bps, b = t % bps;
    const u32x4* ip = in + (uint64_t)s * 6 * cols + b * 64 + lane;
    u32x4 x0 = ld<NTL>(ip), x1 = ld<NTL>(ip + cols), x2 = ld<NTL>(ip + 2 * cols), x3 = ld<NTL>(ip + 3 * cols);
    st<NTS>(const_cast<u32x4*>(ip) + 4 * cols, x0 ^ x1);
    st<NTS>(const_cast<u32x4*>(ip) + 5 * cols, x2 ^ x3);
  }
}

template <typename F>
float timeit(F f, int iters) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  for (int i = 0; i < 3; ++i) f(i);
  (void)hipEventRecord(a);
  for (int i = 0; i < iters; ++i) f(i);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms;
  (void)hipEventElapsedTime(&ms, a, b);
  return ms / iters;
}

int main() {
  hipDeviceProp_t prop;
  (void)hipGetDeviceProperties(&prop, 0);
  const int cus = prop.multiProcessorCount;
  const size_t bytes = size_t(1) << 30;  // 1 GiB src + 1 GiB dst
  u32x4 *s, *d;
  if (hipMalloc(&s, bytes) || hipMalloc(&d, bytes)) return 1;
  (void)hipMemset(s, 1, bytes);
  (void)hipMemset(d, 0, bytes);
  const size_t n = bytes / 16;
  auto copy = [&](auto kern, int U, int bpc, const char* name) {
    const unsigned grid = cus * bpc;
    float ms = timeit([&](int) { hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, s, d, n); }, 10);
    printf("copy %-22s U=%d blocks/CU=%2d : %7.1f GB/s\n", name, U, bpc, 2.0 * bytes / ms / 1e6);
  };
  for (int bpc : {2, 4, 8, 16}) {
    copy(copy_k<false, false, 1>, 1, bpc, "plain/plain");
    copy(copy_k<true, true, 1>, 1, bpc, "nt/nt");
    copy(copy_k<false, false, 4>, 4, bpc, "plain/plain");
    copy(copy_k<true, true, 4>, 4, bpc, "nt/nt");
    copy(copy_k<false, true, 4>, 4, bpc, "plain/nt");
    copy(copy_k<true, false, 4>, 4, bpc, "nt/plain");
  }
  // RS-shaped 4:2 mix over 6 rotating 384 MiB batches (N=65536, S=1 KiB)
  const uint32_t N = 65536, cols = 64;
  const size_t batch = (size_t)N * 6 * cols * 16;
  std::vector<u32x4*> bufs(6);
  for (auto& p : bufs)
    if (hipMalloc(&p, batch)) return 1;
  for (auto& p : bufs) (void)hipMemset(p, 7, batch);
  auto mix = [&](auto kern, int bpc, const char* name) {
    const unsigned grid = cus * bpc;
    float ms = timeit([&](int i) { hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, bufs[i % 6], bufs[i % 6], N, cols); }, 30);
    printf("mix42 %-20s blocks/CU=%2d : %7.1f GB/s (%.1f us)\n", name, bpc, (double)N * 6 * cols * 16 / ms / 1e6, ms * 1e3);
  };
  for (int bpc : {2, 4, 7, 8, 16}) {
    mix(mix42_k<false, false>, bpc, "plain/plain");
    mix(mix42_k<true, true>, bpc, "nt/nt");
    mix(mix42_k<false, true>, bpc, "plain/nt");
  }
  return 0;
}
