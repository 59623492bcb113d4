// hbm_probe4.hip -- compute-free ceiling of the RS(K+M) split-layout traffic for the
// K/M sweep (BASELINE configs[3]), 64 KiB stripes: reads K shards, writes M.
// Build: hipcc --offload-arch=gfx950 -O3 -o hbm_probe4 hbm_probe4.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int K, int M>
__global__ __launch_bounds__(256) void mix(const u32x4* __restrict__ d, u32x4* __restrict__ p, uint32_t N,
                                           uint32_t P16 /* pitch in 16-B units */, uint32_t bps) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
  const uint32_t nw = gridDim.x * 4;
  const uint32_t tasks = N * bps;
  for (uint32_t t = wave; t < tasks; t += nw) {
    const uint32_t s = t / bps, b = t % bps;
    if (b * 64 + lane >= P16) continue;  // columns past the slot: never touch
    const u32x4* ip = d + (uint64_t)s * K * P16 + b * 64 + lane;
    u32x4* op = p + (uint64_t)s * M * P16 + b * 64 + lane;
    u32x4 x[K];
#pragma unroll
    for (int c = 0; c < K; ++c) x[c] = __builtin_nontemporal_load(ip + c * P16);
#pragma unroll
    for (int r = 0; r < M; ++r) {
      u32x4 y = x[r];
#pragma unroll
      for (int c = 0; c < K; ++c) y ^= x[c] * (r + 1);  // cheap, keeps every load live
      __builtin_nontemporal_store(y, op + r * P16);
    }
  }
}

template <int K, int M>
void run(int cus, uint32_t S) {
  const uint32_t P = (S + 63) / 64 * 64, P16 = P / 16, bps = (P16 + 63) / 64;
  const uint32_t N = 16384;
  const size_t db = (size_t)N * K * P, pb = (size_t)N * M * P;
  const int nb = 2;
  std::vector<u32x4*> d(nb), p(nb);
  for (int i = 0; i < nb; ++i) {
    if (hipMalloc(&d[i], db) || hipMalloc(&p[i], pb)) return;
    (void)hipMemset(d[i], 1, db);
  }
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int bpc : {2, 4, 6, 8}) {
    const unsigned grid = cus * bpc;
    for (int i = 0; i < 2; ++i) hipLaunchKernelGGL((mix<K, M>), dim3(grid), dim3(256), 0, 0, d[i % nb], p[i % nb], N, P16, bps);
    (void)hipEventRecord(e0);
    for (int i = 0; i < 10; ++i) hipLaunchKernelGGL((mix<K, M>), dim3(grid), dim3(256), 0, 0, d[i % nb], p[i % nb], N, P16, bps);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    ms /= 10;
    printf("RS(%d+%d) S=%u compute-free bpc=%d: %7.1f GB/s (alg bytes %.0f MB)\n", K, M, S, bpc,
           (double)N * S * (K + M) / ms / 1e6, (double)N * S * (K + M) / 1e6);
  }
  for (int i = 0; i < nb; ++i) {
    (void)hipFree(d[i]);
    (void)hipFree(p[i]);
  }
}

int main() {
  hipDeviceProp_t prop;
  (void)hipGetDeviceProperties(&prop, 0);
  run<10, 4>(prop.multiProcessorCount, 6554);
  run<10, 4>(prop.multiProcessorCount, 6656);
  return 0;
}
