// hbm_probe2.hip -- which access pattern gives the RS(4+2) traffic mix the most HBM
// bandwidth on MI355X?  No GF math (XOR only): an upper bound for the RS kernels.
// Patterns:
//   layout   unified : stripe = 6 slots x S contiguous (data 0..3, parity 4..5)
//            split   : data region N x 4S contiguous, parity region N x 2S contiguous
//   U        tasks (1 KiB column blocks) per wave per loop trip (loads in flight)
//   mapping  gs = grid-stride over tasks, ct = contiguous task range per wave
// Build: hipcc --offload-arch=gfx950 -O3 -o hbm_probe2 hbm_probe2.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ u32x4 ld(const u32x4* p) { return __builtin_nontemporal_load(p); }
__device__ __forceinline__ void st(u32x4* p, u32x4 v) { __builtin_nontemporal_store(v, p); }

struct Geo {
  u32x4* data;     // unified: base of stripes; split: data region
  u32x4* parity;   // split: parity region
  uint32_t N, cols;  // cols = 16-B columns per shard
  bool split;
};

template <int U, bool CT>
__global__ __launch_bounds__(256) void mix_k(Geo g) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
  const uint32_t nw = gridDim.x * 4;
  const uint32_t bps = g.cols / 64;
  const uint64_t tasks = (uint64_t)g.N * bps;
  uint64_t t, tend, step;
  if (CT) {
    t = tasks * wave / nw;
    tend = tasks * (wave + 1) / nw;
    step = 1;
  } else {
    t = wave;
    tend = tasks;
    step = nw;
  }
  for (; t < tend; t += step * U) {
    u32x4 x[U][4];
    u32x4* ob[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      uint64_t tt = t + u * step;
      if (tt >= tend) tt = t;
      const uint32_t s = tt / bps, b = tt % bps;
      const u32x4* ip;
      if (g.split) {
        ip = g.data + (uint64_t)s * 4 * g.cols + b * 64 + lane;
        ob[u] = g.parity + (uint64_t)s * 2 * g.cols + b * 64 + lane;
      } else {
        ip = g.data + (uint64_t)s * 6 * g.cols + b * 64 + lane;
        ob[u] = const_cast<u32x4*>(ip) + 4 * g.cols;
      }
#pragma unroll
      for (int c = 0; c < 4; ++c) x[u][c] = ld(ip + c * g.cols);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (t + u * step < tend) {
        st(ob[u], x[u][0] ^ x[u][1]);
        st(ob[u] + g.cols, x[u][2] ^ x[u][3]);
      }
    }
  }
}

__global__ __launch_bounds__(256) void read4_k(Geo g, u32x4* sink) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wave = blockIdx.x * 4 + (threadIdx.x >> 6);
  const uint32_t nw = gridDim.x * 4;
  const uint32_t bps = g.cols / 64;
  const uint64_t tasks = (uint64_t)g.N * bps;
  u32x4 acc = {0, 0, 0, 0};
  for (uint64_t t = wave; t < tasks; t += nw) {
    const uint32_t s = t / bps, b = t % bps;
    const u32x4* ip = g.data + (uint64_t)s * 4 * g.cols + b * 64 + lane;
#pragma unroll
    for (int c = 0; c < 4; ++c) acc ^= ld(ip + c * g.cols);
  }
  if ((acc[0] ^ acc[1] ^ acc[2] ^ acc[3]) == 0x12345678u) sink[0] = acc;
}

__global__ __launch_bounds__(256) void write2_k(Geo g) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wave = blockIdx.x * 4 + (threadIdx.x >> 6);
  const uint32_t nw = gridDim.x * 4;
  const uint32_t bps = g.cols / 64;
  const uint64_t tasks = (uint64_t)g.N * bps;
  const u32x4 v = {lane, wave, 1, 2};
  for (uint64_t t = wave; t < tasks; t += nw) {
    const uint32_t s = t / bps, b = t % bps;
    u32x4* op = g.parity + (uint64_t)s * 2 * g.cols + b * 64 + lane;
    st(op, v);
    st(op + g.cols, v);
  }
}

int main() {
  hipDeviceProp_t prop;
  (void)hipGetDeviceProperties(&prop, 0);
  const int cus = prop.multiProcessorCount;
  struct Shape {
    uint32_t N, cols;
    const char* name;
  };
  const Shape shapes[] = {{65536, 64, "4KiB stripes"}, {16384, 1024, "64KiB stripes"}};
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  u32x4* sink;
  (void)hipMalloc(&sink, 64);
  for (const Shape& sh : shapes) {
    const size_t stripe = (size_t)sh.cols * 16 * 6;
    const size_t bytes = (size_t)sh.N * stripe;  // 384 MiB (4K) / 1.5 GiB (64K)
    const int nb = bytes < (size_t(1) << 30) ? 6 : 2;
    std::vector<u32x4*> bufs(nb);
    for (auto& p : bufs) {
      if (hipMalloc(&p, bytes)) return 1;
      (void)hipMemset(p, 3, bytes);
    }
    auto geo = [&](int i, bool split) {
      Geo g;
      g.data = bufs[i % nb];
      g.parity = reinterpret_cast<u32x4*>(reinterpret_cast<char*>(bufs[i % nb]) + (size_t)sh.N * sh.cols * 16 * 4);
      g.N = sh.N;
      g.cols = sh.cols;
      g.split = split;
      return g;
    };
    auto bench = [&](const char* name, auto launch) {
      for (int i = 0; i < 3; ++i) launch(i);
      (void)hipEventRecord(e0);
      const int it = 20;
      for (int i = 0; i < it; ++i) launch(i);
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      return ms / it;
    };
    printf("== %s (%.0f MiB per batch, %d batches)\n", sh.name, bytes / 1048576.0, nb);
    for (int bpc : {1, 2, 3, 4, 8}) {
      const unsigned grid = cus * bpc;
      float ms;
#define RUN(U, CT, SPLIT)                                                                            \
  ms = bench("", [&](int i) { hipLaunchKernelGGL((mix_k<U, CT>), dim3(grid), dim3(256), 0, 0, geo(i, SPLIT)); }); \
  printf("mix42 %-7s U=%d %s bpc=%d : %7.1f GB/s\n", SPLIT ? "split" : "unified", U, CT ? "ct" : "gs", bpc,          \
         bytes / ms / 1e6);
      RUN(1, false, false) RUN(1, false, true) RUN(2, false, false) RUN(2, false, true)
      RUN(1, true, false) RUN(1, true, true) RUN(2, true, true) RUN(4, false, true)
      ms = bench("", [&](int i) { hipLaunchKernelGGL(read4_k, dim3(grid), dim3(256), 0, 0, geo(i, true), sink); });
      printf("read4 only        bpc=%d : %7.1f GB/s\n", bpc, bytes * 4.0 / 6 / ms / 1e6);
      ms = bench("", [&](int i) { hipLaunchKernelGGL(write2_k, dim3(grid), dim3(256), 0, 0, geo(i, true)); });
      printf("write2 only       bpc=%d : %7.1f GB/s\n", bpc, bytes * 2.0 / 6 / ms / 1e6);
    }
    for (auto p : bufs) (void)hipFree(p);
  }
  return 0;
}
