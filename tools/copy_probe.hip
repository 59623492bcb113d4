// copy_probe.hip -- streaming-copy sweep for the bench's HBM yardstick (tools/, not product).
//
// The RS kernels move ~402 MB per launch (RS(4+2) 4 KiB bench batch) over 6 rotating
// batches; the old yardstick copied one 1 GiB buffer into another.  This sweep times
// copies of the same traffic per launch, rotating over buffer pairs the same way, for
// several task shapes, loads in flight per lane and workgroups per CU, so the copy that
// bench.py and rs_device_copy use is the fastest measured one.
//   block:  block-contiguous (lane l of block b loads b*256*U + u*256 + l, as copy_kernel)
//   wave:   wave-contiguous  (wave w copies U KiB: u*64 + lane of its U KiB chunk)
//   wave-sc1: as wave, stores device-scope write-through (cpol SC1) instead of NT
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/copy_probe tools/copy_probe.hip
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                     \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                               \
    }                                                                             \
  } while (0)

template <int U>
__global__ __launch_bounds__(256) void copy_block(const u32x4* __restrict__ src, u32x4* __restrict__ dst, uint64_t n16) {
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * 256u * U;
  for (uint64_t base = static_cast<uint64_t>(blockIdx.x) * 256u * U + threadIdx.x; base < n16; base += stride) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (base + u * 256u < n16) v[u] = __builtin_nontemporal_load(src + base + u * 256u);
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (base + u * 256u < n16) __builtin_nontemporal_store(v[u], dst + base + u * 256u);
  }
}

template <int U, int CPOL>
__global__ __launch_bounds__(256) void copy_wave(const u32x4* __restrict__ src, u32x4* __restrict__ dst, uint64_t n16) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t wave = static_cast<uint64_t>(blockIdx.x) * 4u + (threadIdx.x >> 6);
  const uint64_t nw = static_cast<uint64_t>(gridDim.x) * 4u;
  const uint64_t chunk = 64u * U;  // 16-B elements per wave task
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<u32x4*>(src), 0, 0x7FFFFFFF, 0x00020000);
  const auto rd = __builtin_amdgcn_make_buffer_rsrc(dst, 0, 0x7FFFFFFF, 0x00020000);
  for (uint64_t t = wave; t * chunk < n16; t += nw) {
    const uint32_t base = static_cast<uint32_t>((t * chunk + lane) * 16u);
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
      v[u] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, base + u * 1024u, 0, 2));
#pragma unroll
    for (int u = 0; u < U; ++u) __builtin_amdgcn_raw_buffer_store_b128(v[u], rd, base + u * 1024u, 0, CPOL);
  }
}

__global__ void fill(uint32_t* p, uint64_t n, uint32_t seed) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) {
    uint32_t x = static_cast<uint32_t>(i) * 2654435761u ^ seed;
    x ^= x >> 13;
    x *= 0x5bd1e995u;
    x ^= x >> 15;
    p[i] = x;
  }
}

struct Variant {
  const char* name;
  const void* fn;
  int U;
  bool wave;
};

int main(int argc, char** argv) {
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  // per launch: copy `half` bytes (traffic 2*half), rotating over `pairs` buffer pairs
  struct Foot {
    const char* name;
    uint64_t half;
    int pairs;
  } feet[] = {{"201MB x6 rot", 201326592ull, 6}, {"1GiB x1", 1ull << 30, 1}};
  Variant vs[] = {
      {"block U=4", (const void*)&copy_block<4>, 4, false},
      {"block U=8", (const void*)&copy_block<8>, 8, false},
      {"wave U=2", (const void*)&copy_wave<2, 2>, 2, true},
      {"wave U=4", (const void*)&copy_wave<4, 2>, 4, true},
      {"wave U=8", (const void*)&copy_wave<8, 2>, 8, true},
      {"wave-sc1 U=4", (const void*)&copy_wave<4, 16>, 4, true},
      {"wave-nt|sc1 U=4", (const void*)&copy_wave<4, 18>, 4, true},
  };
  const int grids[] = {1, 2, 4, 8, 16};
  const double min_ms = argc > 1 ? std::atof(argv[1]) : 100.0;
  std::printf("CUs %d, min timed %.0f ms per point\n", cus, min_ms);
  for (const Foot& f : feet) {
    std::vector<void*> a(f.pairs), b(f.pairs);
    for (int i = 0; i < f.pairs; ++i) {
      CK(hipMalloc(&a[i], f.half));
      CK(hipMalloc(&b[i], f.half));
      hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, static_cast<uint32_t*>(a[i]), f.half / 4, 77u + i);
    }
    CK(hipDeviceSynchronize());
    const uint64_t n16 = f.half / 16;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (const Variant& v : vs) {
      for (int g : grids) {
        const uint64_t tasks = v.wave ? (n16 + 64u * v.U - 1) / (64u * v.U) : (n16 + 256u * v.U - 1) / (256u * v.U);
        const uint64_t need = v.wave ? (tasks + 3) / 4 : tasks;
        const uint32_t grid = static_cast<uint32_t>(std::min<uint64_t>(need, static_cast<uint64_t>(cus) * g));
        const u32x4* s0 = nullptr;
        u32x4* d0 = nullptr;
        void* args[] = {&s0, &d0, const_cast<uint64_t*>(&n16)};
        auto run = [&](int iters) {
          for (int it = 0; it < iters; ++it) {
            s0 = static_cast<const u32x4*>(a[it % f.pairs]);
            d0 = static_cast<u32x4*>(b[it % f.pairs]);
            CK(hipLaunchKernel(v.fn, dim3(grid), dim3(256), args, 0, 0));
          }
        };
        run(6);
        CK(hipEventRecord(e0, 0));
        run(12);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms = 0.f;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const int iters = std::max(12, static_cast<int>(min_ms / (ms / 12.0)) / f.pairs * f.pairs);
        CK(hipEventRecord(e0, 0));
        run(iters);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
        std::printf("%-14s %-16s G=%-2d %8.1f GB/s  (%d launches, %.1f us each)\n", f.name, v.name, g,
                    2.0 * f.half * iters / (ms * 1e-3) / 1e9, iters, ms * 1e3 / iters);
        std::fflush(stdout);
      }
    }
    for (int i = 0; i < f.pairs; ++i) {
      CK(hipFree(a[i]));
      CK(hipFree(b[i]));
    }
  }
  return 0;
}
