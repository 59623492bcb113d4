// pattern_probe.hip -- compute-free ceilings of the RS kernels' HBM access patterns
// (split layout: data [N, K, P], parity [N, M, P]), to separate memory-pattern
// limits from compute / issue limits.  Every kernel reads K shards and writes M
// per stripe with a trivial dependence (y = x[r] ^ x[c]*(r+1)) so no load is dead.
//
//   A  1 KiB tasks (64 columns x 16 B), all K loads then M stores, plain stores
//      behind `if (col < cols)` (round-1 hbm_probe4 shape)
//   B  as A, stores as raw buffer stores dropped by offset for lanes past the end
//      (apply_kernel's discipline), lanes past the end re-read the last column
//   C  2 KiB tasks (columns c and c+64 per lane), buffer stores (bitsliced shape)
//   D  as B, software-pipelined: task t+1's K loads are issued before task t's
//      stores (two register sets, loop unrolled by 2)
//   E  as B but one task = the whole stripe (loop over its blocks inside the wave)
//   copy: streaming copy of 1 GiB, U loads in flight per lane, G blocks per CU
//
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/pattern_probe tools/pattern_probe.hip
// Run:   tools/pattern_probe   (prints GB/s of algorithmic bytes N*S*(K+M))
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define CHECK(x)                                                         \
  do {                                                                   \
    hipError_t e_ = (x);                                                 \
    if (e_ != hipSuccess) {                                              \
      std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); \
      std::exit(1);                                                      \
    }                                                                    \
  } while (0)

struct Geo {
  const uint8_t* d;
  uint8_t* p;
  uint32_t N, S, P, cols, full;  // cols = ceil(S/16), full = S/16
  uint32_t sfull;                 // columns whose stores land (full, or whole 128-B lines)
};

__device__ __forceinline__ u32x4 ld(const uint8_t* p) { return __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p)); }

__device__ __forceinline__ const uint8_t* uni(const uint8_t* p) {
  const uint64_t v = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(v));
  const uint32_t hi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(v >> 32));
  return reinterpret_cast<const uint8_t*>((static_cast<uint64_t>(hi) << 32) | lo);
}

__device__ __forceinline__ void st_drop(uint8_t* base, uint32_t off, bool live, u32x4 v) {
  const auto r = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(uni(base)), 0, 0x7FFFFFFF, 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b128(v, r, live ? off : 0x80000000u, 0, 2);
}

template <int K, int M>
__global__ __launch_bounds__(256) void pA(Geo g) {
  const uint32_t lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
  const uint32_t nw = gridDim.x * 4, bps = (g.cols + 63) / 64, tasks = g.N * bps;
  for (uint32_t t = wave; t < tasks; t += nw) {
    const uint32_t s = t / bps, b = t - s * bps, col = b * 64 + lane;
    if (col >= g.cols) continue;
    const uint8_t* ip = g.d + (uint64_t)s * K * g.P + col * 16;
    uint8_t* op = g.p + (uint64_t)s * M * g.P + col * 16;
    u32x4 x[K];
#pragma unroll
    for (int c = 0; c < K; ++c) x[c] = ld(ip + (uint64_t)c * g.P);
#pragma unroll
    for (int r = 0; r < M; ++r) {
      u32x4 y = x[r];
#pragma unroll
      for (int c = 0; c < K; ++c) y ^= x[c] * (r + 1);
      __builtin_nontemporal_store(y, reinterpret_cast<u32x4*>(op + (uint64_t)r * g.P));
    }
  }
}

template <int K, int M>
__device__ __forceinline__ void task_load(const Geo& g, uint32_t s, uint32_t col, u32x4 (&x)[K], uint32_t* off) {
  *off = (col < g.cols ? col : g.cols - 1) * 16;
  const uint8_t* ip = uni(g.d + (uint64_t)s * K * g.P);
#pragma unroll
  for (int c = 0; c < K; ++c) x[c] = ld(ip + (uint64_t)c * g.P + *off);
}

template <int K, int M>
__device__ __forceinline__ void task_store(const Geo& g, uint32_t s, uint32_t col, uint32_t off, const u32x4 (&x)[K]) {
  uint8_t* ob = g.p + (uint64_t)s * M * g.P;
#pragma unroll
  for (int r = 0; r < M; ++r) {
    u32x4 y = x[r];
#pragma unroll
    for (int c = 0; c < K; ++c) y ^= x[c] * (r + 1);
    st_drop(ob + (uint64_t)r * g.P, col * 16, col < g.sfull, y);
  }
}

template <int K, int M>
__global__ __launch_bounds__(256) void pB(Geo g) {
  const uint32_t lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
  const uint32_t nw = gridDim.x * 4, bps = (g.cols + 63) / 64, tasks = g.N * bps;
  for (uint32_t t = wave; t < tasks; t += nw) {
    const uint32_t s = t / bps, b = t - s * bps, col = b * 64 + lane;
    u32x4 x[K];
    uint32_t off;
    task_load<K, M>(g, s, col, x, &off);
    task_store<K, M>(g, s, col, off, x);
  }
}

template <int K, int M>
__global__ __launch_bounds__(256) void pC(Geo g) {
  const uint32_t lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
  const uint32_t nw = gridDim.x * 4, bps = (g.cols + 127) / 128, tasks = g.N * bps;
  for (uint32_t t = wave; t < tasks; t += nw) {
    const uint32_t s = t / bps, b = t - s * bps, ca = b * 128 + lane, cb = ca + 64;
    u32x4 xa[K], xb[K];
    uint32_t oa, ob;
    task_load<K, M>(g, s, ca, xa, &oa);
    task_load<K, M>(g, s, cb, xb, &ob);
    task_store<K, M>(g, s, ca, oa, xa);
    task_store<K, M>(g, s, cb, ob, xb);
  }
}

template <int K, int M>
__global__ __launch_bounds__(256) void pD(Geo g) {
  const uint32_t lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
  const uint32_t nw = gridDim.x * 4, bps = (g.cols + 63) / 64, tasks = g.N * bps;
  u32x4 xa[K], xb[K];
  uint32_t oa = 0, ob = 0, sa = 0, sb = 0, ca = 0, cb = 0;
  uint32_t t = wave;
  if (t < tasks) {
    sa = t / bps;
    ca = (t - sa * bps) * 64 + lane;
    task_load<K, M>(g, sa, ca, xa, &oa);
  }
  while (t < tasks) {
    const uint32_t t1 = t + nw;
    if (t1 < tasks) {
      sb = t1 / bps;
      cb = (t1 - sb * bps) * 64 + lane;
      task_load<K, M>(g, sb, cb, xb, &ob);
    }
    task_store<K, M>(g, sa, ca, oa, xa);
    if (t1 >= tasks) break;
    const uint32_t t2 = t1 + nw;
    if (t2 < tasks) {
      sa = t2 / bps;
      ca = (t2 - sa * bps) * 64 + lane;
      task_load<K, M>(g, sa, ca, xa, &oa);
    }
    task_store<K, M>(g, sb, cb, ob, xb);
    t = t2;
  }
}

// G: 1 KiB tasks over PAIRS of stripes -- lane l owns column c of stripe 2p and
// the same column of stripe 2p+1 (32 B per lane, as a bitsliced encode needs,
// without C's 2 KiB-wide rows: the encode matrix is the same for every stripe).
template <int K, int M>
__global__ __launch_bounds__(256) void pG(Geo g) {
  const uint32_t lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
  const uint32_t nw = gridDim.x * 4, bps = (g.cols + 63) / 64, pairs = (g.N + 1) / 2, tasks = pairs * bps;
  for (uint32_t t = wave; t < tasks; t += nw) {
    const uint32_t sp = t / bps, b = t - sp * bps, col = b * 64 + lane;
    const uint32_t sa = 2 * sp, sb = 2 * sp + 1 < g.N ? 2 * sp + 1 : 2 * sp;
    u32x4 xa[K], xb[K];
    uint32_t oa, ob;
    task_load<K, M>(g, sa, col, xa, &oa);
    task_load<K, M>(g, sb, col, xb, &ob);
    task_store<K, M>(g, sa, col, oa, xa);
    task_store<K, M>(g, sb, col, ob, xb);
  }
}

template <int K, int M>
__global__ __launch_bounds__(256) void pE(Geo g) {
  const uint32_t lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
  const uint32_t nw = gridDim.x * 4, bps = (g.cols + 63) / 64;
  for (uint32_t s = wave; s < g.N; s += nw) {
    for (uint32_t b = 0; b < bps; ++b) {
      const uint32_t col = b * 64 + lane;
      u32x4 x[K];
      uint32_t off;
      task_load<K, M>(g, s, col, x, &off);
      task_store<K, M>(g, s, col, off, x);
    }
  }
}

// R: per-stripe reconstruct read pattern, compute-free: K reads per task of which
// the first NP come from the parity region (slots 0..NP-1) and the rest from data
// slots NP..K-1 (as a stripe missing NP data shards reads NP parity survivors), and
// E writes out of place (out + i*E*P + r*P).  NP = 0 is the all-data read mix.
template <int K, int NP, int E>
__global__ __launch_bounds__(256) void pR(Geo g, uint8_t* out) {
  const uint32_t lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
  const uint32_t nw = gridDim.x * 4, bps = (g.cols + 63) / 64, tasks = g.N * bps;
  for (uint32_t t = wave; t < tasks; t += nw) {
    const uint32_t s = t / bps, b = t - s * bps, col = b * 64 + lane;
    const uint32_t off = (col < g.cols ? col : g.cols - 1) * 16;
    const uint8_t* db = uni(g.d + (uint64_t)s * K * g.P);
    const uint8_t* pb = uni(g.p + (uint64_t)s * 4 * g.P);
    u32x4 x[K];
#pragma unroll
    for (int c = 0; c < K; ++c)
      x[c] = c < NP ? ld(pb + (uint64_t)c * g.P + off) : ld(db + (uint64_t)c * g.P + off);
    uint8_t* ob = out + (uint64_t)s * 4 * g.P;
#pragma unroll
    for (int r = 0; r < E; ++r) {
      u32x4 y = x[r];
#pragma unroll
      for (int c = 0; c < K; ++c) y ^= x[c] * (r + 1);
      st_drop(ob + (uint64_t)r * g.P, off, col < g.full, y);
    }
  }
}

struct RRun {
  const void* fn;
  Geo g;
  uint8_t* out;
  uint32_t grid;
};
static void launch_rrun(void* a) {
  RRun* r = static_cast<RRun*>(a);
  void* args[] = {&r->g, &r->out};
  CHECK(hipLaunchKernel(r->fn, dim3(r->grid), dim3(256), args, 0, nullptr));
}

static float time_it(void (*launch)(void*), void* arg, int iters);

// Input fill: constant 0x01 bytes (the round-1/2 default) or, with "rand" as the
// second argument, splitmix64 pseudo-random bytes -- DVFS and the DRAM bus both
// see the data, so ceilings are quoted on random data too.
static bool g_random = false;
static bool g_real_tables = false;
static bool g_line_stores = false;  // mode 'w': stores cover whole 128-B lines (pad written)  // compute_geometry: real GF product tables (third arg "real")
__global__ void fill_rand(uint64_t* p, uint64_t n8, uint64_t seed) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n8; i += (uint64_t)gridDim.x * 256) {
    uint64_t z = (i + seed) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    p[i] = z ^ (z >> 31);
  }
}
static void fill(void* p, size_t bytes) {
  if (!g_random) {
    CHECK(hipMemset(p, 1, bytes));
    return;
  }
  hipLaunchKernelGGL(fill_rand, dim3(4096), dim3(256), 0, nullptr, static_cast<uint64_t*>(p), bytes / 8,
                     reinterpret_cast<uint64_t>(p));
  CHECK(hipDeviceSynchronize());
}

static void read_mix(int cus, uint32_t S, uint32_t N) {
  const uint32_t P = (S + 255) / 256 * 256;
  uint8_t *d, *p, *o;
  CHECK(hipMalloc(&d, (size_t)N * 10 * P));
  CHECK(hipMalloc(&p, (size_t)N * 4 * P));
  CHECK(hipMalloc(&o, (size_t)N * 4 * P));
  fill(d, (size_t)N * 10 * P);
  fill(p, (size_t)N * 4 * P);
  Geo g{d, p, N, S, P, (S + 15) / 16, S / 16, S / 16};
  struct V { const char* name; const void* fn; int e; } vs[] = {
      {"10 data, 1 out", (const void*)&pR<10, 0, 1>, 1}, {"9 data + 1 parity, 1 out", (const void*)&pR<10, 1, 1>, 1},
      {"10 data, 2 out", (const void*)&pR<10, 0, 2>, 2}, {"8 data + 2 parity, 2 out", (const void*)&pR<10, 2, 2>, 2}};
  for (auto& v : vs)
    for (int bpc : {2, 6}) {
      RRun r{v.fn, g, o, (uint32_t)(cus * bpc)};
      const float ms = time_it(launch_rrun, &r, 10);
      const double alg = (double)N * S * (10 + v.e);
      std::printf("RS(10+4) S=%u read mix %-26s bpc=%d  %7.1f GB/s  (%.1f%% of 8 TB/s)\n", S, v.name, bpc,
                  alg / ms / 1e6, alg / ms / 1e6 / 80.0);
    }
  CHECK(hipFree(d));
  CHECK(hipFree(p));
  CHECK(hipFree(o));
}


// F: one workgroup per stripe at a time: the stripe's K data shards (one contiguous
// K*P-byte region in the split layout) stream into LDS with LDS-DMA (1 KiB per
// wave-instruction, in address order), then the waves compute column blocks from
// LDS and write the M parity rows (contiguous M*P bytes).  Occupancy: LDS-bound.
template <int K, int M>
__global__ __launch_bounds__(256) void pF(Geo g) {
  extern __shared__ __attribute__((aligned(16))) uint8_t stage[];
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint32_t chunks = (uint32_t)(((uint64_t)K * g.P) / 1024);  // P multiple of 256: K*P multiple of 1024 for K%4==2..
  const uint32_t bps = (g.cols + 63) / 64;
  for (uint32_t s = blockIdx.x; s < g.N; s += gridDim.x) {
    const uint8_t* src = g.d + (uint64_t)s * K * g.P;
    for (uint32_t j = w; j < chunks; j += 4) {
      __builtin_amdgcn_global_load_lds(src + (uint64_t)j * 1024 + lane * 16,
                                       (__attribute__((address_space(3))) void*)(stage + j * 1024), 16, 0, 0);
    }
    __builtin_amdgcn_s_waitcnt(0x3F70);  // vmcnt(0)
    __syncthreads();
    uint8_t* ob = g.p + (uint64_t)s * M * g.P;
    for (uint32_t b = w; b < bps; b += 4) {
      const uint32_t col = b * 64 + lane;
      const uint32_t off = (col < g.cols ? col : g.cols - 1) * 16;
      u32x4 x[K];
#pragma unroll
      for (int c = 0; c < K; ++c) x[c] = *reinterpret_cast<const u32x4*>(stage + (uint64_t)c * g.P + off);
#pragma unroll
      for (int r = 0; r < M; ++r) {
        u32x4 y = x[r];
#pragma unroll
        for (int c = 0; c < K; ++c) y ^= x[c] * (r + 1);
        st_drop(ob + (uint64_t)r * g.P, off, col < g.full, y);
      }
    }
    __syncthreads();
  }
}

struct FRun {
  const void* fn;
  Geo g[2];
  uint32_t grid, lds;
  int i;
};
static void launch_frun(void* a) {
  FRun* r = static_cast<FRun*>(a);
  Geo g = r->g[r->i++ & 1];
  void* args[] = {&g};
  CHECK(hipLaunchKernel(r->fn, dim3(r->grid), dim3(256), args, r->lds, nullptr));
}

template <int K, int M>
static void lds_geometry(int cus, uint32_t S, uint32_t N) {
  const uint32_t P = (S + 255) / 256 * 256;
  Geo g[2];
  for (auto& x : g) {
    uint8_t *d, *p;
    CHECK(hipMalloc(&d, (size_t)N * K * P));
    CHECK(hipMalloc(&p, (size_t)N * M * P));
    fill(d, (size_t)N * K * P);
    x = Geo{d, p, N, S, P, (S + 15) / 16, S / 16, g_line_stores ? (S + 127) / 128 * 8 : S / 16};
  }
  const uint32_t lds = K * P;
  CHECK(hipFuncSetAttribute((const void*)&pF<K, M>, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  const double alg = (double)N * S * (K + M);
  for (int bpc : {1, 2}) {
    if (bpc * lds > 160 * 1024) continue;
    FRun r{(const void*)&pF<K, M>, {g[0], g[1]}, (uint32_t)(cus * bpc), lds, 0};
    const float ms = time_it(launch_frun, &r, 10);
    std::printf("RS(%d+%d) S=%u P=%u  F lds-stripe      bpc=%d  %7.1f GB/s  (%.1f%% of 8 TB/s)\n", K, M, S, P, bpc,
                alg / ms / 1e6, alg / ms / 1e6 / 80.0);
  }
  for (auto& x : g) {
    CHECK(hipFree(const_cast<uint8_t*>(x.d)));
    CHECK(hipFree(x.p));
  }
}

// ---- the same patterns with the engine's GF(2^8) lookup arithmetic ----------------
// E outputs x K inputs, 3 v_perm + 1.5 v_bitop3 per product (rs_kernels.hip), the
// coefficient tables wave-uniform (kernel argument -> SGPRs).
struct Tabs {
  const uint32_t* t;  // device array of 4*10*5 table dwords
};

static float time_it(void (*launch)(void*), void* arg, int iters);

__device__ __forceinline__ uint32_t x3(uint32_t a, uint32_t b, uint32_t c) { return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96); }

template <int K, int E>
__device__ __forceinline__ void gf_compute(const Tabs& tb0, const u32x4 (&x)[K], u32x4 (&y)[E]) {
  u32x4 pend[E];
#pragma unroll
  for (int r = 0; r < E; ++r) y[r] = u32x4{0, 0, 0, 0};
#pragma unroll
  for (int c = 0; c < K; ++c) {
    uint32_t ia[4], ib[4], ic[4];
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      ia[d] = x[c][d] & 0x07070707u;
      ib[d] = (x[c][d] >> 3) & 0x07070707u;
      ic[d] = (x[c][d] >> 6) & 0x03030303u;
    }
    // tables re-read (scalar cache) per input, as rs_kernels.hip does: an opaque
    // pointer per input keeps the compiler from hoisting 200 dwords into SGPRs
    const uint32_t* tp = tb0.t;
    asm volatile("" : "+s"(tp));
#pragma unroll
    for (int r = 0; r < E; ++r) {
      const __attribute__((address_space(4))) uint32_t* q =
          (const __attribute__((address_space(4))) uint32_t*)(tp) + (r * K + c) * 5;
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        const uint32_t prod = x3(__builtin_amdgcn_perm(q[1], q[0], ia[d]), __builtin_amdgcn_perm(q[3], q[2], ib[d]),
                                 __builtin_amdgcn_perm(0u, q[4], ic[d]));
        if (c & 1)
          y[r][d] = x3(y[r][d], pend[r][d], prod);
        else if (c == K - 1)
          y[r][d] ^= prod;
        else
          pend[r][d] = prod;
      }
    }
  }
}

template <int K, int M, int E>
__device__ __forceinline__ void gf_store(const Geo& g, const Tabs& tb, uint32_t s, uint32_t col, uint32_t off,
                                         const u32x4 (&x)[K]) {
  u32x4 y[E];
  gf_compute<K, E>(tb, x, y);
  uint8_t* ob = g.p + (uint64_t)s * M * g.P;
#pragma unroll
  for (int r = 0; r < E; ++r) st_drop(ob + (uint64_t)r * g.P, col * 16, col < g.sfull, y[r]);
}

template <int K, int M, int E>
__global__ __launch_bounds__(256) void cB(Geo g, Tabs tb) {
  const uint32_t lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
  const uint32_t nw = gridDim.x * 4, bps = (g.cols + 63) / 64, tasks = g.N * bps;
  for (uint32_t t = wave; t < tasks; t += nw) {
    const uint32_t s = t / bps, b = t - s * bps, col = b * 64 + lane;
    u32x4 x[K];
    uint32_t off;
    task_load<K, M>(g, s, col, x, &off);
    gf_store<K, M, E>(g, tb, s, col, off, x);
  }
}

template <int K, int M, int E>
__global__ __launch_bounds__(256) void cD(Geo g, Tabs tb) {
  const uint32_t lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
  const uint32_t nw = gridDim.x * 4, bps = (g.cols + 63) / 64, tasks = g.N * bps;
  u32x4 xa[K], xb[K];
  uint32_t oa = 0, ob = 0, sa = 0, sb = 0, ca = 0, cb = 0;
  uint32_t t = wave;
  if (t < tasks) {
    sa = t / bps;
    ca = (t - sa * bps) * 64 + lane;
    task_load<K, M>(g, sa, ca, xa, &oa);
  }
  while (t < tasks) {
    const uint32_t t1 = t + nw;
    if (t1 < tasks) {
      sb = t1 / bps;
      cb = (t1 - sb * bps) * 64 + lane;
      task_load<K, M>(g, sb, cb, xb, &ob);
    }
    gf_store<K, M, E>(g, tb, sa, ca, oa, xa);
    if (t1 >= tasks) break;
    const uint32_t t2 = t1 + nw;
    if (t2 < tasks) {
      sa = t2 / bps;
      ca = (t2 - sa * bps) * 64 + lane;
      task_load<K, M>(g, sa, ca, xa, &oa);
    }
    gf_store<K, M, E>(g, tb, sb, cb, ob, xb);
    t = t2;
  }
}

struct CRun {
  const void* fn;
  Geo g[2];
  Tabs tb;
  uint32_t grid;
  int i;
};

static void launch_crun(void* a) {
  CRun* r = static_cast<CRun*>(a);
  Geo g = r->g[r->i++ & 1];
  void* args[] = {&g, &r->tb};
  CHECK(hipLaunchKernel(r->fn, dim3(r->grid), dim3(256), args, 0, nullptr));
}

template <int K, int M, int E>
static void compute_geometry(int cus, uint32_t S, uint32_t N) {
  const uint32_t P = (S + 255) / 256 * 256;
  Geo g[2];
  for (auto& x : g) {
    uint8_t *d, *p;
    CHECK(hipMalloc(&d, (size_t)N * K * P));
    CHECK(hipMalloc(&p, (size_t)N * M * P));
    fill(d, (size_t)N * K * P);
    x = Geo{d, p, N, S, P, (S + 15) / 16, S / 16, g_line_stores ? (S + 127) / 128 * 8 : S / 16};
  }
  std::vector<uint32_t> ht(200);
  for (int i = 0; i < 200; ++i) ht[i] = 0x01020304u * (i + 1);
  if (g_real_tables) {  // real 3-chunk product tables of pseudo-random nonzero coefficients
    auto mul = [](uint32_t a, uint32_t b) {
      uint32_t r = 0;
      for (; b; b >>= 1, a = (a << 1) ^ ((a & 0x80) ? 0x11d : 0))
        if (b & 1) r ^= a;
      return r & 0xFF;
    };
    uint32_t x = 12345;
    for (int q = 0; q < 40; ++q) {
      x = x * 1103515245u + 12345u;
      const uint32_t f = 1 + (x >> 16) % 255;
      auto pack4 = [&](int base, int shift) {
        uint32_t w = 0;
        for (int j = 0; j < 4; ++j) w |= mul(f, ((base + j) << shift) & 0xFF) << (8 * j);
        return w;
      };
      ht[q * 5 + 0] = pack4(0, 0);
      ht[q * 5 + 1] = pack4(4, 0);
      ht[q * 5 + 2] = pack4(0, 3);
      ht[q * 5 + 3] = pack4(4, 3);
      ht[q * 5 + 4] = pack4(0, 6);
    }
  }
  uint32_t* dt;
  CHECK(hipMalloc(&dt, 800));
  CHECK(hipMemcpy(dt, ht.data(), 800, hipMemcpyHostToDevice));
  Tabs tb{dt};
  const double alg = (double)N * S * (K + E);
  struct V {
    const char* name;
    const void* fn;
  } vs[] = {{"B+gf  1KiB", (const void*)&cB<K, M, E>}, {"D+gf pipelined", (const void*)&cD<K, M, E>}};
  for (auto& v : vs) {
    for (int bpc : {1, 2, 3, 4, 6}) {
      CRun r{v.fn, {g[0], g[1]}, tb, (uint32_t)(cus * bpc), 0};
      const float ms = time_it(launch_crun, &r, 10);
      std::printf("RS(%d+%d) E=%d S=%u  %-16s bpc=%d  %7.1f GB/s  (%.1f%% of 8 TB/s)\n", K, M, E, S, v.name, bpc,
                  alg / ms / 1e6, alg / ms / 1e6 / 80.0);
    }
  }
  for (auto& x : g) {
    CHECK(hipFree(const_cast<uint8_t*>(x.d)));
    CHECK(hipFree(x.p));
  }
}

// default cache policy (plain loads / stores) for comparison with the nt copy
template <int U>
__global__ __launch_bounds__(256) void copyd(const u32x4* __restrict__ src, u32x4* __restrict__ dst, uint64_t n16) {
  const uint64_t stride = (uint64_t)gridDim.x * 256 * U;
  for (uint64_t base = (uint64_t)blockIdx.x * 256 * U + threadIdx.x; base < n16; base += stride) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (base + u * 256 < n16) v[u] = src[base + u * 256];
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (base + u * 256 < n16) dst[base + u * 256] = v[u];
  }
}

template <int U>
__global__ __launch_bounds__(256) void copyk(const u32x4* __restrict__ src, u32x4* __restrict__ dst, uint64_t n16) {
  const uint64_t stride = (uint64_t)gridDim.x * 256 * U;
  for (uint64_t base = (uint64_t)blockIdx.x * 256 * U + threadIdx.x; base < n16; base += stride) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (base + u * 256 < n16) v[u] = __builtin_nontemporal_load(src + base + u * 256);
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (base + u * 256 < n16) __builtin_nontemporal_store(v[u], dst + base + u * 256);
  }
}

static float time_it(void (*launch)(void*), void* arg, int iters) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int i = 0; i < 2; ++i) launch(arg);
  CHECK(hipEventRecord(e0));
  for (int i = 0; i < iters; ++i) launch(arg);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  CHECK(hipEventDestroy(e0));
  CHECK(hipEventDestroy(e1));
  return ms / iters;
}

struct Run {
  const void* fn;
  Geo g[2];
  uint32_t grid;
  int i;
};

static void launch_run(void* a) {
  Run* r = static_cast<Run*>(a);
  Geo g = r->g[r->i++ & 1];
  void* args[] = {&g};
  CHECK(hipLaunchKernel(r->fn, dim3(r->grid), dim3(256), args, 0, nullptr));
}

// B (1 KiB tasks), C (2 KiB-wide tasks) and G (1 KiB tasks over stripe pairs), two
// passes in alternating order.
template <int K, int M>
static void geometry_pairs(int cus, uint32_t S, uint32_t N) {
  const uint32_t P = (S + 255) / 256 * 256;
  Geo g[2];
  for (auto& x : g) {
    uint8_t *d, *p;
    CHECK(hipMalloc(&d, (size_t)N * K * P));
    CHECK(hipMalloc(&p, (size_t)N * M * P));
    fill(d, (size_t)N * K * P);
    x = Geo{d, p, N, S, P, (S + 15) / 16, S / 16, S / 16};
  }
  const double alg = (double)N * S * (K + M);
  struct V {
    const char* name;
    const void* fn;
  } vs[] = {{"B bufdrop 1KiB", (const void*)&pB<K, M>},
            {"C bufdrop 2KiB", (const void*)&pC<K, M>},
            {"G stripe-pair 1KiB", (const void*)&pG<K, M>}};
  for (int pass = 0; pass < 2; ++pass)
    for (int i = 0; i < 3; ++i) {
      const V& v = vs[pass ? 2 - i : i];
      for (int bpc : {2, 4}) {
        Run r{v.fn, {g[0], g[1]}, (uint32_t)(cus * bpc), 0};
        const float ms = time_it(launch_run, &r, 20);
        std::printf("RS(%d+%d) S=%u P=%u  %-18s bpc=%d  %7.1f GB/s  (%.1f%% of 8 TB/s)\n", K, M, S, P, v.name, bpc,
                    alg / ms / 1e6, alg / ms / 1e6 / 80.0);
      }
    }
  for (auto& x : g) {
    CHECK(hipFree(const_cast<uint8_t*>(x.d)));
    CHECK(hipFree(x.p));
  }
}

template <int K, int M>
static void geometry(int cus, uint32_t S, uint32_t N, uint32_t pitch = 0, bool only_b = false) {
  const uint32_t P = pitch ? pitch : (S + 255) / 256 * 256;
  Geo g[2];
  for (auto& x : g) {
    uint8_t *d, *p;
    CHECK(hipMalloc(&d, (size_t)N * K * P));
    CHECK(hipMalloc(&p, (size_t)N * M * P));
    fill(d, (size_t)N * K * P);
    x = Geo{d, p, N, S, P, (S + 15) / 16, S / 16, g_line_stores ? (S + 127) / 128 * 8 : S / 16};
  }
  const double alg = (double)N * S * (K + M);
  struct V {
    const char* name;
    const void* fn;
  } vs[] = {{"A plain-if 1KiB", (const void*)&pA<K, M>},
            {"B bufdrop 1KiB", (const void*)&pB<K, M>},
            {"C bufdrop 2KiB", (const void*)&pC<K, M>},
            {"D pipelined 1KiB", (const void*)&pD<K, M>},
            {"E stripe-per-wave", (const void*)&pE<K, M>}};
  for (auto& v : vs) {
    if (only_b && v.fn != (const void*)&pB<K, M>) continue;
    for (int bpc : {2, 4, 8}) {
      Run r{v.fn, {g[0], g[1]}, (uint32_t)(cus * bpc), 0};
      const float ms = time_it(launch_run, &r, 10);
      std::printf("RS(%d+%d) S=%u P=%u  %-18s bpc=%d  %7.1f GB/s  (%.1f%% of 8 TB/s)\n", K, M, S, P, v.name, bpc,
                  alg / ms / 1e6, alg / ms / 1e6 / 80.0);
    }
  }
  for (auto& x : g) {
    CHECK(hipFree(const_cast<uint8_t*>(x.d)));
    CHECK(hipFree(x.p));
  }
}

struct CopyRun {
  const void* fn;
  const u32x4* s;
  u32x4* d;
  uint64_t n16;
  uint32_t grid;
};
static void launch_copy(void* a) {
  CopyRun* r = static_cast<CopyRun*>(a);
  void* args[] = {&r->s, &r->d, &r->n16};
  CHECK(hipLaunchKernel(r->fn, dim3(r->grid), dim3(256), args, 0, nullptr));
}

int main(int argc, char** argv) {
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  const bool only_copy = argc > 1 && (argv[1][0] == 'c' || argv[1][0] == 'C');
  g_random = argc > 2 && argv[2][0] == 'r';
  g_real_tables = argc > 3 && argv[3][0] == 'r';
  std::printf("input data: %s\n", g_random ? "random (splitmix64)" : "constant 0x01");
  if (argc > 1 && argv[1][0] == 'f') {  // LDS-staged whole-stripe streaming
    lds_geometry<10, 4>(cus, 6554, 16384);
    lds_geometry<8, 4>(cus, 8192, 16384);
    lds_geometry<4, 2>(cus, 16384, 16384);
    lds_geometry<6, 3>(cus, 10923, 16384);
    return 0;
  }
  if (argc > 1 && argv[1][0] == 'p') {  // shard pitch sweep, pattern B
    for (uint32_t P : {6656u, 6912u, 7168u, 7680u, 8192u, 10240u}) geometry<10, 4>(cus, 6554, 16384, P, true);
    for (uint32_t P : {8192u, 8448u, 9216u, 10240u}) geometry<8, 4>(cus, 8192, 16384, P, true);
    for (uint32_t P : {1024u, 1280u, 1536u, 2048u}) geometry<4, 2>(cus, 1024, 65536, P, true);
    for (uint32_t P : {16384u, 16640u, 17408u}) geometry<4, 2>(cus, 16384, 16384, P, true);
    return 0;
  }
  if (argc > 1 && argv[1][0] == 'R') {  // per-stripe reconstruct read mixes
    read_mix(cus, 6554, 16384);
    return 0;
  }
  if (argc > 1 && argv[1][0] == 'w') {  // partial-line stores vs whole-line stores
    for (int ls = 0; ls < 2; ++ls) {
      g_line_stores = ls;
      std::printf("--- stores: %s\n", ls ? "whole 128-B lines (pitch padding written)" : "exact S/16 columns");
      geometry<10, 4>(cus, 6554, 16384, 0, true);
      geometry<6, 3>(cus, 10923, 16384, 0, true);
      compute_geometry<10, 4, 2>(cus, 6554, 16384);
      compute_geometry<10, 4, 4>(cus, 6554, 16384);
    }
    geometry<10, 4>(cus, 6656, 16384, 0, true);
    return 0;
  }
  if (argc > 1 && argv[1][0] == 'P') {  // stripe-pair tasks vs 1 KiB and 2 KiB tasks
    geometry_pairs<8, 4>(cus, 8192, 16384);
    geometry_pairs<10, 4>(cus, 6656, 16384);
    geometry_pairs<10, 4>(cus, 6554, 16384);
    geometry_pairs<4, 2>(cus, 16384, 16384);
    return 0;
  }
  if (argc > 1 && argv[1][0] == 'g') {
    compute_geometry<10, 4, 2>(cus, 6554, 16384);
    compute_geometry<10, 4, 4>(cus, 6554, 16384);
    compute_geometry<8, 4, 4>(cus, 8192, 16384);
    compute_geometry<4, 2, 2>(cus, 1024, 65536);
    return 0;
  }
  if (!only_copy) {
    geometry<10, 4>(cus, 6554, 16384);
    geometry<10, 4>(cus, 6656, 16384);
    geometry<8, 4>(cus, 8192, 16384);
    geometry<4, 2>(cus, 1024, 65536);
  }
  const uint64_t bytes = (argc > 1 && argv[1][0] == 'C') ? (4ull << 30) : (1ull << 30);
  u32x4 *a, *b;
  CHECK(hipMalloc(&a, bytes));
  CHECK(hipMalloc(&b, bytes));
  fill(a, bytes);
  struct C {
    const char* name;
    const void* fn;
  } cs[] = {{"U=2", (const void*)&copyk<2>}, {"U=4", (const void*)&copyk<4>}, {"U=8", (const void*)&copyk<8>},
            {"U=16", (const void*)&copyk<16>}, {"dflt U=4", (const void*)&copyd<4>},
            {"dflt U=8", (const void*)&copyd<8>}};
  std::printf("copy buffer: %llu MiB each way\n", (unsigned long long)(bytes >> 20));
  for (auto& c : cs)
    for (int g : {1, 2, 4, 8, 16, 32}) {
      CopyRun r{c.fn, a, b, bytes / 16, (uint32_t)(cus * g)};
      const float ms = time_it(launch_copy, &r, 10);
      std::printf("copy %-5s blocks/CU=%-2d %7.1f GB/s (read+write)\n", c.name, g, 2.0 * bytes / ms / 1e6);
    }
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  CHECK(hipMemcpy(b, a, bytes, hipMemcpyDeviceToDevice));
  CHECK(hipEventRecord(e0));
  for (int i = 0; i < 10; ++i) CHECK(hipMemcpyAsync(b, a, bytes, hipMemcpyDeviceToDevice, nullptr));
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  std::printf("hipMemcpyAsync D2D          %7.1f GB/s (read+write)\n", 2.0 * bytes / (ms / 10) / 1e6);
  return 0;
}
