// hbm_probe3.hip -- why does the uniform erasure pattern {0,1} (read data slots 2,3
// + parity 0,1, write data slots 0,1) stream slower than encode (read data 0..3,
// write parity 0,1)?  Compute-free (XOR only), split layout, RS(4+2), 4 KiB stripes.
// Variants: store policy (nt / plain / sc1-ish via __hip_atomic_store is not 16 B, so
// nt vs plain only), output placement (in place vs a separate region), stripe
// ordering of the writes (same task vs a lagged task), workgroups per CU.
// Build: hipcc --offload-arch=gfx950 -O3 -o hbm_probe3 hbm_probe3.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ void st(u32x4* p, u32x4 v) {
  if constexpr (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}
__device__ __forceinline__ u32x4 ld(const u32x4* p) { return __builtin_nontemporal_load(p); }

struct G {
  u32x4* data;    // N x 4 x cols
  u32x4* parity;  // N x 2 x cols
  u32x4* out;     // N x 2 x cols (separate region variant)
  uint32_t N, cols;
};

// MODE 0: encode-like   read d0..d3, write p0,p1
// MODE 1: {0,1} in place read d2,d3,p0,p1, write d0,d1
// MODE 2: {0,1} to a separate output region
// MODE 3: {0,1} in place, but each wave writes the outputs of the task it processed
//         LAG trips earlier (stores trail reads by LAG tasks of this wave)
template <int MODE, bool NT>
__global__ __launch_bounds__(256) void k(G g) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
  const uint32_t nw = gridDim.x * 4;
  const uint32_t bps = g.cols / 64;
  const uint32_t tasks = g.N * bps;
  u32x4 y0 = {0, 0, 0, 0}, y1 = {0, 0, 0, 0};
  u32x4* po = nullptr;
  bool have = false;
  for (uint32_t t = wave; t < tasks; t += nw) {
    const uint32_t s = t / bps, b = t % bps;
    u32x4* d = g.data + (uint64_t)s * 4 * g.cols + b * 64 + lane;
    u32x4* p = g.parity + (uint64_t)s * 2 * g.cols + b * 64 + lane;
    if (MODE == 0) {
      u32x4 a = ld(d), bb = ld(d + g.cols), c = ld(d + 2 * g.cols), e = ld(d + 3 * g.cols);
      st<NT>(p, a ^ bb);
      st<NT>(p + g.cols, c ^ e);
    } else if (MODE == 3) {
      // stores of the previous task, issued after this task's loads
      u32x4 a = ld(d + 2 * g.cols), bb = ld(d + 3 * g.cols), c = ld(p), e = ld(p + g.cols);
      if (have) {
        st<NT>(po, y0);
        st<NT>(po + g.cols, y1);
      }
      y0 = a ^ c;
      y1 = bb ^ e;
      po = d;
      have = true;
    } else {
      u32x4 a = ld(d + 2 * g.cols), bb = ld(d + 3 * g.cols), c = ld(p), e = ld(p + g.cols);
      u32x4* o = MODE == 2 ? g.out + (uint64_t)s * 2 * g.cols + b * 64 + lane : d;
      if (MODE == 4) {
        st<NT>(o + g.cols, bb ^ e);
        st<NT>(o, a ^ c);
      } else {
        st<NT>(o, a ^ c);
        st<NT>(o + g.cols, bb ^ e);
      }
    }
  }
  if (MODE == 3 && have) {
    st<NT>(po, y0);
    st<NT>(po + g.cols, y1);
  }
}

int main() {
  hipDeviceProp_t prop;
  (void)hipGetDeviceProperties(&prop, 0);
  const int cus = prop.multiProcessorCount;
  const uint32_t N = 65536, cols = 64;
  const size_t dbytes = (size_t)N * 4 * cols * 16, pbytes = (size_t)N * 2 * cols * 16;
  const int nb = 5;
  std::vector<G> gs(nb);
  for (auto& g : gs) {
    if (hipMalloc(&g.data, dbytes) || hipMalloc(&g.parity, pbytes) || hipMalloc(&g.out, pbytes)) return 1;
    (void)hipMemset(g.data, 1, dbytes);
    (void)hipMemset(g.parity, 2, pbytes);
    (void)hipMemset(g.out, 3, pbytes);
    g.N = N;
    g.cols = cols;
  }
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  auto run = [&](const char* name, auto kern, int bpc) {
    const unsigned grid = cus * bpc;
    for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, gs[i % nb]);
    (void)hipEventRecord(e0);
    const int it = 30;
    for (int i = 0; i < it; ++i) hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, gs[i % nb]);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    ms /= it;
    printf("%-34s bpc=%d : %7.1f GB/s  (%.1f us)\n", name, bpc, (dbytes + pbytes) / ms / 1e6, ms * 1e3);
  };
  for (int bpc : {1, 2, 4}) {
    run("encode-like  nt", k<0, true>, bpc);
    run("encode-like  plain", k<0, false>, bpc);
    run("{0,1} in place  nt", k<1, true>, bpc);
    run("{0,1} in place  plain", k<1, false>, bpc);
    run("{0,1} separate region  nt", k<2, true>, bpc);
    run("{0,1} separate region  plain", k<2, false>, bpc);
    run("{0,1} in place lag-1  nt", k<3, true>, bpc);
    run("{0,1} in place reversed  nt", k<4, true>, bpc);
  }
  return 0;
}
