// rs_kernels.hip -- CDNA4 (gfx950) kernels for Reed-Solomon encode/reconstruct.
//
// One kernel family computes  Y[e x S] = C[e x K] (x) X[K x S]  over GF(2^8) for
// a batch of independent stripes.  Encode (C = parity rows of the encode matrix,
// [upstream klauspost reedsolomon.go Encode -> codeSomeShards], called from
// internal/ec/ec.go:54-56) and reconstruct (C = composed decode rows over the
// first K present shards, [upstream reconstruct], internal/ec/ec.go:59-61) are
// the same kernel with different coefficient plans.
//
// GF(2^8) multiply by a wave-uniform coefficient f, 4 bytes per VALU op:
//   x = x[2:0] | x[5:3]<<3 | x[7:6]<<6, and multiplication is GF(2)-linear, so
//   f*x = A[x[2:0]] ^ B[x[5:3]] ^ C[x[7:6]]  with 8-, 8- and 4-entry product
//   tables.  An 8-entry byte table is exactly one v_perm_b32 byte pool (two
//   dwords), so each table lookup is ONE v_perm_b32 on 4 packed bytes, with no
//   LDS traffic and no data-dependent bank conflicts.  Per (coefficient, data
//   dword): 3 v_perm_b32 + ~1.5 v_xor3_b32; per data dword 5 ops of index prep
//   shared by all M outputs.  The tables (5 dwords per coefficient) are
//   wave-uniform and live in SGPRs.
//
// Memory: HBM-bound streaming.  Each wave owns one (stripe, 1 KiB column block)
// task: lane l reads 16 B at byte offset 16*(64*blk+l) of each of the K input
// shards (K coalesced 1 KiB wave loads), and writes 16 B of each output shard.
// Layout (device): shard s of stripe i at base + i*stripe_pitch + s*shard_pitch,
// shard_pitch and stripe_pitch multiples of 16, shard_pitch >= round_up(S, 16):
// reads of the tail column may touch the shard slot's padding; writes never do.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rs_plan.hpp"

namespace rs {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

struct Idx3 {
  uint32_t a, b, c;
};

__device__ __forceinline__ Idx3 split3(uint32_t x) {
  Idx3 r;
  r.a = x & 0x07070707u;
  r.b = (x >> 3) & 0x07070707u;
  r.c = (x >> 6) & 0x03030303u;
  return r;
}

__device__ __forceinline__ uint32_t lookup3(const Idx3& i, uint32_t t0, uint32_t t1, uint32_t t2,
                                            uint32_t t3, uint32_t t4) {
  return __builtin_amdgcn_perm(t1, t0, i.a) ^ __builtin_amdgcn_perm(t3, t2, i.b) ^
         __builtin_amdgcn_perm(0u, t4, i.c);
}

__device__ __forceinline__ u32x4 load16(const uint8_t* p) {
  return __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
}

__device__ __forceinline__ void store16(uint8_t* p, u32x4 v) {
  __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(p));
}

__device__ __forceinline__ void store_tail(uint8_t* p, u32x4 v, uint32_t nbytes) {
  // nbytes in [1, 15]: byte stores of the valid prefix of the last column.
  for (uint32_t q = 0; q < nbytes; ++q) p[q] = static_cast<uint8_t>(v[q >> 2] >> (8 * (q & 3)));
}

__device__ __forceinline__ uint32_t wave_uniform(uint32_t v) {
  return __builtin_amdgcn_readfirstlane(v);
}

// ---------------------------------------------------------------------------
// Specialised kernel: compile-time K and M (max outputs), fully unrolled.
// PER_STRIPE: plan chosen per stripe from present_masks via a missing-mask LUT.
template <int K, int M, bool PER_STRIPE>
__global__ __launch_bounds__(256) void apply_kernel(const KernelArgs a) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wave = wave_uniform(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6));
  const uint32_t nwaves = gridDim.x * (blockDim.x >> 6);
  const uint64_t ntasks = static_cast<uint64_t>(a.n_stripes) * a.blocks_per_stripe;
  const PlanView pv0(a.plans, K, M);

  for (uint64_t t = wave; t < ntasks; t += nwaves) {
    const uint32_t stripe = static_cast<uint32_t>(t / a.blocks_per_stripe);
    const uint32_t blk = static_cast<uint32_t>(t - static_cast<uint64_t>(stripe) * a.blocks_per_stripe);
    const uint8_t* plan = a.plans;
    if (PER_STRIPE) {
      const uint32_t present = as_const<uint32_t>(a.present_masks)[stripe];
      const uint32_t missing = (~present) & a.full_mask;
      const uint32_t pid = as_const<uint16_t>(a.lut)[missing];
      if (pid == kPlanInvalid) {
        if (lane == 0 && blk == 0) atomicOr(a.status, 1u);
        continue;
      }
      plan = a.plans + static_cast<uint64_t>(pid) * a.plan_bytes;
    }
    const PlanView pv(plan, K, M);
    const uint32_t n_out = pv.n_out();
    if (n_out == 0) continue;

    const uint32_t col = blk * 64u + lane;
    const uint32_t off = col * 16u;
    if (off >= a.shard_len) continue;

    const uint8_t* in_base = a.in + static_cast<uint64_t>(stripe) * a.in_stripe_pitch;
    uint8_t* out_base = a.out + static_cast<uint64_t>(stripe) * a.out_stripe_pitch;

    u32x4 x[K];
#pragma unroll
    for (int c = 0; c < K; ++c) x[c] = load16(in_base + static_cast<uint64_t>(pv.in_idx(c)) * a.shard_pitch + off);

    Idx3 ix[K][4];
#pragma unroll
    for (int c = 0; c < K; ++c)
#pragma unroll
      for (int d = 0; d < 4; ++d) ix[c][d] = split3(x[c][d]);

    const uint32_t tail = a.shard_len - off;  // >= 1
#pragma unroll
    for (int r = 0; r < M; ++r) {
      if (r >= static_cast<int>(n_out)) break;
      u32x4 y = {0u, 0u, 0u, 0u};
#pragma unroll
      for (int c = 0; c < K; ++c) {
        const RS_CONST uint32_t* tb = pv.tab(r, c);
        const uint32_t t0 = tb[0], t1 = tb[1], t2 = tb[2], t3 = tb[3], t4 = tb[4];
#pragma unroll
        for (int d = 0; d < 4; ++d) y[d] ^= lookup3(ix[c][d], t0, t1, t2, t3, t4);
      }
      uint8_t* dst = out_base + static_cast<uint64_t>(pv.out_idx(r)) * a.shard_pitch + off;
      if (tail >= 16u)
        store16(dst, y);
      else
        store_tail(dst, y, tail);
    }
  }
}

// ---------------------------------------------------------------------------
// Generic kernel: runtime K (<= kMaxK), outputs in groups of 4.
template <bool PER_STRIPE>
__global__ __launch_bounds__(256) void apply_kernel_generic(const KernelArgs a) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wave = wave_uniform(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6));
  const uint32_t nwaves = gridDim.x * (blockDim.x >> 6);
  const uint64_t ntasks = static_cast<uint64_t>(a.n_stripes) * a.blocks_per_stripe;
  const int K = a.k, M = a.m;

  for (uint64_t t = wave; t < ntasks; t += nwaves) {
    const uint32_t stripe = static_cast<uint32_t>(t / a.blocks_per_stripe);
    const uint32_t blk = static_cast<uint32_t>(t - static_cast<uint64_t>(stripe) * a.blocks_per_stripe);
    const uint8_t* plan = a.plans;
    if (PER_STRIPE) {
      const uint32_t present = as_const<uint32_t>(a.present_masks)[stripe];
      const uint32_t missing = (~present) & a.full_mask;
      const uint32_t pid = as_const<uint16_t>(a.lut)[missing];
      if (pid == kPlanInvalid) {
        if (lane == 0 && blk == 0) atomicOr(a.status, 1u);
        continue;
      }
      plan = a.plans + static_cast<uint64_t>(pid) * a.plan_bytes;
    }
    const PlanView pv(plan, K, M);
    const int n_out = static_cast<int>(pv.n_out());
    const uint32_t col = blk * 64u + lane;
    const uint32_t off = col * 16u;
    if (n_out == 0 || off >= a.shard_len) continue;
    const uint8_t* in_base = a.in + static_cast<uint64_t>(stripe) * a.in_stripe_pitch;
    uint8_t* out_base = a.out + static_cast<uint64_t>(stripe) * a.out_stripe_pitch;
    const uint32_t tail = a.shard_len - off;

    for (int r0 = 0; r0 < n_out; r0 += 4) {
      u32x4 y[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) y[q] = u32x4{0u, 0u, 0u, 0u};
      for (int c = 0; c < K; ++c) {
        const u32x4 x = load16(in_base + static_cast<uint64_t>(pv.in_idx(c)) * a.shard_pitch + off);
        Idx3 ix[4];
#pragma unroll
        for (int d = 0; d < 4; ++d) ix[d] = split3(x[d]);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          if (r0 + q >= n_out) break;
          const RS_CONST uint32_t* tb = pv.tab(r0 + q, c);
          const uint32_t t0 = tb[0], t1 = tb[1], t2 = tb[2], t3 = tb[3], t4 = tb[4];
#pragma unroll
          for (int d = 0; d < 4; ++d) y[q][d] ^= lookup3(ix[d], t0, t1, t2, t3, t4);
        }
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (r0 + q >= n_out) break;
        uint8_t* dst = out_base + static_cast<uint64_t>(pv.out_idx(r0 + q)) * a.shard_pitch + off;
        if (tail >= 16u)
          store16(dst, y[q]);
        else
          store_tail(dst, y[q], tail);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Streaming copy (bench only): the measured HBM ceiling next to the RS kernels.
__global__ __launch_bounds__(256) void copy_kernel(const u32x4* __restrict__ src, u32x4* __restrict__ dst,
                                                   uint64_t n16) {
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n16; i += stride)
    __builtin_nontemporal_store(__builtin_nontemporal_load(src + i), dst + i);
}

// ---------------------------------------------------------------------------
// Host-side launch dispatch.
template <int K, int M>
static bool try_launch(const KernelArgs& a, int k, int m, bool per_stripe, dim3 grid, hipStream_t s) {
  if (k != K || m != M) return false;
  if (per_stripe)
    hipLaunchKernelGGL((apply_kernel<K, M, true>), grid, dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL((apply_kernel<K, M, false>), grid, dim3(256), 0, s, a);
  return true;
}

const char* launch_apply(const KernelArgs& a, bool per_stripe, uint32_t grid_blocks, hipStream_t s,
                         bool force_generic) {
  const dim3 grid(grid_blocks);
  if (!force_generic) {
    if (try_launch<4, 2>(a, a.k, a.m, per_stripe, grid, s)) return "apply_kernel<4,2>";
    if (try_launch<8, 4>(a, a.k, a.m, per_stripe, grid, s)) return "apply_kernel<8,4>";
    if (try_launch<10, 4>(a, a.k, a.m, per_stripe, grid, s)) return "apply_kernel<10,4>";
    if (try_launch<6, 3>(a, a.k, a.m, per_stripe, grid, s)) return "apply_kernel<6,3>";
  }
  if (per_stripe)
    hipLaunchKernelGGL((apply_kernel_generic<true>), grid, dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL((apply_kernel_generic<false>), grid, dim3(256), 0, s, a);
  return "apply_kernel_generic";
}

void launch_copy(const void* src, void* dst, uint64_t bytes, uint32_t grid_blocks, hipStream_t s) {
  hipLaunchKernelGGL(copy_kernel, dim3(grid_blocks), dim3(256), 0, s, static_cast<const u32x4*>(src),
                     static_cast<u32x4*>(dst), bytes / 16);
}

int apply_kernel_max_blocks_per_cu(int k, int m, bool per_stripe) {
  int nb = 0;
  const void* fn = nullptr;
#define RS_PICK(KK, MM)                                                                          \
  if (k == KK && m == MM)                                                                        \
    fn = per_stripe ? reinterpret_cast<const void*>(&apply_kernel<KK, MM, true>)                 \
                    : reinterpret_cast<const void*>(&apply_kernel<KK, MM, false>);
  RS_PICK(4, 2) RS_PICK(8, 4) RS_PICK(10, 4) RS_PICK(6, 3)
#undef RS_PICK
  if (!fn)
    fn = per_stripe ? reinterpret_cast<const void*>(&apply_kernel_generic<true>)
                    : reinterpret_cast<const void*>(&apply_kernel_generic<false>);
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, fn, 256, 0) != hipSuccess || nb < 1) nb = 1;
  return nb;
}

}  // namespace rs
