// rs_plan.hpp -- device-visible coefficient plans and kernel arguments.
//
// A plan is one coefficient matrix C[e x K] in the form the kernels consume,
// plus the shard slots it reads and writes:
//   encode       : in = data shards 0..K-1, out = parity 0..M-1   (rows K..K+M-1 of
//                  the encode matrix, [upstream reedsolomon.go Encode])
//   reconstruct  : in = first K present shards in index order, out = every missing
//                  shard (data then parity, index order), C = composed decode rows
//                  ([upstream reedsolomon.go reconstruct] phases 1+2 folded).
// Byte layout (plan_bytes = plan_stride(K, M), 128-B aligned):
//   u32 n_out; u32 present; u32 out_mask; u32 reserved; u32 in_idx[K]; u32 out_idx[M];
//   pad to 16;   (present: the shards the plan reads from; out_mask: the shards it
//                 may fill -- all, or the data shards for ReconstructData)
//   u8 coef[M][plan_coef_row(K)] -- the coefficients C[r][c] themselves, rows padded to
//                        4 B; pad to 16 (RS(10+4): header + coef = the plan's first 128 B)
//   u32 tab[K][M][5]  -- per coefficient f = C[r][c]: the 3-chunk v_perm tables
//                        {A_lo, A_hi, B_lo, B_hi, C_lo} (see rs_kernels.hip), input-major
//                        so one input's E rows are one contiguous scalar load
// The kernels derive the input / output slots from the present mask itself (first
// K present in index order / every missing one), which is exactly how these plans
// are built; in_idx / out_idx are kept for the generic kernel and for checks.
#pragma once

#include <stdint.h>


namespace rs {

constexpr int kMaxK = 32;
constexpr int kMaxM = 16;
constexpr uint32_t kPlanInvalid = 0xFFFFu;
// Largest column range one launch covers: the kernels' dropped-store descriptors
// span 2 GiB from a shard base, so launch_apply runs longer shards as a sequence of
// 1 GiB column windows (the codec is column-wise).
constexpr uint32_t kColumnWindow = 1u << 30;

__host__ __device__ constexpr uint32_t plan_coef_row(int k) { return (static_cast<uint32_t>(k) + 3u) & ~3u; }
__host__ __device__ constexpr uint32_t plan_coef_offset(int k, int m) {
  return (16u + 4u * static_cast<uint32_t>(k) + 4u * static_cast<uint32_t>(m) + 15u) & ~15u;
}
__host__ __device__ constexpr uint32_t plan_tab_offset(int k, int m) {
  return (plan_coef_offset(k, m) + static_cast<uint32_t>(m) * plan_coef_row(k) + 15u) & ~15u;
}
__host__ __device__ constexpr uint32_t plan_stride(int k, int m) {
  return (plan_tab_offset(k, m) + 20u * static_cast<uint32_t>(k) * static_cast<uint32_t>(m) + 127u) & ~127u;
}

// Plans, masks and LUT are written by the host before a launch and never by a
// kernel, so device code reads them through the constant address space: uniform
// addresses then lower to scalar (s_load) reads into SGPRs.
#if defined(__HIP_DEVICE_COMPILE__)
#define RS_CONST __attribute__((address_space(4)))
#else
#define RS_CONST
#endif
template <typename T>
__host__ __device__ inline const RS_CONST T* as_const(const void* p) {
  return (const RS_CONST T*)(p);
}

struct PlanView {
  const uint8_t* p;
  int k, m;
  __host__ __device__ PlanView(const uint8_t* plan, int kk, int mm) : p(plan), k(kk), m(mm) {}
  __host__ __device__ uint32_t n_out() const { return *as_const<uint32_t>(p); }
  __host__ __device__ uint32_t present() const { return as_const<uint32_t>(p)[1]; }
  __host__ __device__ uint32_t out_mask() const { return as_const<uint32_t>(p)[2]; }
  __host__ __device__ uint32_t in_idx(int c) const { return as_const<uint32_t>(p + 16)[c]; }
  __host__ __device__ uint32_t out_idx(int r) const { return as_const<uint32_t>(p + 16 + 4 * k)[r]; }
  // the five table dwords of coefficient (r, c): quad(r, c)[0..3] and c4(r, c)
  __host__ __device__ const RS_CONST uint32_t* quad(int r, int c) const {
    return as_const<uint32_t>(p + plan_tab_offset(k, m)) + (c * m + r) * 5;
  }
  __host__ __device__ uint32_t c4(int r, int c) const { return quad(r, c)[4]; }
  // coefficient bytes C[r][0..K) as dwords (4 per dword, little-endian)
  __host__ __device__ const RS_CONST uint32_t* coef_words(int r) const {
    return as_const<uint32_t>(p + plan_coef_offset(k, m) + static_cast<uint32_t>(r) * plan_coef_row(k));
  }
};

// Shard slot s of stripe i lives at
//   s <  k : data   + i*data_sp   + s*shard_pitch
//   s >= k : parity + i*parity_sp + (s-k)*shard_pitch
// (a unified K+M-slot layout is parity = data + k*shard_pitch, parity_sp = data_sp).
struct KernelArgs {
  uint8_t* data;
  uint8_t* parity;
  uint64_t data_sp;
  uint64_t parity_sp;
  uint64_t shard_pitch;
  uint32_t shard_len;
  uint32_t n_stripes;
  uint32_t blocks_per_stripe;  // ceil(ceil(S/16) / 64): 64-column blocks, a partial column included
  uint32_t full_cols;          // S / 16: full 16-B columns
  int32_t k, m;
  uint32_t full_mask;          // (1 << (k+m)) - 1
  uint32_t plan_bytes;
  const uint8_t* plans;            // uniform plan, or plan array (PER_STRIPE)
  const uint32_t* present_masks;   // PER_STRIPE: bit s = shard s present
  const uint32_t* lut;             // PER_STRIPE: missing mask -> plan index
  uint32_t* status;                // PER_STRIPE: bit 0 set if a stripe had < K shards, bit 1 if a
                                   //   stripe missed more than max_out shards
  uint32_t max_out;                // PER_STRIPE: the launch's erasure bound E (set by launch_apply)
  uint8_t* out;                    // null: outputs in place (slot addresses); else the
  uint64_t out_sp;                 //   r-th output of stripe i at out + i*out_sp + r*shard_pitch
  uint32_t* bad;                   // verify: per-stripe bit r set = parity r mismatches
  const uint64_t* stripe_plans;    // PER_STRIPE, generic kernel: plan address per stripe (0 =
                                   //   invalid) instead of mask -> LUT; k+m > 16 batches
  uint32_t encode_net;             // 1: uniform plan is the encode matrix and the generated
                                   //    bitsliced XOR program for (k, m) matches it
  uint32_t data_inputs;            // 1: uniform plan reads data shards 0..k-1 (encode)
  const uint64_t* shard_ptrs;      // pointer-table launches: stripe i's shard s at device address
                                   //   shard_ptrs[i*(k+m) + s] (inputs: present shards; outputs:
                                   //   the missing shards' buffers), each S bytes, 16-B aligned
  const uint32_t* row_offsets;     // packed outputs (out != null): the r-th missing shard of stripe
                                   //   i at out + (row_offsets[i] + r) * shard_pitch (N+1 entries,
                                   //   an exclusive prefix sum of the stripes' erasure counts)
};

// Parity rows the generated bitsliced encode program of (k, m) was derived from
// (rs_xor_networks.inc), or nullptr if there is none.  The engine enables the
// bitsliced kernel only if they equal its runtime encode matrix.
const uint8_t* bitsliced_encode_rows(int k, int m);

// Default workgroups (256 threads) per CU of the batched kernels with k inputs and
// e outputs per stripe (blocks_per_cu = 0 in the launch helpers below).
uint32_t default_blocks_per_cu(int k, int e);

// Launch helpers implemented in rs_kernels.hip (host code; needs hip_runtime.h first).
// e = outputs per stripe to compute (<= m): for per-stripe plans the launch's erasure
// bound (stripes missing more are skipped and flagged, status bit 1).  Returns the
// main kernel's name, or nullptr if the launch failed.  Any shard_len up to
// 0xFFFFFFF0 (column windows).  blocks_per_cu = 0: the chosen kernel's default.
// occ_cap: waves per SIMD the launch may hold (rs_set_occupancy_cap): -1 = the
// kernel's tuned default, 0 = uncapped, c = at most c.
const char* launch_apply(const KernelArgs& a, int e, bool per_stripe, uint32_t blocks_per_cu,
                         uint32_t cu_count, hipStream_t s, int occ_cap = -1);
void launch_copy(const void* src, void* dst, uint64_t bytes, uint32_t grid_blocks, hipStream_t s);
// The main kernel launches that follow on this thread also update `ev` as they
// complete (the kernel's own completion signal, hipExtLaunchKernel) and set *used;
// set_stop_event(nullptr, nullptr) ends it.  Launches that bypass it leave *used alone.
void set_stop_event(hipEvent_t ev, bool* used);
// n uint32 words from src (pinned host memory the GPU maps, or device memory) to dst
// (device memory), on s: per-stripe host masks staged by a kernel on the launch stream.
// n2 > 0: the next n2 words of src go to dst2 in the same launch.
bool launch_words_copy(const uint32_t* src, uint32_t* dst, uint64_t n, hipStream_t s, uint32_t* dst2 = nullptr,
                       uint64_t n2 = 0);
// dst[i] = sum over j < i of popcount(~masks[j] & full) for i <= n (dst has n + 1 words):
// the output row of stripe i's first missing shard in a packed batch; a stripe missing
// more than max_rows counts 0.  One workgroup walks the masks in chunks on s.
bool launch_row_offsets(const uint32_t* masks, uint32_t full, uint32_t max_rows, uint32_t* dst, uint64_t n,
                        hipStream_t s);
// Verify: recompute parity from the data shards (uniform encode plan) and compare
// with the stored parity; a.bad[i] |= bit r for every mismatching parity shard r.
// Per-stripe plans (masks -> LUT) over a table of shard addresses instead of a
// strided layout: every shard its own buffer of exactly S bytes (caller memory the
// coalescer addresses in place).  Loads never touch a byte past the dword holding a
// shard's byte S-1, stores never past byte S-1.  e = the launch's erasure bound.
const char* launch_apply_ptrs(const KernelArgs& a, int e, uint32_t blocks_per_cu, uint32_t cu_count, hipStream_t s);
bool apply_ptrs_supported(int k, int m);  // a specialised pointer-table kernel exists
// a.bad must be zeroed first (launch_verify does it on s).
const char* launch_verify(const KernelArgs& a, uint32_t blocks_per_cu, uint32_t cu_count, hipStream_t s);

}  // namespace rs
