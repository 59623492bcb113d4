// rs_kernels.hip -- CDNA4 (gfx950) kernels for Reed-Solomon encode/reconstruct.
//
// One kernel family computes  Y[e x S] = C[e x K] (x) X[K x S]  over GF(2^8) for a
// batch of independent stripes.  Encode (C = parity rows of the encode matrix,
// [upstream klauspost reedsolomon.go Encode -> codeSomeShards], called from
// internal/ec/ec.go:54-56) and reconstruct (C = composed decode rows over the first
// K present shards, [upstream reconstruct], internal/ec/ec.go:59-61) are the same
// kernel with different coefficient plans.
//
// GF(2^8) multiply by a wave-uniform coefficient f, 4 bytes per VALU op:
//   x = x[2:0] | x[5:3]<<3 | x[7:6]<<6 and multiplication is GF(2)-linear, so
//   f*x = A[x[2:0]] ^ B[x[5:3]] ^ C[x[7:6]]  with 8-, 8- and 4-entry product tables.
//   An 8-entry byte table is exactly the byte pool of one v_perm_b32 (two dwords),
//   so each lookup is ONE v_perm_b32 on 4 packed bytes: no LDS traffic, no
//   data-dependent bank conflicts.  Per (coefficient, data dword): 3 v_perm_b32 +
//   1.5 v_xor3_b32; per data dword 5 ops of index prep shared by all outputs.  The
//   tables (5 dwords per coefficient) are wave-uniform and live in SGPRs.
//
// Memory (HBM-bound streaming; measured pattern study in tools/hbm_probe2.hip):
//   * split layout: data shards of stripe i at data + i*data_sp + s*P (s < K),
//     parity at parity + i*parity_sp + (s-K)*P -- two sequential streams;
//   * grid-stride over tasks (task = one stripe's 1 KiB column block, lane l owns
//     the 16 B at column 64*blk + l of every shard), 1-2 workgroups per CU;
//   * 16-B non-temporal loads and stores (one 1 KiB wave instruction each).
// Every loop trip issues the same vector-memory sequence -- [mask(t+1)] [K loads]
// [E stores] -- with no branch around any of them (lanes past the last column load
// the last column again, and stores that must not land are raw buffer stores the
// hardware drops on its range check), so the compiler's s_waitcnt vmcnt(N) counts
// stay exact and the per-stripe plan lookup of the NEXT task overlaps the current
// task.  A partial last column (S % 16 != 0) is loaded and computed like any other
// (its 16-B column lies inside the slot) and stored byte-exact by the lane that
// holds it, in a wave-uniform branch taken only by a stripe's last block.  Every
// store is a buffer store: in order in vmcnt, unlike flat stores.
//
// Ragged shard lengths (columns not a multiple of the task width, e.g. RS(10+4) at
// 64 KiB objects: 410 columns) waste the idle lanes of each stripe's last task.
// The flat-task kernels (bitsliced encode, scrub, per-stripe out-of-place
// reconstruct) instead cut the batch's columns -- each stripe rounded up to whole
// 128-B lines -- into tasks that may straddle two stripes (round 2).
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <mutex>
#include <type_traits>
#include <utility>
#include <vector>

#include "rs_plan.hpp"

namespace rs {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// RS_PATTERN_ONLY=1 builds the compute-free twin of every reconstruct / encode
// kernel (tools/ceiling_probe.sh): the same launches, tasks, loads and stores, with
// the GF(2^8) arithmetic replaced by one XOR per input dword -- the ceiling of each
// kernel's memory pattern on its shipped launch shape.  Its bytes are NOT codewords.
#ifndef RS_PATTERN_ONLY
#define RS_PATTERN_ONLY 0
#endif

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

// 3-input XOR in one VALU op: gfx950 has no v_xor3_b32, but v_bitop3_b32 evaluates
// any 3-input truth table (0x96 = a ^ b ^ c).
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// perm(hi, lo, sel) picks byte sel (0..7) of the 8-byte pool {hi:lo}.
__device__ __forceinline__ uint32_t lookup3(const Idx3& i, uint32_t t0, uint32_t t1, uint32_t t2, uint32_t t3,
                                            uint32_t t4) {
  return xor3(__builtin_amdgcn_perm(t1, t0, i.a), __builtin_amdgcn_perm(t3, t2, i.b),
              __builtin_amdgcn_perm(0u, t4, i.c));
}

__device__ __forceinline__ u32x4 load16(const uint8_t* p) {
  return __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
}

// 16-B non-temporal buffer load: an offset past the descriptor's range fetches
// nothing and returns zeros.
__device__ __forceinline__ u32x4 bload16(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
  return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 2 /* nt */));
}

__device__ __forceinline__ void store16(uint8_t* p, u32x4 v) {
  __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(p));
}

// Stores the first nbytes (< 16) of v at a 16-B aligned p with at most 4 naturally
// aligned stores (8, 4, 2, 1 B) instead of one store per byte.
__device__ __forceinline__ void store_tail(uint8_t* p, u32x4 v, uint32_t nbytes) {
  uint32_t q = 0;  // bytes stored so far (multiple of the next store's size)
  if (nbytes & 8u) {
    *reinterpret_cast<uint2*>(p) = make_uint2(v[0], v[1]);
    q = 8;
  }
  if (nbytes & 4u) {
    *reinterpret_cast<uint32_t*>(p + q) = v[q >> 2];
    q += 4;
  }
  const uint32_t w = q < 16u ? v[q >> 2] : 0u;  // dword holding the remaining 1-3 bytes
  if (nbytes & 2u) {
    *reinterpret_cast<uint16_t*>(p + q) = static_cast<uint16_t>(w);
    q += 2;
  }
  if (nbytes & 1u) p[q] = static_cast<uint8_t>(w >> (8 * (q & 3u)));
}

__device__ __forceinline__ uint32_t wave_uniform(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

// Global wave index of a grid-stride kernel (256-thread blocks).  Blocks are dealt
// round-robin over the 8 XCDs, so consecutive tasks run on different XCDs; that
// placement is kept on purpose: giving each XCD a contiguous eighth of every pass
// measured level for RS(4+2) and 3-4 points slower for RS(10+4)
// (profiles/r02c_ab_xcd_remap_rejected.log).
__device__ __forceinline__ uint32_t wave_index() {
  return wave_uniform(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6));
}

// Offset past every descriptor's range: a buffer store there is dropped.
constexpr uint32_t kDropOffset = 0x80000000u;

// Pins a wave-uniform pointer into SGPRs so loads through it stay scalar.
__device__ __forceinline__ const uint8_t* uniform_ptr(const uint8_t* p) {
  const uint64_t v = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(v));
  const uint32_t hi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(v >> 32));
  return reinterpret_cast<const uint8_t*>((static_cast<uint64_t>(hi) << 32) | lo);
}

// Raw buffer descriptor over [base, base + 2 GiB); base must be wave-uniform.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t out_rsrc(uint8_t* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(uniform_ptr(base)), 0, 0x7FFFFFFF, 0x00020000);
}

// Cache policy of the output stores (the aux / cpol operand of the buffer store).
// gfx950: bit 1 = NT (streaming), bit 4 = SC1 (device scope: the store writes
// through the XCD's L2).  Measured by read:write mix (profiles/r03l_ab_store_*.log,
// interleaved A/B, >= 100 ms per kernel): a launch that reads K >= 8 inputs per
// output row it writes (1-erasure reconstruct of RS(8+4) / RS(10+4)) streams fastest
// with device-scope write-through stores (RS(8+4) 72.0 -> 76.7 %, RS(10+4) 65.3 ->
// 69.1 % of 8 TB/s); RS(10+4) with two rows per stripe with NT + SC1 (68.6 -> 70.0 %);
// every other mix (RS(4+2), RS(8+4) 2-erasure, encodes) with NT alone, as before
// (SC1 there costs 1.5-8 points).
constexpr int kCpolNt = 2;
constexpr int kCpolSc1 = 16;
template <int K, int E>
constexpr int out_cpol() {
  return (E == 1 && K >= 8) ? kCpolSc1 : (E == 2 && K >= 10) ? (kCpolSc1 | kCpolNt) : kCpolNt;
}
// The segmented flat E = m kernel's 1-row path stores NT (round 5, same-process A/B,
// profiles/r05h_ab_same_fp1.log, RS(10+4) 64 KiB): unbounded 1-erasure 68.4 ->
// 71.5 %, mixed 0..4 61.7 -> 63.1 %, mixed 1..4 66.8 -> 68.4 %, others level; the
// bounded E = 1 kernels keep SC1 (NT there: -2.9 flat, -5.1 stripe-aligned RS(8+4),
// profiles/r05g_ab_same_cpol.log).
constexpr int kCpolFlatPath1 = kCpolNt;

// Per-stripe kernels sized for E > 2 outputs (device masks without a caller bound:
// E = M) compute only the rows a task's stripe(s) miss and then pick, in a
// wave-uniform branch, the store sequence of that row count: 1 or 2 rows store with
// their own policy (path_cpol below) and issue no dropped stores for the other rows,
// more rows store E rows with out_cpol<K, E> (round 4).
// Every store instruction has one policy for all its lanes and every 128-B output
// line one writer instruction.
// Store policy of those paths: the 1-row path with out_cpol<K, 1> (SC1 for K >= 8),
// the 2-row path NT.  Interleaved A/B against the bounded kernels' policies
// (profiles/r04t_ab_p2nt.log, RS(10+4) 64 KiB, >= 100 ms per point, 3 rounds):
// unbounded 2-erasure 69.5 -> 70.5 % (median), mixed 0..4 erasures 59.5-59.8 ->
// 60.6 % (host masks 56.9-57.0 -> 57.6-57.7 %), mixed 1..4 65.3-65.8 -> 66.7-66.9 %;
// the bounded E = 2 kernel keeps NT|SC1.  out_cpol<K, E> on every path (all NT) was
// 4-7 points slower on 1-erasure (profiles/r04s_ab_em_cpol_mix.log).
template <int K, int E, int NR>
constexpr int path_cpol() {
  return NR == 1 ? out_cpol<K, 1>() : kCpolNt;
}
// Launch bounds asking the compiler to fit the apply_kernel instantiations with K <= 8
// and E <= 2 into 4 waves per SIMD.  The uniform-plan RS(8+4) 2-erasure kernel then
// drops from 135 to 117 VGPRs (3 -> 4 waves, no scratch): same-process A/B
// (profiles/r05n_ab_lb4.log) one pattern for the batch +6.0 points out of place, +3.9
// in place; every other shape level.  K = 10 with E >= 2 would spill to scratch at 4
// waves and is left alone.
constexpr int kApplyMinWaves = 4;

// 16-B store at base + off, or nothing at all when !live: a raw buffer
// store whose offset then fails the range check, so the hardware drops it -- no
// branch around the store and no sink line to write back.  off < 2 GiB.
template <int CPOL = kCpolNt>
__device__ __forceinline__ void store16_or_drop(uint8_t* base, uint32_t off, bool live, u32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(v, out_rsrc(base), live ? off : kDropOffset, 0, CPOL);
}

typedef int i32x2 __attribute__((ext_vector_type(2)));

// The first nb (1..15, wave-uniform) bytes of v at base + off in at most four
// naturally aligned buffer stores (8, 4, 2, 1 B), landing only for `live` lanes.
// Same cache policy as the kernel's full-column stores (one line may get both).
template <int CPOL = kCpolNt>
__device__ __forceinline__ void store_part_or_drop(uint8_t* base, uint32_t off, bool live, u32x4 v, uint32_t nb) {
  const auto rsrc = out_rsrc(base);
  const uint32_t o = live ? off : kDropOffset;
  uint32_t q = 0;  // bytes stored so far
  if (nb & 8u) {
    __builtin_amdgcn_raw_buffer_store_b64(i32x2{static_cast<int>(v[0]), static_cast<int>(v[1])}, rsrc, o, 0, CPOL);
    q = 8;
  }
  uint32_t w = q ? v[2] : v[0];  // dword holding byte q
  if (nb & 4u) {
    __builtin_amdgcn_raw_buffer_store_b32(static_cast<int>(w), rsrc, live ? off + q : kDropOffset, 0, CPOL);
    q += 4;
    w = q == 12u ? v[3] : v[1];
  }
  if (nb & 2u) {
    __builtin_amdgcn_raw_buffer_store_b16(static_cast<short>(w), rsrc, live ? off + q : kDropOffset, 0, CPOL);
    q += 2;
    w >>= 16;
  }
  if (nb & 1u)
    __builtin_amdgcn_raw_buffer_store_b8(static_cast<char>(w), rsrc, live ? off + q : kDropOffset, 0, CPOL);
}

// The first nb (1..15, wave-uniform) bytes of v at voff (+ soff) of descriptor r in at
// most four naturally aligned buffer stores, landing only for `live` lanes (the
// range check applies to voff: a dropped lane's offset is kDropOffset).
template <int CPOL = kCpolNt>
__device__ __forceinline__ void store_part_rsrc(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff, bool live,
                                                u32x4 v, uint32_t nb) {
  const uint32_t o = live ? voff : kDropOffset;
  uint32_t q = 0;  // bytes stored so far
  if (nb & 8u) {
    __builtin_amdgcn_raw_buffer_store_b64(i32x2{static_cast<int>(v[0]), static_cast<int>(v[1])}, r, o, soff, CPOL);
    q = 8;
  }
  uint32_t w = q ? v[2] : v[0];  // dword holding byte q
  if (nb & 4u) {
    __builtin_amdgcn_raw_buffer_store_b32(static_cast<int>(w), r, live ? voff + q : kDropOffset, soff, CPOL);
    q += 4;
    w = q == 12u ? v[3] : v[1];
  }
  if (nb & 2u) {
    __builtin_amdgcn_raw_buffer_store_b16(static_cast<short>(w), r, live ? voff + q : kDropOffset, soff, CPOL);
    q += 2;
    w >>= 16;
  }
  if (nb & 1u) __builtin_amdgcn_raw_buffer_store_b8(static_cast<char>(w), r, live ? voff + q : kDropOffset, soff, CPOL);
}

// Shard slot s of stripe i (s < k: data region, else parity region).
__device__ __forceinline__ uint8_t* slot_ptr(const KernelArgs& a, int k, uint32_t stripe, uint32_t s) {
  return s < static_cast<uint32_t>(k)
             ? a.data + static_cast<uint64_t>(stripe) * a.data_sp + static_cast<uint64_t>(s) * a.shard_pitch
             : a.parity + static_cast<uint64_t>(stripe) * a.parity_sp +
                   static_cast<uint64_t>(s - static_cast<uint32_t>(k)) * a.shard_pitch;
}

// r-th output of stripe i: in place (its shard slot) or out of place.
__device__ __forceinline__ uint8_t* out_ptr(const KernelArgs& a, int k, uint32_t stripe, uint32_t r, uint32_t slot) {
  if (a.out && a.row_offsets)  // packed: the stripe's rows start at its row offset
    return a.out + (static_cast<uint64_t>(as_const<uint32_t>(a.row_offsets)[stripe]) + r) * a.shard_pitch;
  return a.out ? a.out + static_cast<uint64_t>(stripe) * a.out_sp + static_cast<uint64_t>(r) * a.shard_pitch
               : slot_ptr(a, k, stripe, slot);
}

// Slot index of the i-th set bit of a wave-uniform mask walk: s = lowest set bit.
__device__ __forceinline__ uint32_t pop_low(uint32_t& bits) {
  const uint32_t s = static_cast<uint32_t>(__builtin_ctz(bits | 0x80000000u));
  bits &= bits - 1u;
  return s;
}

// ---------------------------------------------------------------------------
// Rows [R0, R0 + NR) of one task: y[r] = sum_c C[R0 + r][c] (x) x[c].
// Input-outer order (as upstream codeSomeShards): one input's chunk indices and
// NR x 5 table dwords live at a time; products of inputs c-1 and c are folded into
// the accumulator with one 3-input XOR.  The scheduling barrier per input stops the
// compiler from hoisting every input's tables into SGPRs at once (K*NR*5 dwords,
// e.g. 100 for RS(10+4) x 2 rows -> SGPR spills through VGPR lanes).
template <int K, int M, int R0, int NR>
__device__ __forceinline__ void gf_rows(const uint8_t* plan, const u32x4 (&x)[K], u32x4 (&y)[NR]) {
  if constexpr (RS_PATTERN_ONLY) {
#pragma unroll
    for (int r = 0; r < NR; ++r) {
      y[r] = x[0] + static_cast<uint32_t>(R0 + r);
#pragma unroll
      for (int c = 1; c < K; ++c) y[r] ^= x[c];
    }
    return;
  }
  u32x4 pend[NR];
#pragma unroll
  for (int r = 0; r < NR; ++r) y[r] = u32x4{0u, 0u, 0u, 0u};
#pragma unroll
  for (int c = 0; c < K; ++c) {
    Idx3 ix[4];
#pragma unroll
    for (int d = 0; d < 4; ++d) ix[d] = split3(x[c][d]);
    // one opaque base per input: the scalar load merger cannot fuse this input's
    // table loads with later inputs' (which would pin them in SGPRs)
    const uint8_t* tcol = plan;
    if constexpr (K * NR * 5 > 48) asm volatile("" : "+s"(tcol));
    const PlanView pc(tcol, K, M);
    auto row = [&](auto r_tag) {
      constexpr int r = decltype(r_tag)::value;
      const RS_CONST uint32_t* tb = pc.quad(R0 + r, c);
      const uint32_t q0 = tb[0], q1 = tb[1], q2 = tb[2], q3 = tb[3], q4 = pc.c4(R0 + r, c);
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        const uint32_t prod = lookup3(ix[d], q0, q1, q2, q3, q4);
        if (c & 1)
          y[r][d] = xor3(y[r][d], pend[r][d], prod);
        else if (c == K - 1)
          y[r][d] ^= prod;
        else
          pend[r][d] = prod;
      }
    };
    row(std::integral_constant<int, 0>{});
    if constexpr (NR > 1) row(std::integral_constant<int, 1>{});
    if constexpr (NR > 2) row(std::integral_constant<int, 2>{});
    if constexpr (NR > 3) row(std::integral_constant<int, 3>{});
    if (c + 1 < K) __builtin_amdgcn_sched_barrier(0);
  }
}

// One row r of a task from the inputs' precomputed chunk indices ix[c][d].  Each
// input's table dwords hang off their own opaque base, so the scalar unit fetches
// them per input and they are never all held in SGPRs at once.  (Rejected, measured:
// coefficient-indexed tables from a 5-KiB compile-time table instead of the plan's
// table block, -0.8 to -1.7 points, profiles/r05j_ab_coef.log; several inputs per
// fetch group.)
template <int K, int M>
__device__ __forceinline__ u32x4 gf_row_ix(const uint8_t* plan, const Idx3 (&ix)[K][4], int r) {
  u32x4 y{0u, 0u, 0u, 0u}, pend{0u, 0u, 0u, 0u};
  if constexpr (RS_PATTERN_ONLY) {
#pragma unroll
    for (int c = 0; c < K; ++c)
#pragma unroll
      for (int d = 0; d < 4; ++d) y[d] ^= ix[c][d].a + static_cast<uint32_t>(r);
    return y;
  }
#pragma unroll
  for (int c = 0; c < K; ++c) {
    const uint8_t* tg = plan;
    asm volatile("" : "+s"(tg));  // one opaque base per input: tables never all in SGPRs
    const PlanView pc(tg, K, M);
    const RS_CONST uint32_t* tb = pc.quad(r, c);
    const uint32_t q0 = tb[0], q1 = tb[1], q2 = tb[2], q3 = tb[3], q4 = tb[4];
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      const uint32_t prod = lookup3(ix[c][d], q0, q1, q2, q3, q4);
      if (c & 1)
        y[d] = xor3(y[d], pend[d], prod);
      else if (c == K - 1)
        y[d] ^= prod;
      else
        pend[d] = prod;
    }
    if (c + 1 < K) __builtin_amdgcn_sched_barrier(0);
  }
  return y;
}

// ---------------------------------------------------------------------------
// Main kernel: compile-time K, plan layout M, E outputs per task (M for encode,
// #erasures for a uniform reconstruct, the batch's bound for per-stripe patterns).
//
// Uniform plans (encode, one erasure pattern for the whole batch): the input and
// output slots are resolved once per launch, so a task's K loads issue at its top
// with addresses from loop-invariant SGPRs.  (Round 2 loaded the plan's slot list
// per task behind an s_waitcnt vmcnt(0) that also drained the previous task's
// stores: config 3's uniform 4 KiB patterns fell from 72-77 % to 67-70 %.)
//
// Per-stripe batches sized for E > 2 outputs (device masks: E = M) split every
// input's bytes into chunk indices once (K x 12 VGPRs) and then compute only the
// rows the stripe misses, one row at a time (gf_row_ix), in wave-uniform branches
// that end in the store sequence of that row count (round 4).
// A stripe missing more than E shards (possible with device masks under a caller's
// max_missing bound) is skipped and flagged (status bit 1).
// Every trip issues the same loads; the wave-uniform branches differ only in VALU
// work and in how many stores end the trip, so the compiler's vmcnt bookkeeping
// stays exact (a branch around the loads does not: `HISTORY.md` §A.5).
template <int K, int M, int E, bool PER_STRIPE>
__global__ __launch_bounds__(256, (K <= 8 && E <= 2) ? kApplyMinWaves : 1) void apply_kernel(
    const KernelArgs a) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wave = wave_index();
  const uint32_t nwaves = gridDim.x * (blockDim.x >> 6);
  const uint32_t bps = a.blocks_per_stripe;   // the partial last column included
  const uint32_t ntasks = a.n_stripes * bps;  // host guarantees < 2^32
  const uint32_t cols = (a.shard_len + 15u) >> 4;
  const uint32_t nb = a.shard_len & 15u;      // bytes of a partial last column (0: none)
  uint32_t bad = 0u;

  // mask of task t's stripe; every lane loads the same word (one request)
  auto load_mask = [&](uint32_t t) -> uint32_t {
    const uint32_t tt = t < ntasks ? t : ntasks - 1u;
    return a.present_masks[tt / bps];
  };

  // uniform plan: slots once per launch
  uint32_t uin[PER_STRIPE ? 1 : K], uout[PER_STRIPE ? 1 : E];
  uint32_t u_nout = 0u;
  if constexpr (!PER_STRIPE) {
    const PlanView pv0(uniform_ptr(a.plans), K, M);
    u_nout = wave_uniform(pv0.n_out());
#pragma unroll
    for (int c = 0; c < K; ++c) uin[c] = wave_uniform(pv0.in_idx(c));
#pragma unroll
    for (int r = 0; r < E; ++r) uout[r] = wave_uniform(static_cast<uint32_t>(r) < u_nout ? pv0.out_idx(r) : 0u);
  }

  // Deferred stores (round 4): per-stripe RS(4+2) launches issue a task's stores
  // behind the NEXT task's loads, so the wave computes while they drain -- vmcnt
  // counts loads and stores in order, and stores issued last no longer hold up the
  // next task's first input.  Interleaved A/B (profiles/r04f_ab_defer_twopass.log,
  // >= 100 ms per point): RS(4+2) 4 KiB 2-erasure 73.3 -> 74.5 %, 64 KiB 73.8 -> 74.2 %,
  // 1-erasure 76.9 -> 77.1 %; the uniform encode 76.7 -> 76.4 % and RS(8+4) bounded
  // 1-erasure 77.4 -> 77.0 % lose, so those keep the in-order stores.
  // Kept here: the previous task's rows, row bases and per-lane offsets (kDropOffset:
  // dropped).
  constexpr bool kDefer = PER_STRIPE && K <= 4 && E <= 2;
  constexpr int kCp = out_cpol<K, E>();
  // (before the first task every store is dropped: the same store sequence on every
  // trip keeps the compiler's vmcnt counts exact)
  [[maybe_unused]] u32x4 py[E];
  [[maybe_unused]] uint8_t* pbase[E];
  [[maybe_unused]] uint32_t poff[E], ppoff[E];
  [[maybe_unused]] bool ppart = false;
#pragma unroll
  for (int r = 0; r < E; ++r) {
    py[r] = u32x4{0u, 0u, 0u, 0u};
    pbase[r] = a.out ? a.out : a.parity;
    poff[r] = ppoff[r] = kDropOffset;
  }
  [[maybe_unused]] auto flush = [&]() {
#pragma unroll
    for (int r = 0; r < E; ++r) __builtin_amdgcn_raw_buffer_store_b128(py[r], out_rsrc(pbase[r]), poff[r], 0, kCp);
    if (ppart) {  // wave-uniform: the task held its stripe's partial column
#pragma unroll
      for (int r = 0; r < E; ++r) store_part_or_drop<kCp>(pbase[r], ppoff[r], ppoff[r] != kDropOffset, py[r], nb);
    }
  };

  uint32_t mask = 0u;
  if (PER_STRIPE && wave < ntasks) mask = load_mask(wave);
  for (uint32_t t = wave; t < ntasks; t += nwaves) {
    const uint32_t stripe = t / bps;
    const uint32_t blk = t - stripe * bps;
    const uint8_t* plan = a.plans;
    [[maybe_unused]] bool work = true;  // the stripe has rows to fill
    if (PER_STRIPE) {
      const uint32_t present = __builtin_amdgcn_readfirstlane(mask);  // waits for this mask only
      mask = load_mask(t + nwaves);                                  // next task's mask in flight
      const uint32_t missing = (~present) & a.full_mask;
      uint32_t pid = as_const<uint32_t>(a.lut)[missing];
      bad |= (pid == kPlanInvalid) ? 1u : 0u;
      pid = (pid == kPlanInvalid) ? 0u : pid;  // plan 0 = nothing missing -> every store dropped
      if constexpr (E < M) {  // more erasures than this launch's bound: skip, flag
        const bool over = static_cast<uint32_t>(__builtin_popcount(missing)) > static_cast<uint32_t>(E);
        bad |= over ? 2u : 0u;
        pid = over ? 0u : pid;
      }
      plan = uniform_ptr(a.plans + static_cast<uint64_t>(pid) * a.plan_bytes);
      work = pid != 0u;
    }
    if constexpr (K * ((PER_STRIPE && E > 2) ? 2 : E) * 5 > 48) {
      // Too many table dwords to keep resident in SGPRs across trips: make the plan
      // pointer opaque per trip so its loads are not hoisted out of the loop (LICM
      // would otherwise spill them through VGPR lanes: v_writelane/v_readlane).
      asm volatile("" : "+s"(plan));
    }
    const PlanView pv(plan, K, M);
    const uint32_t col = blk * 64u + lane;
    const bool full = col < a.full_cols;
    // clamped, never branched: a lane past the end re-reads the last column (lines
    // the wave's other lanes fetch anyway) and its stores are dropped
    const uint32_t off = (col < cols ? col : cols - 1u) * 16u;

    u32x4 x[K];
    if constexpr (PER_STRIPE && E > 2) {
      // Launches sized for E = M (device masks without a bound: a scan's batch of intact
      // and damaged stripes) load through a descriptor over each input's slot
      // (range-checked), and an intact or skipped stripe's loads are all out of range:
      // nothing is fetched, and every trip keeps the same load sequence (round 4).
      // Interleaved A/B (profiles/r04j_ab_psbuf.log): RS(8+4) mixed 0..4 erasures
      // 57.0 -> 66.1 % (host masks 49.7 -> 56.7 %), uniform 1-erasure 76.2 -> 77.1 %;
      // the E <= 2 kernels lose 0.8-2.0 points with these loads, so they keep global
      // loads (their callers know the stripes are damaged).
      const uint32_t loff = work ? off : kDropOffset;
#pragma unroll
      for (int c = 0; c < K; ++c) {
        // range: the slot's columns (cols * 16 <= 1 GiB + 16 per column window), never
        // the pitch, which may exceed 32 bits in plane-major layouts
        const auto r = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<uint8_t*>(uniform_ptr(slot_ptr(a, K, stripe, pv.in_idx(c)))), 0, cols * 16u, 0x00020000);
        x[c] = bload16(r, loff, 0);
      }
    } else {
      // E <= 2 per-stripe launches run one task per wave (a full grid), so a task of an
      // intact (or skipped) stripe ends its wave here: no loads, no stores.  (Rejected,
      // round 6, profiles/r06p_ab_mslots.log: the input slots taken from the mask so
      // the loads issue before the LUT -> plan chain returns -- level, -0.6 to +0.7.)  RS(4+2)
      // device masks without a bound are this kernel (E = M = 2), and a scan's mixed
      // batch had every intact stripe read for nothing.
      if constexpr (PER_STRIPE) {
        if (!work) continue;
      }
#pragma unroll
      for (int c = 0; c < K; ++c) x[c] = load16(slot_ptr(a, K, stripe, PER_STRIPE ? pv.in_idx(c) : uin[c]) + off);
    }

    const uint32_t n_out = PER_STRIPE ? pv.n_out() : u_nout;
    // stores rows [0, NR) of the task (the rest of the launch's E rows need none)
    // with cache policy CPOL; dropped per lane past the stripe's outputs
    auto emit = [&](auto nr_tag, auto cpol_tag, const auto& yy) {
      constexpr int NR = decltype(nr_tag)::value;
      constexpr int CPOL = decltype(cpol_tag)::value;
#pragma unroll
      for (int r = 0; r < NR; ++r)
        store16_or_drop<CPOL>(out_ptr(a, K, stripe, r, PER_STRIPE ? pv.out_idx(r) : uout[r]), off,
                              full && static_cast<uint32_t>(r) < n_out, yy[r]);
      if (nb != 0u && blk + 1u == bps) {  // wave-uniform: this task holds the stripe's partial column
        const bool part = col == a.full_cols;
#pragma unroll
        for (int r = 0; r < NR; ++r)
          store_part_or_drop<CPOL>(out_ptr(a, K, stripe, r, PER_STRIPE ? pv.out_idx(r) : uout[r]), off,
                                   part && static_cast<uint32_t>(r) < n_out, yy[r], nb);
      }
    };
    u32x4 y[E];
    if constexpr (PER_STRIPE && E > 2) {
      // An intact or skipped stripe: its loads fetched nothing, and it has no row to
      // compute either (round 6, same-process A/B, profiles/r06c_ab_fast.log: RS(8+4)
      // 64 KiB mixed 0..4 erasures 71.9 -> 73.9 % of 8 TB/s; it used to compute and
      // drop one row).
      if (!work) continue;
    }
    if constexpr (PER_STRIPE && E > 2) {
      // every input's chunk indices once, then only the rows this stripe misses
      // (wave-uniform branches): a 1-erasure stripe computes one row, a 2-erasure
      // stripe two.  Round 2: RS(10+4) 64 KiB 1-erasure 63.5-66.9 -> 69.4-70.9 %,
      // 2-erasure 62.9-65.1 -> 65.9-67.1 %, 4-erasure 47.5-48.7 -> 57.3-57.9 %
      // (profiles/r02c_ab_ix_rows.log).  Input-outer passes of <= 2 rows instead
      // (round 4) lost 9-10 points on 4-erasure and mixed batches
      // (profiles/r04g_ab_twopass.log, `HISTORY.md` §A.5); input-outer per row count,
      // as the flat kernel does since round 6, lost 8-14 here (166 VGPRs, 252 SGPR
      // spills in this grid-stride loop, profiles/r06r_ab_psinout.log).
      Idx3 ix[K][4];
#pragma unroll
      for (int c = 0; c < K; ++c)
#pragma unroll
        for (int d = 0; d < 4; ++d) ix[c][d] = split3(x[c][d]);
      // (Storing each of 3+ rows as soon as it is computed, as the flat kernel does,
      // lost 2.3-4.2 points here: SGPRs spill, profiles/r05i_ab_emit_each.log.)
      const uint32_t nrow = pv.n_out();
      y[0] = gf_row_ix<K, M>(plan, ix, 0);
#pragma unroll
      for (int r = 1; r < E; ++r) {
        y[r] = y[0];  // dropped unless computed
        if (static_cast<uint32_t>(r) < nrow) y[r] = gf_row_ix<K, M>(plan, ix, r);
      }
      if (n_out <= 2u) {  // wave-uniform: the bounded kernels' store policy
        if (n_out <= 1u)
          emit(std::integral_constant<int, 1>{}, std::integral_constant<int, path_cpol<K, E, 1>()>{}, y);
        else
          emit(std::integral_constant<int, 2>{}, std::integral_constant<int, path_cpol<K, E, 2>()>{}, y);
        continue;
      }
    } else if constexpr (kDefer) {
      flush();  // the previous task's stores, behind this task's loads
      if (E == 2 && n_out <= 1u) {
        // wave-uniform: a 1-erasure stripe of a scan computes one row, not two (round
        // 6, profiles/r06u_ab_nout1.log: RS(4+2) mixed 0..2 erasures at 4 KiB / 64 KiB
        // / 1 MiB +2.0 / +2.7 / +1.3 points, host masks +2.2; the same branch in the
        // k >= 8 kernels cost RS(8+4) bounded 2-erasure 1.9)
        u32x4 y1[1];
        gf_rows<K, M, 0, 1>(plan, x, y1);
#pragma unroll
        for (int r = 0; r < E; ++r) y[r] = y1[0];
      } else {
        gf_rows<K, M, 0, E>(plan, x, y);
      }
      const bool part = col == a.full_cols;
#pragma unroll
      for (int r = 0; r < E; ++r) {
        const bool row = static_cast<uint32_t>(r) < n_out;
        py[r] = y[r];
        pbase[r] = out_ptr(a, K, stripe, r, PER_STRIPE ? pv.out_idx(r) : uout[r]);
        poff[r] = full && row ? off : kDropOffset;
        ppoff[r] = part && row ? off : kDropOffset;
      }
      ppart = nb != 0u && blk + 1u == bps;
      continue;
    } else {
      gf_rows<K, M, 0, E>(plan, x, y);
    }
    emit(std::integral_constant<int, E>{}, std::integral_constant<int, out_cpol<K, E>()>{}, y);
  }
  if constexpr (kDefer) flush();
  if (PER_STRIPE && bad && lane == 0u) atomicOr(a.status, bad);
}

// ---------------------------------------------------------------------------
// Generic kernel: runtime K (<= kMaxK) and M, outputs in groups of 4, inline tail
// handling.  Serves the (K, M) shapes without a specialisation.
template <bool PER_STRIPE>
__global__ __launch_bounds__(256) void apply_kernel_generic(const KernelArgs a) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wave = wave_index();
  const uint32_t nwaves = gridDim.x * (blockDim.x >> 6);
  const uint32_t bps = a.blocks_per_stripe;
  const uint32_t ntasks = a.n_stripes * bps;
  const int K = a.k, M = a.m;

  for (uint32_t t = wave; t < ntasks; t += nwaves) {
    const uint32_t stripe = t / bps;
    const uint32_t blk = t - stripe * bps;
    const uint8_t* plan = a.plans;
    if (PER_STRIPE && a.stripe_plans) {  // a plan per stripe (any k+m)
      plan = reinterpret_cast<const uint8_t*>(as_const<uint64_t>(a.stripe_plans)[stripe]);
      if (!plan) {
        if (lane == 0 && blk == 0) atomicOr(a.status, 1u);
        continue;
      }
    } else if (PER_STRIPE) {
      const uint32_t present = as_const<uint32_t>(a.present_masks)[stripe];
      const uint32_t missing = (~present) & a.full_mask;
      const uint32_t pid = as_const<uint32_t>(a.lut)[missing];
      if (pid == kPlanInvalid) {
        if (lane == 0 && blk == 0) atomicOr(a.status, 1u);
        continue;
      }
      plan = a.plans + static_cast<uint64_t>(pid) * a.plan_bytes;
    }
    const PlanView pv(plan, K, M);
    const int n_out = static_cast<int>(pv.n_out());
    if (PER_STRIPE && static_cast<uint32_t>(n_out) > a.max_out) {  // beyond the launch's erasure bound
      if (lane == 0 && blk == 0) atomicOr(a.status, 2u);
      continue;
    }
    const uint32_t off = (blk * 64u + lane) * 16u;
    if (n_out == 0 || off >= a.shard_len) continue;
    const uint32_t tail = a.shard_len - off;

    for (int r0 = 0; r0 < n_out; r0 += 4) {
      u32x4 y[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) y[q] = u32x4{0u, 0u, 0u, 0u};
      for (int c = 0; c < K; ++c) {
        const u32x4 x = load16(slot_ptr(a, K, stripe, pv.in_idx(c)) + off);
        Idx3 ix[4];
#pragma unroll
        for (int d = 0; d < 4; ++d) ix[d] = split3(x[d]);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          if (r0 + q >= n_out) break;
          const RS_CONST uint32_t* tb = pv.quad(r0 + q, c);
          const uint32_t q0 = tb[0], q1 = tb[1], q2 = tb[2], q3 = tb[3], q4 = pv.c4(r0 + q, c);
#pragma unroll
          for (int d = 0; d < 4; ++d) y[q][d] ^= lookup3(ix[d], q0, q1, q2, q3, q4);
        }
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (r0 + q >= n_out) break;
        uint8_t* dst = out_ptr(a, K, stripe, r0 + q, pv.out_idx(r0 + q)) + off;
        if (tail >= 16u)
          store16(dst, y[q]);
        else
          store_tail(dst, y[q], tail);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Bitsliced encode for the fixed encode matrices of the specialised shapes.
//
// GF(2^8) multiplication by a constant is an 8x8 matrix over GF(2).  With 32
// bytes of a shard bitsliced into 8 dwords (plane j = bit j of each byte), a
// parity plane is the XOR of the data planes its bit matrix selects: full-rate
// v_xor_b32 where the lookup kernel spends half-rate v_perm_b32 / v_bitop3_b32
// (tools/valu_probe.hip).  The encode matrix of RS(K, M) is fixed, so the XOR
// program is generated at build time with shared subexpressions
// (tools/gen_xor_networks.py -> rs_xor_networks.inc).  Per 32-byte column of a
// stripe: one 8x8 bit transpose per data and per parity shard (3 delta-swap
// stages, its own inverse) plus the program (RS(10+4): 682 XORs vs the lookup
// kernel's 320 perms + 160 bitop3 + 80 index ops for the same bytes).
template <int K, int M>
struct BsNet {
  static constexpr bool kAvailable = false;
};
template <int K, int M, int C>
__device__ __forceinline__ void bs_step(const uint32_t (&x)[8], uint32_t (&y)[8 * M]);
// Pair programs of the 1 KiB-task encode (encode_bs16_kernel): shapes whose encode
// matrix satisfies C[r ^ 1][c] = C[r][c ^ 1] (tools/gen_xor_networks.py).
template <int K, int M>
struct Bs16Net {
  static constexpr bool kAvailable = false;
};
template <int K, int M, int P>
__device__ __forceinline__ void bs16_step(const uint32_t (&x)[8], uint32_t (&ya)[4 * M], uint32_t (&yb)[4 * M]);

#include "rs_xor_networks.inc"

// 8x8 bit transpose in every byte lane across 8 dwords: afterwards dword r, byte
// b, bit q = bit r of byte b of the original dword q.  An involution.
// Each delta swap is two shifts and two bit selects (v_bitop3_b32 0xCA = m ? x : y):
// 4 VALU instructions instead of the XOR form's 5 (tools/valu_probe.hip: shifts and
// bitop3 issue at the same half rate, so this saves issue cycles too).
__device__ __forceinline__ void transpose8(uint32_t (&d)[8]) {
  auto swap = [&](int a, int b, int sh, uint32_t mask) {
    const uint32_t oa = d[a], ob = d[b];
    d[b] = __builtin_amdgcn_bitop3_b32(mask, oa >> sh, ob, 0xCA);
    d[a] = __builtin_amdgcn_bitop3_b32(mask << sh, ob << sh, oa, 0xCA);
  };
  swap(0, 4, 4, 0x0F0F0F0Fu);
  swap(1, 5, 4, 0x0F0F0F0Fu);
  swap(2, 6, 4, 0x0F0F0F0Fu);
  swap(3, 7, 4, 0x0F0F0F0Fu);
  swap(0, 2, 2, 0x33333333u);
  swap(1, 3, 2, 0x33333333u);
  swap(4, 6, 2, 0x33333333u);
  swap(5, 7, 2, 0x33333333u);
  swap(0, 1, 1, 0x55555555u);
  swap(2, 3, 1, 0x55555555u);
  swap(4, 5, 1, 0x55555555u);
  swap(6, 7, 1, 0x55555555u);
}

// One lane-column of a flat task: global column g = (stripe s0, column c0 + i) of the
// batch's N x cols columns, i < 64 <= cols, so the column lies in stripe s0 or s0+1.
struct FlatCol {
  uint32_t col;   // column within its stripe
  uint32_t doff;  // byte offset from the task's data stripe base (next stripe: + data_sp)
  uint32_t poff;  // same for parity
  bool live;      // the stripe exists (the batch's last task may run past the end)
};

__device__ __forceinline__ FlatCol flat_col(const KernelArgs& a, uint32_t s0, uint32_t c, uint32_t cstride,
                                            uint32_t cols) {
  const bool next = c >= cstride;
  FlatCol f;
  f.col = next ? c - cstride : c;
  f.live = s0 + (next ? 1u : 0u) < a.n_stripes;
  // a dead lane re-reads the task's first column (in the batch) and stores nothing;
  // a lane in the line-alignment gap (col >= cols) re-reads its stripe's last column
  const uint32_t col = f.live ? min(f.col, cols - 1u) : 0u;
  const bool nx = f.live && next;
  f.doff = (nx ? static_cast<uint32_t>(a.data_sp) : 0u) + col * 16u;
  f.poff = (nx ? static_cast<uint32_t>(a.parity_sp) : 0u) + col * 16u;
  return f;
}

// ---------------------------------------------------------------------------
// Bitsliced encode over 1 KiB-wide tasks (64 columns, 16 B of every shard per lane).
//
// Bitslicing needs 32 B per lane to fill 8 plane dwords; round 1-3's 2 KiB-row kernel
// gave each lane two columns, and that task shape streams about 3 points below 1 KiB
// rows at RS(8+4) (compute-free probe).  Here a lane fills its planes from two INPUTS
// instead: 16 B of input c (even) in dwords
// 0-3 and of input c ^ 1 in dwords 4-7, so after transpose8 plane j holds bit j of
// input c in the low nibble of each byte and of input c ^ 1 in the high nibble.
// The RS(8+4) and RS(10+4) encode matrices satisfy C[r ^ 1][c] = C[r][c ^ 1], so for
// an even row r, A = C[r][c], B = C[r][c ^ 1]: A * P + B * nibswap(P) is row r of the
// pair in the low nibbles and row r ^ 1 in the high nibbles.  The generated pair
// program accumulates A * P (ya) and B * P (yb); nibswap is linear, so one
// ya ^ nibswap(yb) per output plane and one transpose8 per packed row give 16 B of
// rows r and r ^ 1 (dwords 0-3 and 4-7).  XORs per 32 B of every shard: RS(8+4) 532
// (pair programs share the A / B terms) vs 564; the transposes: K / 2 + M / 2 per 16 B,
// the same count per byte as the 2 KiB kernel, plus 4 VALU ops per packed plane.
// Flat column space: the batch's columns, each stripe rounded up to whole 128-B lines
// (a straddling wave access then splits at a line boundary), cut into 64-column tasks
// that may straddle two stripes, so no lane idles at a stripe's ragged end (RS(10+4)
// at 64 KiB objects: 6.5 tasks per stripe instead of 7).  Addresses: one buffer
// descriptor per region off the task's first stripe, a per-lane 32-bit offset (next
// stripe: + its pitch) and the slot as the scalar offset.  Host preconditions
// (launch_window): cols >= 128, data_sp / parity_sp + 16 * cols < 2^31.
// Full columns store 16 B; the lane holding a stripe's partial last column stores it
// byte-exact in a wave-uniform branch taken by tasks that contain one.
// Interleaved A/B against the 2 KiB kernel (round 4, profiles/r04zb_ab_bs16.log, 64 KiB
// objects, >= 100 ms per point, 3 rounds): RS(8+4) 69.4-70.4 -> 72.0-73.1 % of 8 TB/s,
// RS(10+4) 66.6-67.6 -> 67.5-68.2 %; a window of 3 pairs and 8 workgroups per CU level.
#ifndef RS_BS16_WINDOW
#define RS_BS16_WINDOW 5
#endif
#ifndef RS_BS16_OCC
#define RS_BS16_OCC 3
#endif
constexpr int kBs16Window = RS_BS16_WINDOW;  // input pairs with loads in flight

template <int K, int M, int P>
__device__ __forceinline__ void bs16_fold(__amdgpu_buffer_rsrc_t din, uint32_t pitch, uint32_t off,
                                          u32x4 (&xa)[kBs16Window], u32x4 (&xb)[kBs16Window],
                                          uint32_t (&ya)[4 * M], uint32_t (&yb)[4 * M]) {
  if constexpr (P < K / 2) {
    constexpr int slot = P % kBs16Window;
    uint32_t d[8] = {xa[slot][0], xa[slot][1], xa[slot][2], xa[slot][3],
                     xb[slot][0], xb[slot][1], xb[slot][2], xb[slot][3]};
    if constexpr (P + kBs16Window < K / 2) {
      xa[slot] = bload16(din, off, (2 * (P + kBs16Window)) * pitch);
      xb[slot] = bload16(din, off, (2 * (P + kBs16Window) + 1) * pitch);
    }
    if constexpr (RS_PATTERN_ONLY) {
#pragma unroll
      for (int i = 0; i < 4 * M; ++i) {
        ya[i] = (P == 0 ? 0u : ya[i]) ^ d[i & 7];
        yb[i] = (P == 0 ? 0u : yb[i]) ^ d[(i + 3) & 7];
      }
    } else {
      transpose8(d);
      bs16_step<K, M, P>(d, ya, yb);
    }
    bs16_fold<K, M, P + 1>(din, pitch, off, xa, xb, ya, yb);
  }
}

template <int K, int M>
__global__ __launch_bounds__(256, RS_BS16_OCC) void encode_bs16_kernel(const KernelArgs a) {
  static_assert(K % 2 == 0 && M % 2 == 0, "pair programs need even K and M");
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wave = wave_index();
  const uint32_t nwaves = gridDim.x * (blockDim.x >> 6);
  const uint32_t cols = (a.shard_len + 15u) >> 4;
  const uint32_t nb = a.shard_len & 15u;  // bytes of a partial last column (0: none)
  const uint32_t cstride = (cols + 7u) & ~7u;
  const uint64_t total = static_cast<uint64_t>(a.n_stripes) * cstride;
  if (static_cast<uint64_t>(wave) * 64u >= total) return;
  const uint32_t pitch = static_cast<uint32_t>(a.shard_pitch);
  const uint64_t g0 = static_cast<uint64_t>(wave) * 64u;
  uint32_t s0 = wave_uniform(static_cast<uint32_t>(g0 / cstride));
  uint32_t c0 = static_cast<uint32_t>(g0 - static_cast<uint64_t>(s0) * cstride);
  const uint64_t gstep = static_cast<uint64_t>(nwaves) * 64u;
  const uint32_t step_s = wave_uniform(static_cast<uint32_t>(gstep / cstride));
  const uint32_t step_c = static_cast<uint32_t>(gstep - static_cast<uint64_t>(step_s) * cstride);
  while (s0 < a.n_stripes) {
    const FlatCol f = flat_col(a, s0, c0 + lane, cstride, cols);
    const auto din = __builtin_amdgcn_make_buffer_rsrc(a.data + static_cast<uint64_t>(s0) * a.data_sp, 0,
                                                       0x7FFFFFFF, 0x00020000);
    const auto pout = __builtin_amdgcn_make_buffer_rsrc(a.parity + static_cast<uint64_t>(s0) * a.parity_sp, 0,
                                                        0x7FFFFFFF, 0x00020000);
    u32x4 xa[kBs16Window], xb[kBs16Window];
#pragma unroll
    for (int p = 0; p < kBs16Window && p < K / 2; ++p) {
      xa[p] = bload16(din, f.doff, (2 * p) * pitch);
      xb[p] = bload16(din, f.doff, (2 * p + 1) * pitch);
    }
    uint32_t ya[4 * M], yb[4 * M];
    bs16_fold<K, M, 0>(din, pitch, f.doff, xa, xb, ya, yb);
    const bool sf = f.live && f.col < a.full_cols;
    const bool pf = nb != 0u && f.live && f.col == a.full_cols;  // this lane holds a partial column
    u32x4 part[M];
#pragma unroll
    for (int q = 0; q < M / 2; ++q) {
      uint32_t d[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const uint32_t b = yb[q * 8 + i];
        d[i] = ya[q * 8 + i] ^ ((b >> 4) & 0x0F0F0F0Fu) ^ ((b << 4) & 0xF0F0F0F0u);
      }
      if constexpr (!RS_PATTERN_ONLY) transpose8(d);
      const u32x4 lo{d[0], d[1], d[2], d[3]}, hi{d[4], d[5], d[6], d[7]};
      __builtin_amdgcn_raw_buffer_store_b128(lo, pout, sf ? f.poff : kDropOffset, (2 * q) * pitch, 2 /* nt */);
      __builtin_amdgcn_raw_buffer_store_b128(hi, pout, sf ? f.poff : kDropOffset, (2 * q + 1) * pitch, 2 /* nt */);
      part[2 * q] = lo;
      part[2 * q + 1] = hi;
    }
    if (nb != 0u && __builtin_amdgcn_ballot_w64(pf) != 0u) {  // wave-uniform
#pragma unroll
      for (int r = 0; r < M; ++r) store_part_rsrc(pout, f.poff, r * pitch, pf, part[r], nb);
    }
    c0 += step_c;
    s0 += step_s;
    if (c0 >= cstride) {
      c0 -= cstride;
      ++s0;
    }
  }
}

// ---------------------------------------------------------------------------
// Per-stripe out-of-place reconstruct over flat 64-column tasks (LUT plans),
// segmented (round 5).
//
// For ragged shard lengths (columns not a multiple of 64, e.g. RS(10+4) at 64 KiB
// objects: S = 6 554, 410 columns) the batch's columns -- each stripe rounded up to
// whole 128-B lines, so a wave access splits only at a line boundary -- are cut into
// 64-column tasks that may straddle two stripes: 6.5 tasks per RS(10+4) stripe
// instead of 7 stripe-aligned ones.  A task whose two stripes have different
// erasure patterns runs as two passes of the single-plan code: the lanes of stripe
// s0 with plan A, then the lanes of stripe s0 + 1 with plan B, the other stripe's
// lanes loading nothing (out-of-range offsets: no fetch) and storing nothing.  The
// kernel so holds one plan's working set (RS(10+4): 58 / 65 / 164 VGPRs for E = 1 /
// 2 / 4); round 2's form selected table dwords per lane between the two plans
// (141 / 129 / 195 VGPRs).  The price is a second pass of VALU work on the one task
// in 13 that straddles two stripes.  A pass over an intact (or skipped) stripe is
// not run at all.  E is the launch's erasure bound: M for device masks without a
// bound and for mixed coalescer batches, the masks' maximum for host masks, the
// caller's max_missing for device masks.  E <= 2 runs input-outer with x[K] as the
// only per-input state; E > 2 splits every input into chunk indices once and then
// computes only the rows the stripe misses, one at a time.
// The E > 2 flat launches take one task per wave (a full grid) like the E <= 2 ones,
// instead of a grid-stride loop over default_blocks_per_cu.
// Out-of-place per-stripe launches whose shard length is a whole number of 64-column
// tasks (no task then straddles) take the flat kernel too for RS(10+4) with a bound
// of 2 or more: same-process A/B at 80 KiB objects (profiles/r05k_ab_flatal.log, S =
// 8 192, 4 rounds) bounded 2-erasure 68.0 -> 76.4 %, unbounded 2-erasure +0.8, mixed
// 70.0 -> 73.0 %; 1-erasure -0.3, and every other shape loses (RS(8+4) 2-erasure
// -1.9 / -5.5, RS(4+2) -4.9 to -7.2, RS(6+3) -1.0) except RS(8+4) mixed (+1.7).
// (Rejected: one-pattern out-of-place reconstructs through this kernel with one plan
// for every stripe; the stripe-aligned uniform kernel, whose slots are resolved once
// per launch, stays ahead, profiles/r05m_ab_uniform.log: RS(10+4) 2-erasure at 64 /
// 80 KiB objects -3.5 / -3.8 points through the flat kernel.)

template <int K, int M, int E>
__global__ __launch_bounds__(256) void apply_flat_seg_kernel(const KernelArgs a) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wave = wave_index();
  const uint32_t nwaves = gridDim.x * (blockDim.x >> 6);
  const uint32_t N = a.n_stripes;
  const uint32_t cols = (a.shard_len + 15u) >> 4;
  const uint32_t nb = a.shard_len & 15u;  // bytes of a partial last column (0: none)
  const uint32_t cstride = (cols + 7u) & ~7u;
  if (static_cast<uint64_t>(wave) * 64u >= static_cast<uint64_t>(N) * cstride) return;
  const uint32_t pitch = static_cast<uint32_t>(a.shard_pitch);
  const uint32_t full = a.full_mask;
  const uint64_t g0 = static_cast<uint64_t>(wave) * 64u;
  uint32_t s0 = wave_uniform(static_cast<uint32_t>(g0 / cstride));
  uint32_t c0 = static_cast<uint32_t>(g0 - static_cast<uint64_t>(s0) * cstride);
  const uint64_t gstep = static_cast<uint64_t>(nwaves) * 64u;
  const uint32_t step_s = wave_uniform(static_cast<uint32_t>(gstep / cstride));
  const uint32_t step_c = static_cast<uint32_t>(gstep - static_cast<uint64_t>(step_s) * cstride);
  uint32_t bad = 0u;

  // stripe s's present mask (a skipped one: all present) and plan; a uniform launch
  // (no masks: one erasure pattern for the batch) has the one plan for every stripe
  const bool uni = a.present_masks == nullptr;
  auto plan_of = [&](uint32_t s, uint32_t& m, uint32_t& nout) -> const uint8_t* {
    if (E > 2 && !uni) {
      // an intact stripe (a scan's common case; launches sized for m outputs are the
      // scans'): nothing to do, decided from the mask alone -- no LUT and plan round
      // trips before the wave can leave (round 6, profiles/r06c_ab_fast.log: RS(10+4)
      // 64 KiB mixed 0..4 erasures +0.7 points)
      const uint32_t present = as_const<uint32_t>(a.present_masks)[s] & full;
      if (present == full) {
        m = full;
        nout = 0u;
        return uniform_ptr(a.plans);
      }
    }
    if (uni) {
      const uint8_t* p = uniform_ptr(a.plans);
      const PlanView pv(p, K, M);
      m = pv.present() & full;
      nout = pv.n_out();
      return p;
    }
    const uint32_t present = as_const<uint32_t>(a.present_masks)[s] & full;
    uint32_t pid = as_const<uint32_t>(a.lut)[(~present) & full];
    bad |= (pid == kPlanInvalid) ? 1u : 0u;
    bool skip = pid == kPlanInvalid;
    if constexpr (E < M) {  // more erasures than this launch's bound: skip, flag
      const bool over = static_cast<uint32_t>(__builtin_popcount((~present) & full)) > static_cast<uint32_t>(E);
      bad |= over ? 2u : 0u;
      skip = skip || over;
    }
    m = skip ? full : present;
    pid = skip ? 0u : pid;  // plan 0 = nothing missing
    const uint8_t* p = uniform_ptr(a.plans + static_cast<uint64_t>(pid) * a.plan_bytes);
    nout = PlanView(p, K, M).n_out();
    return p;
  };

  while (s0 < N) {
    const uint32_t cl = c0 + lane;
    const bool inB = cl >= cstride;
    const uint32_t colr = inB ? cl - cstride : cl;
    const bool straddle = c0 + 63u >= cstride && s0 + 1u < N;  // wave-uniform
    const bool live = !inB || straddle;                         // past the batch end: dead
    const uint32_t col = live ? min(colr, cols - 1u) : 0u;      // clamped load column
    uint32_t mA, nA, mB, nB;
    const uint8_t* planA = plan_of(s0, mA, nA);
    const uint8_t* planB = planA;
    mB = mA;
    nB = nA;
    if (straddle) planB = plan_of(s0 + 1u, mB, nB);
    const bool two = planA != planB;  // wave-uniform: two passes, one per stripe
    const bool lb = live && inB;      // B lanes are addressed off stripe s0's base
    const uint32_t offD = (lb ? static_cast<uint32_t>(a.data_sp) : 0u) + col * 16u;
    const uint32_t offP = (lb ? static_cast<uint32_t>(a.parity_sp) : 0u) + col * 16u;
    // out of place: the r-th missing shard of the lane's stripe at out + s*out_sp + r*P,
    // or packed at out + (row_offsets[s] + r)*P
    uint64_t obase = static_cast<uint64_t>(s0) * a.out_sp;
    uint32_t osp = static_cast<uint32_t>(a.out_sp);
    if (a.row_offsets) {  // wave-uniform
      const uint32_t r0 = as_const<uint32_t>(a.row_offsets)[s0];
      obase = static_cast<uint64_t>(r0) * pitch;
      osp = straddle ? (as_const<uint32_t>(a.row_offsets)[s0 + 1u] - r0) * pitch : 0u;
    }
    const uint32_t offO = (lb ? osp : 0u) + col * 16u;
    const bool fullc = live && colr < a.full_cols;
    const bool part = nb != 0u && live && colr == a.full_cols;
    const auto din = __builtin_amdgcn_make_buffer_rsrc(a.data + static_cast<uint64_t>(s0) * a.data_sp, 0,
                                                       0x7FFFFFFF, 0x00020000);
    const auto pin = __builtin_amdgcn_make_buffer_rsrc(a.parity + static_cast<uint64_t>(s0) * a.parity_sp, 0,
                                                       0x7FFFFFFF, 0x00020000);
    const auto oout = __builtin_amdgcn_make_buffer_rsrc(a.out + obase, 0, 0x7FFFFFFF, 0x00020000);
    for (uint32_t seg = 0; seg < (two ? 2u : 1u); ++seg) {
      const bool sb = seg != 0u;
      const uint8_t* plan = sb ? planB : planA;
      uint32_t bits = sb ? mB : mA;
      const uint32_t nout = sb ? nB : nA;  // wave-uniform
      if (nout == 0u) continue;           // an intact (or skipped) stripe: no loads, no stores
      const bool mine = !two || inB == sb;
      const uint32_t oD = mine ? offD : kDropOffset, oP = mine ? offP : kDropOffset;
      u32x4 x[K];
#pragma unroll
      for (int c = 0; c < K; ++c) {
        const uint32_t s = pop_low(bits);
        x[c] = s < static_cast<uint32_t>(K) ? bload16(din, oD, s * pitch)
                                            : bload16(pin, oP, (s - static_cast<uint32_t>(K)) * pitch);
      }
      const uint32_t nl = mine ? nout : 0u;
      const uint32_t miss = ~(sb ? mB : mA) & full;  // in place: the rows' own slots
      // stores rows [0, NR) with cache policy CPOL, dropped per lane past its stripe's outputs
      auto emit = [&](auto nr_tag, auto cpol_tag, const auto& yy) {
        constexpr int NR = decltype(nr_tag)::value;
        constexpr int CPOL = decltype(cpol_tag)::value;
        if (!a.out) {
          // in place (round 6): row r into the stripe's r-th missing slot, through the
          // inputs' own descriptors (RS(10+4) 80 KiB objects, per-stripe device masks,
          // +3.9 points over the stripe-aligned kernel; at 64 KiB, where tasks straddle
          // stripes, -0.9, so ragged in-place batches stay stripe-aligned,
          // profiles/r06ac_ab_inplace.log)
          uint32_t mb = miss;
          const bool anyp = __builtin_amdgcn_ballot_w64(part) != 0u;
#pragma unroll
          for (int r = 0; r < NR; ++r) {
            const uint32_t sl = pop_low(mb);
            const bool isd = sl < static_cast<uint32_t>(K);
            const uint32_t so = (isd ? sl : sl - static_cast<uint32_t>(K)) * pitch;
            const uint32_t vo = isd ? oD : oP;
            __builtin_amdgcn_raw_buffer_store_b128(yy[r], isd ? din : pin,
                                                   fullc && static_cast<uint32_t>(r) < nl ? vo : kDropOffset, so,
                                                   CPOL);
            if (anyp) store_part_rsrc<CPOL>(isd ? din : pin, vo, so, part && static_cast<uint32_t>(r) < nl, yy[r], nb);
          }
          return;
        }
#pragma unroll
        for (int r = 0; r < NR; ++r)
          __builtin_amdgcn_raw_buffer_store_b128(yy[r], oout,
                                                 fullc && static_cast<uint32_t>(r) < nl ? offO : kDropOffset,
                                                 r * pitch, CPOL);
        if (__builtin_amdgcn_ballot_w64(part) != 0u) {  // wave-uniform
#pragma unroll
          for (int r = 0; r < NR; ++r)
            store_part_rsrc<CPOL>(oout, offO, r * pitch, part && static_cast<uint32_t>(r) < nl, yy[r], nb);
        }
      };
      if constexpr (E <= 2) {
        u32x4 y[E];
        gf_rows<K, M, 0, E>(plan, x, y);
        emit(std::integral_constant<int, E>{}, std::integral_constant<int, out_cpol<K, E>()>{}, y);
      } else {
        // E > 2 (device masks without a bound, mixed batches): input-outer over only the
        // rows the stripe misses, one specialisation per row count, in wave-uniform
        // branches (round 6, profiles/r06r_ab_inout.log, same process under one-wave
        // workgroups: RS(10+4) 64 KiB mixed 0..4 +1.8, 4-erasure +2.2, unbounded
        // 2-erasure +1.9, 1-erasure -0.5, 80 KiB mixed +1.8 points against round 5's
        // chunk-index array computed once and read per row -- 144 VGPRs instead of 165;
        // forced down to 4 waves per SIMD (128 VGPRs, scratch spills) it lost 10).
        // (Rejected, round 6: the tasks scattered over the waves so a CU holds many
        // stripes' erasure counts at once -- -5 to -12, profiles/r06b_ab_perm.log; the
        // survivors of a task 512-4096 tasks ahead fetched into L2 by LDS-DMA loads
        // while the own inputs load, -15 to -22, profiles/r06h_ab_prefetch.log.)
        if (nout <= 1u) {
          u32x4 y[1];
          gf_rows<K, M, 0, 1>(plan, x, y);
          emit(std::integral_constant<int, 1>{}, std::integral_constant<int, kCpolFlatPath1>{}, y);
        } else if (nout == 2u) {
          u32x4 y[2];
          gf_rows<K, M, 0, 2>(plan, x, y);
          emit(std::integral_constant<int, 2>{}, std::integral_constant<int, path_cpol<K, E, 2>()>{}, y);
        } else if (E < 4 || nout == 3u) {
          u32x4 y[3];
          gf_rows<K, M, 0, 3>(plan, x, y);
          emit(std::integral_constant<int, 3>{}, std::integral_constant<int, out_cpol<K, E>()>{}, y);
        } else if constexpr (E >= 4) {
          u32x4 y[4];
          gf_rows<K, M, 0, 4>(plan, x, y);
          emit(std::integral_constant<int, 4>{}, std::integral_constant<int, out_cpol<K, E>()>{}, y);
        }
      }
    }
    c0 += step_c;  // grid stride in the flat column space
    s0 += step_s;
    if (c0 >= cstride) {
      c0 -= cstride;
      ++s0;
    }
  }
  if (bad && lane == 0u) atomicOr(a.status, bad);
}

// ---------------------------------------------------------------------------
// Per-stripe plans over a table of shard addresses (round 3): the coalescer's
// batches whose objects lie in the caller's registered (pinned, GPU-mapped) buffers
// are read and written in place -- no staging copy of the request body, no copy of
// the parity back.  A slot staged as usual simply points
// into the staging.  Every shard is its own buffer of exactly S bytes, so each is
// addressed through a buffer descriptor whose range ends with the shard: loads stop
// at the dword holding byte S-1 (out-of-range dwords are not fetched and read as
// zero), stores at byte S-1 (the partial last column in byte-exact pieces).
// Stripe-aligned 64-column tasks: per-object shards are large (the objects that
// gain from skipping the copy), so the idle lanes of a stripe's last task are few.
template <int K, int M, int E>
__global__ __launch_bounds__(256) void apply_ptr_kernel(const KernelArgs a) {
  constexpr int T = K + M;
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wave = wave_index();
  const uint32_t nwaves = gridDim.x * (blockDim.x >> 6);
  const uint32_t bps = a.blocks_per_stripe;
  const uint32_t ntasks = a.n_stripes * bps;  // host guarantees < 2^32
  const uint32_t S = a.shard_len;
  const uint32_t cols = (S + 15u) >> 4;
  const uint32_t nb = S & 15u;
  const uint32_t in_range = (S + 3u) & ~3u;  // whole dwords: the last one holds byte S-1
  const uint32_t full = a.full_mask;
  uint32_t bad = 0u;
  for (uint32_t t = wave; t < ntasks; t += nwaves) {
    const uint32_t stripe = t / bps;
    const uint32_t blk = t - stripe * bps;
    const uint32_t present = as_const<uint32_t>(a.present_masks)[stripe] & full;
    uint32_t pid = as_const<uint32_t>(a.lut)[(~present) & full];
    bool skip = pid == kPlanInvalid;
    bad |= skip ? 1u : 0u;
    if constexpr (E < M) {  // more erasures than this launch's bound: skip, flag
      const bool over = static_cast<uint32_t>(__builtin_popcount((~present) & full)) > static_cast<uint32_t>(E);
      bad |= over ? 2u : 0u;
      skip = skip || over;
    }
    pid = skip ? 0u : pid;  // plan 0 = nothing missing: every store dropped
    const uint8_t* plan = uniform_ptr(a.plans + static_cast<uint64_t>(pid) * a.plan_bytes);
    if constexpr (K * E * 5 > 48) asm volatile("" : "+s"(plan));  // tables per trip (as apply_kernel)
    const PlanView pv(plan, K, M);
    const uint64_t* sp = as_const<uint64_t>(a.shard_ptrs) + static_cast<uint64_t>(stripe) * T;
    const uint32_t col = blk * 64u + lane;
    const uint32_t off = (col < cols ? col : cols - 1u) * 16u;  // past the end: re-read the last column
    u32x4 x[K];
#pragma unroll
    for (int c = 0; c < K; ++c) {
      const uint32_t s = skip ? static_cast<uint32_t>(c) : pv.in_idx(c);
      uint8_t* base = reinterpret_cast<uint8_t*>(as_const<uint64_t>(sp)[s]);
      const auto r = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(uniform_ptr(base)), 0, in_range,
                                                       0x00020000);
      x[c] = bload16(r, off, 0);
    }
    u32x4 y[E];
    const uint32_t n_out = pv.n_out();
    if constexpr (E > 2) {
      Idx3 ix[K][4];
#pragma unroll
      for (int c = 0; c < K; ++c)
#pragma unroll
        for (int d = 0; d < 4; ++d) ix[c][d] = split3(x[c][d]);
      y[0] = gf_row_ix<K, M>(plan, ix, 0);
#pragma unroll
      for (int r = 1; r < E; ++r) {
        y[r] = y[0];  // dropped unless computed
        if (static_cast<uint32_t>(r) < n_out) y[r] = gf_row_ix<K, M>(plan, ix, r);
      }
    } else {
      gf_rows<K, M, 0, E>(plan, x, y);
    }
    const bool fullc = col < a.full_cols;
    const bool part = nb != 0u && col == a.full_cols;
    const bool last = nb != 0u && blk + 1u == bps;  // wave-uniform: the task holds the partial column
#pragma unroll
    for (int r = 0; r < E; ++r) {
      const bool row = static_cast<uint32_t>(r) < n_out;
      uint8_t* base = reinterpret_cast<uint8_t*>(as_const<uint64_t>(sp)[row ? pv.out_idx(r) : 0u]);
      const auto ro = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(uniform_ptr(base)), 0, S, 0x00020000);
      __builtin_amdgcn_raw_buffer_store_b128(y[r], ro, fullc && row ? off : kDropOffset, 0, out_cpol<K, E>());
      if (last) store_part_rsrc<out_cpol<K, E>()>(ro, off, 0, part && row, y[r], nb);
    }
  }
  if (bad && lane == 0u) atomicOr(a.status, bad);
}

// ---------------------------------------------------------------------------
// Verify / scrub ([upstream reedsolomon.go Verify]: re-encode and compare; the
// reference lists bit-rot detection as missing, docs/ARCHITECTURE.md:175-178).
// Same lookup arithmetic as apply_kernel, but the M stored parity columns are
// loaded next to the K data columns and nothing is stored: a task ends in one
// compare per parity row, and only a mismatching lane issues an atomic.  All
// columns, the partial last one included, run here: a byte mask limits the
// compare to the shard's S bytes (16-B loads stay inside the shard slot).
__device__ __forceinline__ uint32_t byte_mask(uint32_t nbytes, int d) {
  const int v = static_cast<int>(nbytes) - 4 * d;  // valid bytes of dword d
  return v >= 4 ? 0xFFFFFFFFu : (v <= 0 ? 0u : (1u << (8 * v)) - 1u);
}

template <int K, int M>
__global__ __launch_bounds__(256) void verify_kernel(const KernelArgs a) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wave = wave_index();
  const uint32_t nwaves = gridDim.x * (blockDim.x >> 6);
  const uint32_t bps = a.blocks_per_stripe;
  const uint32_t ntasks = a.n_stripes * bps;
  const uint8_t* const plan0 = uniform_ptr(a.plans);
  for (uint32_t t = wave; t < ntasks; t += nwaves) {
    const uint32_t stripe = t / bps;
    const uint32_t blk = t - stripe * bps;
    const uint8_t* plan = plan0;
    uint64_t pitch = a.shard_pitch;
    if constexpr (K * M * 5 > 48) {
      // opaque per trip (see apply_kernel): neither the tables nor the K+M slot
      // offsets c*pitch may be hoisted into SGPRs for the whole loop
      asm volatile("" : "+s"(plan));
      asm volatile("" : "+s"(pitch));
    }
    const PlanView pv(plan, K, M);
    const uint32_t col = blk * 64u + lane;
    const uint32_t start = col * 16u;
    const uint32_t nbytes = start < a.shard_len ? min(16u, a.shard_len - start) : 0u;
    const uint32_t off = nbytes ? start : 0u;
    const uint8_t* dbase = a.data + static_cast<uint64_t>(stripe) * a.data_sp + off;
    const uint8_t* pbase = a.parity + static_cast<uint64_t>(stripe) * a.parity_sp + off;
    u32x4 x[K], st[M];
#pragma unroll
    for (int c = 0; c < K; ++c) x[c] = load16(dbase + static_cast<uint64_t>(c) * pitch);
#pragma unroll
    for (int r = 0; r < M; ++r) st[r] = load16(pbase + static_cast<uint64_t>(r) * pitch);
    u32x4 y[M], pend[M];
#pragma unroll
    for (int r = 0; r < M; ++r) y[r] = st[r];  // y = stored ^ recomputed: zero when intact
#pragma unroll
    for (int c = 0; c < K; ++c) {
      Idx3 ix[4];
#pragma unroll
      for (int d = 0; d < 4; ++d) ix[d] = split3(x[c][d]);
      // one opaque base per input: the scalar load merger cannot fuse this
      // input's table loads with later inputs' (which would pin them in SGPRs)
      const uint8_t* tcol = plan;
      if constexpr (K * M * 5 > 48) asm volatile("" : "+s"(tcol));
      const PlanView pc(tcol, K, M);
#pragma unroll
      for (int r = 0; r < M; ++r) {
        const RS_CONST uint32_t* tb = pc.quad(r, c);
        const uint32_t q0 = tb[0], q1 = tb[1], q2 = tb[2], q3 = tb[3], q4 = pc.c4(r, c);
#pragma unroll
        for (int d = 0; d < 4; ++d) {
          const uint32_t prod = lookup3(ix[d], q0, q1, q2, q3, q4);
          if (c & 1)
            y[r][d] = xor3(y[r][d], pend[r][d], prod);
          else if (c == K - 1)
            y[r][d] ^= prod;
          else
            pend[r][d] = prod;
        }
      }
      if (c + 1 < K) __builtin_amdgcn_sched_barrier(0);
    }
    uint32_t bits = 0u;
#pragma unroll
    for (int r = 0; r < M; ++r) {
      uint32_t diff = 0u;
#pragma unroll
      for (int d = 0; d < 4; ++d) diff |= y[r][d] & byte_mask(nbytes, d);
      bits |= diff ? (1u << r) : 0u;
    }
    if (bits) atomicOr(a.bad + stripe, bits);
  }
}

// The same check over flat 64-column tasks (each stripe rounded up to whole 128-B
// lines, a task may straddle two stripes; see encode_bs16_kernel): RS(10+4)
// at 64 KiB objects runs 6.5 tasks per stripe instead of 7 stripe-aligned ones.
// Host preconditions as for the flat encode (cols >= 64 here).
template <int K, int M>
__global__ __launch_bounds__(256) void verify_flat_kernel(const KernelArgs a) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wave = wave_index();
  const uint32_t nwaves = gridDim.x * (blockDim.x >> 6);
  const uint32_t cols = (a.shard_len + 15u) >> 4;
  const uint32_t cstride = (cols + 7u) & ~7u;
  const uint64_t total = static_cast<uint64_t>(a.n_stripes) * cstride;
  if (static_cast<uint64_t>(wave) * 64u >= total) return;
  const uint32_t pitch0 = static_cast<uint32_t>(a.shard_pitch);
  const uint64_t g0 = static_cast<uint64_t>(wave) * 64u;
  uint32_t s0 = wave_uniform(static_cast<uint32_t>(g0 / cstride));
  uint32_t c0 = static_cast<uint32_t>(g0 - static_cast<uint64_t>(s0) * cstride);
  const uint64_t gstep = static_cast<uint64_t>(nwaves) * 64u;
  const uint32_t step_s = wave_uniform(static_cast<uint32_t>(gstep / cstride));
  const uint32_t step_c = static_cast<uint32_t>(gstep - static_cast<uint64_t>(step_s) * cstride);
  const uint8_t* const plan0 = uniform_ptr(a.plans);
  while (s0 < a.n_stripes) {
    const uint8_t* plan = plan0;
    uint32_t pitch = pitch0;
    if constexpr (K * M * 5 > 48) {
      // opaque per trip, as in verify_kernel
      asm volatile("" : "+s"(plan));
      asm volatile("" : "+s"(pitch));
    }
    const FlatCol f = flat_col(a, s0, c0 + lane, cstride, cols);
    const uint32_t start = f.col * 16u;
    const uint32_t nbytes = f.live && start < a.shard_len ? min(16u, a.shard_len - start) : 0u;
    const auto din = __builtin_amdgcn_make_buffer_rsrc(a.data + static_cast<uint64_t>(s0) * a.data_sp, 0,
                                                       0x7FFFFFFF, 0x00020000);
    const auto pin = __builtin_amdgcn_make_buffer_rsrc(a.parity + static_cast<uint64_t>(s0) * a.parity_sp, 0,
                                                       0x7FFFFFFF, 0x00020000);
    u32x4 x[K], st[M];
#pragma unroll
    for (int c = 0; c < K; ++c) x[c] = bload16(din, f.doff, c * pitch);
#pragma unroll
    for (int r = 0; r < M; ++r) st[r] = bload16(pin, f.poff, r * pitch);
    u32x4 y[M], pend[M];
#pragma unroll
    for (int r = 0; r < M; ++r) y[r] = st[r];  // y = stored ^ recomputed: zero when intact
#pragma unroll
    for (int c = 0; c < K; ++c) {
      Idx3 ix[4];
#pragma unroll
      for (int d = 0; d < 4; ++d) ix[d] = split3(x[c][d]);
      // one opaque base per input: the scalar load merger cannot fuse this
      // input's table loads with later inputs' (which would pin them in SGPRs)
      const uint8_t* tcol = plan;
      if constexpr (K * M * 5 > 48) asm volatile("" : "+s"(tcol));
      const PlanView pc(tcol, K, M);
#pragma unroll
      for (int r = 0; r < M; ++r) {
        const RS_CONST uint32_t* tb = pc.quad(r, c);
        const uint32_t q0 = tb[0], q1 = tb[1], q2 = tb[2], q3 = tb[3], q4 = pc.c4(r, c);
#pragma unroll
        for (int d = 0; d < 4; ++d) {
          const uint32_t prod = lookup3(ix[d], q0, q1, q2, q3, q4);
          if (c & 1)
            y[r][d] = xor3(y[r][d], pend[r][d], prod);
          else if (c == K - 1)
            y[r][d] ^= prod;
          else
            pend[r][d] = prod;
        }
      }
      if (c + 1 < K) __builtin_amdgcn_sched_barrier(0);
    }
    uint32_t bits = 0u;
#pragma unroll
    for (int r = 0; r < M; ++r) {
      uint32_t diff = 0u;
#pragma unroll
      for (int d = 0; d < 4; ++d) diff |= y[r][d] & byte_mask(nbytes, d);
      bits |= diff ? (1u << r) : 0u;
    }
    if (bits) atomicOr(a.bad + s0 + (c0 + lane >= cstride ? 1u : 0u), bits);
    c0 += step_c;
    s0 += step_s;
    if (c0 >= cstride) {
      c0 -= cstride;
      ++s0;
    }
  }
}

// Runtime K/M variant (shapes without a specialisation).
__global__ __launch_bounds__(256) void verify_kernel_generic(const KernelArgs a) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wave = wave_index();
  const uint32_t nwaves = gridDim.x * (blockDim.x >> 6);
  const uint32_t bps = a.blocks_per_stripe;
  const uint32_t ntasks = a.n_stripes * bps;
  const int K = a.k, M = a.m;
  const PlanView pv(a.plans, K, M);
  for (uint32_t t = wave; t < ntasks; t += nwaves) {
    const uint32_t stripe = t / bps;
    const uint32_t blk = t - stripe * bps;
    const uint32_t start = (blk * 64u + lane) * 16u;
    if (start >= a.shard_len) continue;
    const uint32_t nbytes = min(16u, a.shard_len - start);
    const uint8_t* dbase = a.data + static_cast<uint64_t>(stripe) * a.data_sp + start;
    const uint8_t* pbase = a.parity + static_cast<uint64_t>(stripe) * a.parity_sp + start;
    uint32_t bits = 0u;
    for (int r = 0; r < M; ++r) {
      u32x4 y = load16(pbase + static_cast<uint64_t>(r) * a.shard_pitch);
      for (int c = 0; c < K; ++c) {
        const u32x4 x = load16(dbase + static_cast<uint64_t>(c) * a.shard_pitch);
        const RS_CONST uint32_t* tb = pv.quad(r, c);
        const uint32_t q0 = tb[0], q1 = tb[1], q2 = tb[2], q3 = tb[3], q4 = pv.c4(r, c);
#pragma unroll
        for (int d = 0; d < 4; ++d) y[d] ^= lookup3(split3(x[d]), q0, q1, q2, q3, q4);
      }
      uint32_t diff = 0u;
#pragma unroll
      for (int d = 0; d < 4; ++d) diff |= y[d] & byte_mask(nbytes, d);
      bits |= diff ? (1u << r) : 0u;
    }
    if (bits) atomicOr(a.bad + stripe, bits);
  }
}

// ---------------------------------------------------------------------------
// Streaming copy (bench only): the measured HBM ceiling next to the RS kernels.
// Wave-contiguous 4 KiB tasks (4 x 16-B loads per lane, 1 KiB per wave instruction),
// non-temporal loads, stores NT + device-scope write-through, one workgroup per CU:
// the fastest of tools/copy_probe.hip's sweep at the RS bench's traffic per launch
// (402 MB over rotating buffers: 6.41 TB/s read+write, profiles/r04c_copy_probe.log;
// the round-1..3 block-contiguous form 6.0-6.2).  Each task's descriptor starts at
// the task and ends with the buffer, so the tail needs no branch and any size works.
__global__ __launch_bounds__(256) void copy_kernel(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                   uint64_t bytes) {
  constexpr uint32_t kTask = 4096;
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t nw = static_cast<uint64_t>(gridDim.x) * (blockDim.x >> 6);
  for (uint64_t t = wave_index(); t * kTask < bytes; t += nw) {
    const uint64_t base = t * kTask;
    const uint64_t left = bytes - base;
    const uint32_t nrec = static_cast<uint32_t>(left < kTask ? left : kTask);
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(src) + base, 0, nrec, 0x00020000);
    const auto rd = __builtin_amdgcn_make_buffer_rsrc(dst + base, 0, nrec, 0x00020000);
    u32x4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = bload16(rs, lane * 16u + u * 1024u, 0);
#pragma unroll
    for (int u = 0; u < 4; ++u)
      __builtin_amdgcn_raw_buffer_store_b128(v[u], rd, lane * 16u + u * 1024u, 0, kCpolNt | kCpolSc1);
  }
}

// ---------------------------------------------------------------------------
// Host-side launch dispatch.
template <int K, int M, int E>
static const void* spec_fn(bool per_stripe) {
  return per_stripe ? reinterpret_cast<const void*>(&apply_kernel<K, M, E, true>)
                    : reinterpret_cast<const void*>(&apply_kernel<K, M, E, false>);
}

// Specialised grid-stride kernels: (K, M, E) with E <= M.
static const void* pick_spec(int k, int m, int e, bool per_stripe, const char** name) {
#define RS_SPEC(KK, MM, EE)                                                                             \
  if (k == KK && m == MM && e == EE) {                                                                  \
    *name = per_stripe ? "apply_kernel<" #KK "," #MM "," #EE ",true>" : "apply_kernel<" #KK "," #MM "," #EE ",false>"; \
    return spec_fn<KK, MM, EE>(per_stripe);                                                             \
  }
  RS_SPEC(4, 2, 1) RS_SPEC(4, 2, 2)
  RS_SPEC(8, 4, 1) RS_SPEC(8, 4, 2) RS_SPEC(8, 4, 3) RS_SPEC(8, 4, 4)
  RS_SPEC(10, 4, 1) RS_SPEC(10, 4, 2) RS_SPEC(10, 4, 3) RS_SPEC(10, 4, 4)
  RS_SPEC(6, 3, 1) RS_SPEC(6, 3, 2) RS_SPEC(6, 3, 3)
#undef RS_SPEC
  return nullptr;
}

const uint8_t* bitsliced_encode_rows(int k, int m) {
#define RS_BS(KK, MM) \
  if (k == KK && m == MM) return BsNet<KK, MM>::kRows;
  RS_BS(8, 4) RS_BS(10, 4)
#undef RS_BS
  return nullptr;
}

template <int K, int M>
static const void* bs16_fn() {
  if constexpr (Bs16Net<K, M>::kAvailable) return reinterpret_cast<const void*>(&encode_bs16_kernel<K, M>);
  return nullptr;
}

// Bitsliced encode kernel of (k, m) (the 1 KiB-task pair kernel, 64-column tasks).
// (4,2) and (6,3) are memory-bound on the lookup kernel already, and the bitsliced
// one was slower / level there (profiles/r01_ab_bitsliced*.log).
static const void* pick_bitsliced(int k, int m, const char** name, uint32_t* task_cols) {
  *task_cols = 64u;
#define RS_BS16K(KK, MM)                                          \
  if (k == KK && m == MM) {                                       \
    if (const void* f = bs16_fn<KK, MM>()) {                      \
      *name = "encode_bs16_kernel<" #KK "," #MM ">";              \
      return f;                                                   \
    }                                                             \
  }
  RS_BS16K(8, 4)
  RS_BS16K(10, 4)
#undef RS_BS16K
  return nullptr;
}

// Flat per-stripe reconstruct for (K, M) and the launch's erasure bound E: E = M,
// or the bound a caller (host masks: their maximum; device masks: max_missing)
// gives -- E <= 2 runs input-outer with x[K] as the only per-input state.
static const void* pick_flat_ps(int k, int m, int e, const char** name) {
#define RS_PSFLAT(KK, MM, EE)                                                 \
  if (k == KK && m == MM && e == EE) {                                        \
    *name = "apply_flat_seg_kernel<" #KK "," #MM "," #EE ">";                 \
    return reinterpret_cast<const void*>(&apply_flat_seg_kernel<KK, MM, EE>); \
  }
  RS_PSFLAT(4, 2, 1) RS_PSFLAT(4, 2, 2)
  RS_PSFLAT(8, 4, 1) RS_PSFLAT(8, 4, 2) RS_PSFLAT(8, 4, 4)
  RS_PSFLAT(10, 4, 1) RS_PSFLAT(10, 4, 2) RS_PSFLAT(10, 4, 4)
  RS_PSFLAT(6, 3, 1) RS_PSFLAT(6, 3, 2) RS_PSFLAT(6, 3, 3)
#undef RS_PSFLAT
  return nullptr;
}

// Default workgroups per CU, measured with tools/ab_bench.py on MI355X
// (profiles/r01_ab_occupancy.log, r04p_bpc_k8_k10.log): the streaming pattern wants
// few waves (tools/hbm_probe2.hip: 1-2 WG/CU beat higher occupancy) until the
// per-byte VALU work (K*E lookups) needs more waves to hide latency.
uint32_t default_blocks_per_cu(int k, int e) { return k * e >= 24 ? 6u : 2u; }

// The stripe-aligned per-stripe kernels sized for E > 2 (apply_kernel<K, M, M,
// true>: occupancy 3) run as many short workgroups instead of a grid-stride loop over
// 6 per CU (round 4, profiles/r04x_bpc_em.log, >= 100 ms per point): RS(8+4) 64 KiB
// unbounded 1-erasure 75.1 -> 80.1 %, 2-erasure 71.4 -> 78.7 %, 4-erasure 69.7 ->
// 70.8 %, mixed 0..4 66.0 -> 70.4 %; RS(10+4) at S = 6144 72.4 -> 75.8 %, 68.9 ->
// 75.0 %, 67.8 -> 68.5 %.  The flat and bitsliced kernels do not gain (r04v, r04p).
constexpr uint32_t kEmBlocksPerCu = 64;

// Grid for `waves` wave-tasks: 4 waves per workgroup, at most blocks_per_cu
// workgroups per CU (the kernels grid-stride over the rest).
static dim3 grid_for(uint64_t waves, uint32_t blocks_per_cu, uint32_t cu_count) {
  const uint64_t cap = static_cast<uint64_t>(cu_count) * blocks_per_cu;
  const uint64_t need = (waves + 3) / 4;
  const uint64_t g = need < cap ? need : cap;
  return dim3(static_cast<uint32_t>(g > 0 ? g : 1));
}

// Grid with one wave per task (4 waves per workgroup), capped at 2^31 - 1 workgroups
// (the kernels grid-stride over anything beyond).
static dim3 full_grid(uint64_t waves) {
  const uint64_t need = (waves + 3) / 4;
  return dim3(static_cast<uint32_t>(need < 0x7FFFFFFFull ? need : 0x7FFFFFFFull));
}

// Occupancy caps (round 5).  A launch's waves per SIMD are set by its registers
// unless capped: a workgroup of 4 waves puts one wave on each SIMD, so c
// workgroups per CU = c waves per SIMD, and a dynamic LDS request of 160 KiB / c
// per workgroup (unused by the kernel) admits exactly c of them.  The streaming
// kernels want few waves in flight per SIMD; the cap sets that number
// directly instead of through the register count.  0 = uncapped.
#ifndef RS_OCC_CAP
#define RS_OCC_CAP 0
#endif
// The segmented flat reconstructs (apply_flat_seg_kernel) at 4 waves per SIMD, one
// task per wave (round 5, same-process A/B over shared buffers, 4 rounds,
// profiles/r05d_ab_same_seg.log, RS(10+4) 64 KiB, against round 4's flat kernel):
// bounded 1-erasure 72.2 -> 73.9 %, bounded 2-erasure 73.4 -> 74.7 % (3 or 5 waves:
// 69.7 / 69.4 %), unbounded 2-erasure 68.3 -> 72.0 %, mixed 0..4 57.9 -> 61.8 %,
// mixed 1..4 65.1 -> 66.9 %; unbounded 1- and 4-erasure 69.7 -> 69.0 % and 66.0 ->
// 63.9 %.  Uncapped, the segmented kernels run at 7-8 waves per SIMD and lose 5-7
// points (profiles/r05b_ab_same_flat.log).
#ifndef RS_OCC_CAP_FLAT_E1
#define RS_OCC_CAP_FLAT_E1 4
#endif
#ifndef RS_OCC_CAP_FLAT_E2
#define RS_OCC_CAP_FLAT_E2 4
#endif
#ifndef RS_OCC_CAP_FLAT_EM
#define RS_OCC_CAP_FLAT_EM 4
#endif
#ifndef RS_OCC_CAP_APPLY
#define RS_OCC_CAP_APPLY RS_OCC_CAP
#endif
#ifndef RS_OCC_CAP_BS
#define RS_OCC_CAP_BS RS_OCC_CAP
#endif
// Per-stripe stripe-aligned reconstructs with a bound of 1 or 2 (apply_kernel<K, M,
// E <= 2, true>): 4 waves per SIMD when a stripe spans several 64-column tasks, 5
// for a 1-erasure bound on single-task stripes, uncapped for 2 on single-task
// stripes.  Same-process A/B over object sizes (profiles/r05k_ab_caps_sizes.log,
// RS(4+2), 4 rounds): 1-erasure 16 KiB / 64 KiB / 1 MiB objects +4.2 / +3.8 / +2.4
// points at 4 waves, 4 KiB objects +1.3 at 5 (-1.0 at 4); 2-erasure +0.8 to +1.1 at
// 4 for 16 KiB and more, 4 KiB objects (the headline) -1.7 at 4 and level at 5-6;
// RS(8+4) 64 KiB 1-erasure +0.6, 2-erasure level.  Encodes and uniform reconstructs
// stay uncapped (4 waves: -1.4 to -5.3).
constexpr size_t kLdsPerCu = 160u * 1024u;

// Raises fn's dynamic-LDS limit on the current device to the whole 160 KiB, once per
// (kernel, device): caps of 1 or 2 workgroups per CU reserve more than the default
// 64 KiB (the attribute used to be set on every such launch).  false
// if the runtime refuses, and the launch then fails instead of running uncapped
// under a label it did not get.
static bool raise_lds_limit(const void* fn) {
  static std::mutex mu;
  static std::vector<std::pair<const void*, int>> done;
  int dev = -1;
  if (hipGetDevice(&dev) != hipSuccess) return false;
  std::lock_guard<std::mutex> g(mu);
  for (const auto& d : done)
    if (d.first == fn && d.second == dev) return true;
  if (hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(kLdsPerCu)) !=
      hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  done.emplace_back(fn, dev);
  return true;
}

// Dynamic LDS bytes that cap `fn` at `cap` workgroups per CU (0: none): halfway
// between 160 KiB / (cap + 1) and 160 KiB / cap, so allocation granularity and any
// static LDS cannot turn c into c - 1 (160 KiB / cap exactly admitted one fewer:
// profiles/r05c_ab_same_occ.log, caps 3 / 5 / 6 ran as 2 / 4 / 5).  kLdsRefused when
// the kernel's LDS limit cannot be raised for the cap.
constexpr size_t kLdsRefused = ~size_t(0);
static size_t occ_lds(const void* fn, uint32_t cap, uint32_t wg_per_wave_slot = 1) {
  if (cap == 0) return 0;
  cap *= wg_per_wave_slot;  // workgroups of fewer than 4 waves: more of them per CU
  const size_t lds = ((kLdsPerCu / cap + kLdsPerCu / (cap + 1)) / 2) & ~size_t(wg_per_wave_slot == 1 ? 1023 : 255);
  if (lds > 65536 && !raise_lds_limit(fn)) return kLdsRefused;  // above the default dynamic-LDS limit
  return lds;
}

// Waves per workgroup of each launch: 4 (256 threads, one wave per SIMD) or 1 (64
// threads).  Every kernel here is wave-independent (no LDS, no barriers), so the
// choice only changes how the dispatcher refills a CU: a 4-wave workgroup frees its
// slots when its slowest wave ends, a 1-wave workgroup as soon as it ends -- which
// pays when the waves of one workgroup do unequal work (the per-stripe erasure counts
// of a mixed scan, the two passes of a task straddling two stripes, stores draining
// behind loads).  Same-process A/B per class (round 6, profiles/r06k_ab_wpw.log, 4
// rounds; points of 8 TB/s, one wave against four):
//   flat E = m reconstruct (scans)      RS(10+4) 64 KiB mixed 0..4 +9.2 (host masks
//                                       +8.4, r06k_ab_wg64.log), 4-erasure +6.8,
//                                       unbounded 2-erasure +1.8            -> 1
//   flat E <= 2                         RS(10+4) bounded 1 / 2: -1.8 / -5.7   -> 4
//   stripe-aligned per-stripe E = m     RS(8+4) mixed +4.3, unbounded 2-erasure +2.0;
//                                       RS(8+4) in place -1.0, RS(6+3) mixed -1.1
//                                                   -> 1 out of place for k >= 8
//   stripe-aligned per-stripe E <= 2    RS(8+4) bounded 1 / 2 +5.1 / +1.7, RS(4+2)
//                                       4 KiB bounded 2 (the headline) +1.2, 1 +1.6,
//                                       16 KiB 1 +4.8; stripes of > 4 tasks (RS(4+2)
//                                       64 KiB / 1 MiB, r06l_ab_pslong.log): 1-erasure
//                                       +2.6 / +3.4, in place +2.0 / +0.8, 2-erasure
//                                       out of place -0.3 to -1.4   -> 1 but for those
//   uniform (encode, one-pattern)       RS(4+2) encode 4 / 64 KiB +1.0 / +4.2,
//                                       one-pattern out of place / in place +1.2 /
//                                       +3.5; RS(6+3) encode -2.4; one-pattern
//                                       reconstructs (r06x_ab_uni.log) RS(10+4)
//                                       +3.4 / +2.6, RS(6+3) +2.7 / +3.6, RS(8+4)
//                                       -0.6 / 0   -> 1 for k <= 4, and for one-pattern
//                                       reconstructs but RS(8+4)'s
//   bitsliced encode                    RS(8+4) +1.7, RS(10+4) -1.2 -> 1 for (8, 4)
//   verify                              RS(10+4) -6.5, RS(4+2) +0.4            -> 4
// RS_WPW_FORCE=4 (or 1) builds every launch with that many (A/B builds).
enum class Wpw { kFlatEm, kFlat, kPsEm, kPs, kUni, kBs, kVerify };
#ifndef RS_WPW_FORCE
#define RS_WPW_FORCE 0
#endif
static uint32_t wpw_for(Wpw cls, const KernelArgs& a) {
  if (RS_WPW_FORCE) return RS_WPW_FORCE;
  switch (cls) {
    case Wpw::kFlatEm: return 1u;
    case Wpw::kPsEm: return a.out && a.k >= 8 ? 1u : 4u;
    case Wpw::kPs:
      return a.k >= 8 || a.blocks_per_stripe <= 4u || a.max_out == 1u || !a.out ? 1u : 4u;
    case Wpw::kUni: return a.k <= 4 || (!a.data_inputs && a.k != 8) ? 1u : 4u;
    case Wpw::kBs: return a.k == 8 && a.m == 4 ? 1u : 4u;
    default: return 4u;
  }
}

// Stop event of the next launches on this thread (set_stop_event): the kernel's own
// completion signal updates it (hipExtLaunchKernel), instead of a marker packet the
// stream processes after the kernel.
#ifndef RS_STOP_EVENT_LAUNCH
#define RS_STOP_EVENT_LAUNCH 1
#endif
static thread_local hipEvent_t t_stop_event = nullptr;
static thread_local bool* t_stop_used = nullptr;

void set_stop_event(hipEvent_t ev, bool* used) {
  t_stop_event = RS_STOP_EVENT_LAUNCH ? ev : nullptr;
  t_stop_used = RS_STOP_EVENT_LAUNCH ? used : nullptr;
}

// hipLaunchKernel of `grid` 4-wave workgroups' worth of waves in workgroups of wpw
// waves, at most `cap` waves per SIMD (0: uncapped; kLdsRefused-style failure if the
// reservation cannot be honoured).  false if the launch fails.
static bool launch_capped(const void* fn, dim3 grid, void** args, uint32_t cap, hipStream_t s, uint32_t wpw = 4) {
  const size_t lds = occ_lds(fn, cap, 4u / wpw);
  if (lds == kLdsRefused) return false;
  uint64_t g = static_cast<uint64_t>(grid.x) * (4u / wpw);
  if (g > 0x7FFFFFFFull) g = 0x7FFFFFFFull - (0x7FFFFFFFull % (4u / wpw));  // kernels grid-stride past it
  if (t_stop_event) {
    if (hipExtLaunchKernel(fn, dim3(static_cast<uint32_t>(g)), dim3(64u * wpw), args, lds, s, nullptr, t_stop_event,
                           0) != hipSuccess)
      return false;
    *t_stop_used = true;
    return true;
  }
  return hipLaunchKernel(fn, dim3(static_cast<uint32_t>(g)), dim3(64u * wpw), args, lds, s) == hipSuccess;
}

// One launch over columns [0, a.shard_len) of every shard (a.shard_len < 2 GiB:
// the dropped-store descriptors cover 2 GiB from the shard base).
static const char* launch_window(const KernelArgs& a, int e, bool per_stripe, uint32_t blocks_per_cu,
                                 uint32_t cu_count, hipStream_t s, int occ_cap) {
  // the launch's waves-per-SIMD cap: the caller's (rs_set_occupancy_cap) or the
  // kernel class's tuned default
  auto cap_of = [&](uint32_t dflt) -> uint32_t { return occ_cap >= 0 ? static_cast<uint32_t>(occ_cap) : dflt; };
  void* args[] = {const_cast<KernelArgs*>(&a)};
  const uint64_t cols = (static_cast<uint64_t>(a.shard_len) + 15u) / 16u;
  const char* name = nullptr;
  const bool generic = a.stripe_plans != nullptr;  // only the generic kernel reads per-stripe plan addresses
  const uint64_t span = cols * 16u + static_cast<uint64_t>(a.k > a.m ? a.k : a.m) * a.shard_pitch;
  if (a.encode_net && !per_stripe && !generic && e == a.m) {
    // flat 128-column tasks straddle at most two stripes (cols >= 128) and address
    // with 32-bit offsets off one stripe base per region
    const bool flat_ok = cols >= 128u && a.data_sp + span < (1ull << 31) && a.parity_sp + span < (1ull << 31);
    uint32_t tc = 128u;
    const void* fn = flat_ok ? pick_bitsliced(a.k, a.m, &name, &tc) : nullptr;
    if (fn) {
      const uint64_t waves = (static_cast<uint64_t>(a.n_stripes) * ((cols + 7u) & ~7ull) + tc - 1u) / tc;
      if (waves == 0) return name;
      // default: one task per wave (profiles/r04zi_bpc_flat.log, >= 100 ms per point:
      // 64 KiB encode RS(8+4) 74.4 -> 80.3 %, RS(10+4) 68.0 -> 76.3 % of 8 TB/s
      // against a grid-stride loop over 6 workgroups per CU)
      const dim3 grid = blocks_per_cu ? grid_for(waves, blocks_per_cu, cu_count) : full_grid(waves);
      // 3 waves per SIMD over the register limit (round 6): RS(8+4) in one-wave
      // workgroups +1.1 points (profiles/r06m_ab_caps.log), RS(10+4) +4.3 / +2.7 at
      // 64 / 80 KiB objects (profiles/r06t_ab_caps2.log)
      const uint32_t bcap = RS_OCC_CAP_BS == 0 ? 3u : RS_OCC_CAP_BS;
      if (!launch_capped(fn, grid, args, cap_of(bcap), s, wpw_for(Wpw::kBs, a))) return nullptr;
      return name;
    }
  }
  if (per_stripe && !generic && (a.out || cols % 64u == 0u) && cols >= 64u &&
      (cols % 64u != 0u || (a.k == 10 && e >= 2)) &&
      a.data_sp + span < (1ull << 31) &&
      a.parity_sp + span < (1ull << 31) && a.out_sp + span < (1ull << 31)) {
    // ragged shard lengths: per-stripe reconstruct over flat 64-column tasks
    if (const void* ff = pick_flat_ps(a.k, a.m, e, &name)) {
      const uint64_t waves = (static_cast<uint64_t>(a.n_stripes) * ((cols + 7u) & ~7ull) + 63u) / 64u;
      if (waves == 0) return name;
      // one task per wave (E <= 2: r04zi, +0.9 / +2.5 points for RS(10+4) 64 KiB 1- /
      // 2-erasure; E = M since round 5's segmented kernel: unbounded 2-erasure and
      // mixed batches +3.5 / +3.9 points, r05b_ab_same_flat.log, r05e_ab_same_em.log)
      const uint32_t bpc = blocks_per_cu ? blocks_per_cu : default_blocks_per_cu(a.k, e);
      const dim3 grid = !blocks_per_cu ? full_grid(waves)
                                                                         : grid_for(waves, bpc, cu_count);
      const uint32_t cap = e == 1 ? RS_OCC_CAP_FLAT_E1 : e == 2 ? RS_OCC_CAP_FLAT_E2 : RS_OCC_CAP_FLAT_EM;
      if (!launch_capped(ff, grid, args, cap_of(cap), s, wpw_for(e > 2 ? Wpw::kFlatEm : Wpw::kFlat, a)))
        return nullptr;
      return name;
    }
  }
  const void* fn = generic ? nullptr : pick_spec(a.k, a.m, e, per_stripe, &name);
  if (!fn) {
    name = per_stripe ? "apply_kernel_generic<true>" : "apply_kernel_generic<false>";
    fn = per_stripe ? reinterpret_cast<const void*>(&apply_kernel_generic<true>)
                    : reinterpret_cast<const void*>(&apply_kernel_generic<false>);
  }
  const uint64_t waves = static_cast<uint64_t>(a.n_stripes) * a.blocks_per_stripe;
  if (waves == 0) return name;
  uint32_t bpc = blocks_per_cu;
  if (!bpc) bpc = (per_stripe && !generic && e > 2) ? kEmBlocksPerCu : default_blocks_per_cu(a.k, e);
  dim3 grid = grid_for(waves, bpc, cu_count);
  // (per-stripe E = M for k < 8 too, round 6, profiles/r06v_ab_emfull.log: RS(6+3)
  // mixed / unbounded 2-erasure +2.1 / +2.3 points under one-wave workgroups; RS(8+4)
  // keeps the capped grid: mixed -1.4, 1-erasure -2.2 with a full one)
  if (!blocks_per_cu && !generic && (a.k < 8 || !(per_stripe && e > 2))) {
    // The specialised E <= 2 and encode kernels run one task per wave: a grid over
    // every task instead of a grid-stride loop over 2 workgroups per CU (round 4,
    // profiles/r04zf_bpc_bounded.log, >= 100 ms per point, 3 rounds): RS(4+2) 4 KiB
    // per-stripe 2-erasure 74.5 -> 78.8 % of 8 TB/s, encode 76.8 -> 79.1 %, uniform
    // 2-erasure 72.6 -> 76.5 %; 64 KiB 2-erasure 74.8 -> 79.8 %, encode 77.1 -> 80.8 %;
    // RS(8+4) 1-/2-erasure 77.6 / 75.2 -> 79.8 / 78.2 %; RS(4+2) 1-erasure 77.2 ->
    // 76.4 %.  Partial grids (32 or 64 per CU, still looping) were slower than both.
    grid = full_grid(waves);
  }
  uint32_t dcap = RS_OCC_CAP_APPLY;
  if (dcap == 0u && per_stripe && !generic && e <= 2)
    dcap = a.k >= 8 && e == 1 ? 3u : a.blocks_per_stripe >= 2u ? 4u : (e == 1 ? 5u : 0u);  // k >= 8, e = 1:
        // 3 in one-wave workgroups, RS(8+4) 64 KiB bounded 1-erasure +1.6 (r06m_ab_caps.log)
  const uint32_t wpw = generic ? 4u : wpw_for(!per_stripe ? Wpw::kUni : e > 2 ? Wpw::kPsEm : Wpw::kPs, a);
  if (!launch_capped(fn, grid, args, generic ? 0u : cap_of(dcap), s, wpw)) return nullptr;
  return name;
}

const char* launch_apply(const KernelArgs& args, int e, bool per_stripe, uint32_t blocks_per_cu, uint32_t cu_count,
                         hipStream_t s, int occ_cap) {
  KernelArgs a = args;
  a.max_out = static_cast<uint32_t>(e);
  if (a.shard_len <= kColumnWindow) return launch_window(a, e, per_stripe, blocks_per_cu, cu_count, s, occ_cap);
  // Shards of 1 GiB or more (one huge Encode of an object of several GiB): the
  // codec is column-wise, so columns [x, x + W) of every shard are an independent
  // batch whose slots all start x bytes later.  Windows run in order on s.
  const char* name = nullptr;
  for (uint64_t x = 0; x < a.shard_len; x += kColumnWindow) {
    KernelArgs w = a;
    w.data += x;
    if (w.parity) w.parity += x;
    if (w.out) w.out += x;
    const uint64_t len = a.shard_len - x < kColumnWindow ? a.shard_len - x : kColumnWindow;
    w.shard_len = static_cast<uint32_t>(len);
    w.full_cols = w.shard_len / 16u;
    w.blocks_per_stripe = ((w.shard_len + 15u) / 16u + 63u) / 64u;
    name = launch_window(w, e, per_stripe, blocks_per_cu, cu_count, s, occ_cap);
    if (!name) return nullptr;
  }
  return name;
}

bool apply_ptrs_supported(int k, int m) {
  return (k == 4 && m == 2) || (k == 8 && m == 4) || (k == 10 && m == 4) || (k == 6 && m == 3);
}

const char* launch_apply_ptrs(const KernelArgs& a, int e_bound, uint32_t blocks_per_cu, uint32_t cu_count,
                              hipStream_t s) {
  const void* fn = nullptr;
  const char* name = nullptr;
  const int e = e_bound <= 2 ? e_bound : a.m;  // E = 1, 2 or m
#define RS_PTRS(KK, MM, EE)                                                 \
  if (!fn && a.k == KK && a.m == MM && e == EE) {                           \
    fn = reinterpret_cast<const void*>(&apply_ptr_kernel<KK, MM, EE>);     \
    name = "apply_ptr_kernel<" #KK "," #MM "," #EE ">";                     \
  }
  RS_PTRS(4, 2, 1) RS_PTRS(4, 2, 2)
  RS_PTRS(8, 4, 1) RS_PTRS(8, 4, 2) RS_PTRS(8, 4, 4)
  RS_PTRS(10, 4, 1) RS_PTRS(10, 4, 2) RS_PTRS(10, 4, 4)
  RS_PTRS(6, 3, 1) RS_PTRS(6, 3, 2) RS_PTRS(6, 3, 3)
#undef RS_PTRS
  if (!fn) return nullptr;  // shapes without a specialisation stage their slots instead
  KernelArgs b = a;
  b.max_out = static_cast<uint32_t>(e);
  void* args[] = {&b};
  const uint64_t waves = static_cast<uint64_t>(a.n_stripes) * a.blocks_per_stripe;
  if (waves == 0) return name;
  if (hipLaunchKernel(fn, grid_for(waves, blocks_per_cu, cu_count), dim3(256), args, 0, s) != hipSuccess) return nullptr;
  return name;
}

const char* launch_verify(const KernelArgs& a, uint32_t blocks_per_cu, uint32_t cu_count, hipStream_t s) {
  const void* fn = nullptr;
  const char* name = "verify_kernel_generic";
#define RS_VSPEC(KK, MM)                                                  \
  if (!fn && a.k == KK && a.m == MM) {                                    \
    fn = reinterpret_cast<const void*>(&verify_kernel<KK, MM>);           \
    name = "verify_kernel<" #KK "," #MM ">";                              \
  }
  RS_VSPEC(4, 2) RS_VSPEC(8, 4) RS_VSPEC(10, 4) RS_VSPEC(6, 3)
#undef RS_VSPEC
  if (!fn) fn = reinterpret_cast<const void*>(&verify_kernel_generic);
  if (hipMemsetAsync(a.bad, 0, static_cast<size_t>(a.n_stripes) * 4u, s) != hipSuccess) return nullptr;
  uint64_t waves = static_cast<uint64_t>(a.n_stripes) * a.blocks_per_stripe;
  // flat 64-column tasks when a stripe's columns do not fill whole 64-column blocks
  const uint64_t cols = (static_cast<uint64_t>(a.shard_len) + 15u) / 16u;
  const uint64_t span = cols * 16u + static_cast<uint64_t>(a.k > a.m ? a.k : a.m) * a.shard_pitch;
  if (cols >= 64u && cols % 64u != 0u && a.data_sp + span < (1ull << 31) &&
      a.parity_sp + span < (1ull << 31)) {
    const void* ff = nullptr;
#define RS_VFLAT(KK, MM) \
    if (!ff && a.k == KK && a.m == MM) { ff = reinterpret_cast<const void*>(&verify_flat_kernel<KK, MM>); name = "verify_flat_kernel<" #KK "," #MM ">"; }
    RS_VFLAT(4, 2) RS_VFLAT(8, 4) RS_VFLAT(10, 4) RS_VFLAT(6, 3)
#undef RS_VFLAT
    if (ff) {
      fn = ff;
      waves = (static_cast<uint64_t>(a.n_stripes) * ((cols + 7u) & ~7ull) + 63u) / 64u;
    }
  }
  if (waves == 0) return name;
  void* args[] = {const_cast<KernelArgs*>(&a)};
  if (!launch_capped(fn, grid_for(waves, blocks_per_cu, cu_count), args, 0u, s, wpw_for(Wpw::kVerify, a)))
    return nullptr;
  return name;
}

// Row offsets of a packed out-of-place batch: an exclusive prefix sum of the
// stripes' erasure counts, by one workgroup of 1024 threads walking the masks in
// chunks of 16 384 (16 per thread, each thread's in a run), a running total carried
// from chunk to chunk.  Tiny next to the reconstruct it precedes (one mask word per
// 64 KiB object); dst[n] = the batch's total row count.  A stripe missing more than
// max_rows shards (fewer than k present: never rebuilt) takes no rows.
__global__ __launch_bounds__(1024) void row_offsets_kernel(const uint32_t* __restrict__ masks, uint32_t full,
                                                           uint32_t max_rows, uint32_t* __restrict__ dst,
                                                           uint64_t n) {
  constexpr uint32_t kPer = 16, kChunk = 1024u * kPer;
  __shared__ uint32_t wsum[16];
  __shared__ uint32_t carry;
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wid = tid >> 6;
  if (tid == 0) carry = 0u;
  __syncthreads();
  for (uint64_t base = 0; base < n; base += kChunk) {
    const uint64_t i0 = base + static_cast<uint64_t>(tid) * kPer;
    uint32_t cnt[kPer], sum = 0u;
#pragma unroll
    for (uint32_t j = 0; j < kPer; ++j) {
      const uint32_t c = i0 + j < n ? static_cast<uint32_t>(__builtin_popcount(~masks[i0 + j] & full)) : 0u;
      cnt[j] = c > max_rows ? 0u : c;
      sum += cnt[j];
    }
    // inclusive scan of the threads' sums within the wave, then across the 16 waves
    uint32_t inc = sum;
#pragma unroll
    for (uint32_t d = 1; d < 64; d <<= 1) {
      const uint32_t v = __shfl_up(inc, d, 64);
      if (lane >= d) inc += v;
    }
    if (lane == 63u) wsum[wid] = inc;
    __syncthreads();
    uint32_t before = carry;
    for (uint32_t w = 0; w < wid; ++w) before += wsum[w];
    uint32_t run = before + inc - sum;  // exclusive start of this thread's run
#pragma unroll
    for (uint32_t j = 0; j < kPer; ++j) {
      if (i0 + j < n) dst[i0 + j] = run;
      run += cnt[j];
    }
    __syncthreads();
    if (tid == 1023u) carry = run;  // the last thread's run ends the chunk
    __syncthreads();
  }
  if (tid == 0) dst[n] = carry;
}

bool launch_row_offsets(const uint32_t* masks, uint32_t full, uint32_t max_rows, uint32_t* dst, uint64_t n,
                        hipStream_t s) {
  hipLaunchKernelGGL(row_offsets_kernel, dim3(1), dim3(1024), 0, s, masks, full, max_rows, dst, n);
  return hipGetLastError() == hipSuccess;
}

// Per-stripe host masks into device memory, read straight from the pinned slot over
// PCIe: one 16-B load per lane (tail words singly), on the launch stream itself.
// Words [0, n) of src to dst, then words [n, n + n2) of src to dst2 (a second array
// staged behind the first in the same pinned slot: a packed batch's row offsets) --
// one launch for both.
__global__ __launch_bounds__(256) void words_copy_kernel(const uint32_t* __restrict__ src, uint32_t* __restrict__ dst,
                                                         uint64_t n, uint32_t* __restrict__ dst2, uint64_t n2) {
  const uint64_t i = (static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x) * 4u;
  if (i + 4u <= n) {
    *reinterpret_cast<u32x4*>(dst + i) = *reinterpret_cast<const u32x4*>(src + i);
    return;
  }
  const uint64_t end = n + n2;
  for (uint64_t j = i; j < i + 4u && j < end; ++j) {
    const uint32_t w = src[j];
    if (j < n)
      dst[j] = w;
    else
      dst2[j - n] = w;
  }
}

bool launch_words_copy(const uint32_t* src, uint32_t* dst, uint64_t n, hipStream_t s, uint32_t* dst2, uint64_t n2) {
  if (n + n2 == 0) return true;
  const uint64_t blocks = (n + n2 + 1023u) / 1024u;
  hipLaunchKernelGGL(words_copy_kernel, dim3(static_cast<uint32_t>(blocks)), dim3(256), 0, s, src, dst, n, dst2, n2);
  return hipGetLastError() == hipSuccess;
}

void launch_copy(const void* src, void* dst, uint64_t bytes, uint32_t grid_blocks, hipStream_t s) {
  hipLaunchKernelGGL(copy_kernel, dim3(grid_blocks), dim3(256), 0, s, static_cast<const uint8_t*>(src),
                     static_cast<uint8_t*>(dst), bytes);
}

}  // namespace rs
