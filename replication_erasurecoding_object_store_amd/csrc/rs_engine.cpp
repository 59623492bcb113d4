// rs_engine.cpp -- librsgpu.so: the C-ABI in include/rsgpu.h.
//
// Host runtime around the gfx950 kernels in rs_kernels.hip:
//   * encode matrix and per-erasure-pattern decode plans (the analogue of
//     klauspost's inversion_tree.go cache, [upstream reedsolomon.go reconstruct]),
//     built once per pattern and kept resident in HBM;
//   * for k+m <= 16 every pattern with 1..m erasures is precomputed at rs_create and
//     indexed by a dense missing-mask -> plan LUT, so a batch may carry a different
//     erasure pattern per stripe with no host work per stripe;
//   * per-object host calls (the IEcDriver drop-in: ec.go:54-61) run on a pool of
//     "lanes" (stream + pinned staging + device slab) so concurrent goroutines do
//     not serialise on one stream;
//   * host-resident batches are pipelined H2D -> kernel -> D2H over 3 streams.
// No CPU arithmetic path exists: every parity / reconstructed byte comes from a
// HIP kernel.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/rsgpu.h"
#include "gf256.hpp"
#include "rs_host_util.hpp"
#include "rs_plan.hpp"
#include "rs_sha256.hpp"

namespace {

using rs::Matrix;

using rs::check_shards;
using rs::DevBuf;
using rs::PinnedBuf;
using rs::round_up;

// Default workgroups (256 threads) per CU for the batched kernels, measured with
// tools/ab_bench.py on MI355X (profiles/r01_ab_occupancy.log): the streaming
// pattern wants few waves (tools/hbm_probe2.hip: 1-2 WG/CU beat higher occupancy)
// until the per-byte VALU work (K*E lookups) needs more waves to hide latency.
constexpr int kDefaultBlocksPerCu = 0;  // 0 = pick by shape
int default_blocks_per_cu(int k, int e) { return k * e >= 24 ? 6 : 2; }

// ---- plan construction -----------------------------------------------------
// 3-chunk v_perm tables for coefficient f (see rs_kernels.hip):
//   A[v] = f*v (v<8), B[v] = f*(v<<3) (v<8), C[v] = f*(v<<6) (v<4).
void perm_tables(uint8_t f, uint32_t* t) {
  const rs::Field& F = rs::field();
  auto pack4 = [&](int base, int shift) {
    uint32_t w = 0;
    for (int j = 0; j < 4; ++j)
      w |= static_cast<uint32_t>(F.mul(f, static_cast<uint8_t>((base + j) << shift))) << (8 * j);
    return w;
  };
  t[0] = pack4(0, 0);
  t[1] = pack4(4, 0);
  t[2] = pack4(0, 3);
  t[3] = pack4(4, 3);
  t[4] = pack4(0, 6);
}

// rows: n_out x k coefficient matrix (row-major).
std::vector<uint8_t> make_plan(int k, int m, const std::vector<int>& in_idx, const std::vector<int>& out_idx,
                               const std::vector<uint8_t>& rows) {
  std::vector<uint8_t> p(rs::plan_stride(k, m), 0);
  const uint32_t n_out = static_cast<uint32_t>(out_idx.size());
  std::memcpy(p.data(), &n_out, 4);
  uint32_t* ii = reinterpret_cast<uint32_t*>(p.data() + 8);
  for (int c = 0; c < k; ++c) ii[c] = static_cast<uint32_t>(in_idx[c]);
  for (size_t r = 0; r < out_idx.size(); ++r) ii[k + r] = static_cast<uint32_t>(out_idx[r]);
  uint32_t* tab = reinterpret_cast<uint32_t*>(p.data() + rs::plan_tab_offset(k, m));
  for (size_t r = 0; r < out_idx.size(); ++r)
    for (int c = 0; c < k; ++c) perm_tables(rows[r * k + c], tab + (r * k + c) * 5);
  return p;
}

// Composed reconstruct plan for a present-shard mask over k+m shards.
// Survivors = first k present shards in index order [upstream reconstruct];
// a missing data shard d is row d of inv(sub) (phase 1); a missing parity shard p
// is P[p] x inv(sub) (phase 2 over the recovered data, folded into one pass).
int make_decode_plan(int k, int m, const Matrix& enc, uint64_t present, bool data_only,
                     std::vector<uint8_t>* out) {
  const rs::Field& F = rs::field();
  const int t = k + m;
  std::vector<int> surv, miss;
  for (int i = 0; i < t; ++i) {
    if ((present >> i) & 1u) {
      if (static_cast<int>(surv.size()) < k) surv.push_back(i);
    } else if (!data_only || i < k) {
      miss.push_back(i);
    }
  }
  if (static_cast<int>(surv.size()) < k) return RS_ERR_TOO_FEW_SHARDS;
  Matrix sub(k, k), dec;
  for (int r = 0; r < k; ++r)
    for (int c = 0; c < k; ++c) sub.at(r, c) = enc.at(surv[r], c);
  if (!rs::invert(sub, &dec)) return RS_ERR_SINGULAR;
  std::vector<uint8_t> rows(miss.size() * k);
  for (size_t r = 0; r < miss.size(); ++r) {
    const int s = miss[r];
    for (int c = 0; c < k; ++c) {
      uint8_t v;
      if (s < k) {
        v = dec.at(s, c);
      } else {
        v = 0;
        for (int d = 0; d < k; ++d) v ^= F.mul(enc.at(s, d), dec.at(d, c));
      }
      rows[r * k + c] = v;
    }
  }
  *out = make_plan(k, m, surv, miss, rows);
  return RS_OK;
}

// ---- buffers -------------------------------------------------------------------
// A lane serves one synchronous host call at a time.
struct Lane {
  hipStream_t stream = nullptr;
  DevBuf dev;
  PinnedBuf host;
};

// Upload slot for per-stripe masks passed in host memory (async device calls).
struct UploadSlot {
  PinnedBuf host;
  DevBuf dev;
  hipEvent_t done = nullptr;
  bool used = false;
};

// Split shard layout shared by host and device buffers (see rs_plan.hpp).
struct Layout {
  uint8_t* data;
  size_t data_sp;
  uint8_t* parity;
  size_t parity_sp;
  size_t pitch;
  uint8_t* slot(int k, size_t stripe, int s) const {
    return s < k ? data + stripe * data_sp + static_cast<size_t>(s) * pitch
                 : parity + stripe * parity_sp + static_cast<size_t>(s - k) * pitch;
  }
  size_t stripe_pitch(int k, int s) const { return s < k ? data_sp : parity_sp; }
};

}  // namespace

// ---- host batch pipeline state ---------------------------------------------------
// Chunks of stripes flow H2D -> kernel -> D2H on kHostStreams streams; each stream
// has its own device slab (split layout), so chunk j+1's copies overlap chunk j's
// kernel and D2H.  Kept in the context: creating streams and slabs per call cost
// more than a small call's transfers.
constexpr int kHostStreams = 4;
constexpr size_t kHostChunkBytes = size_t(16) << 20;  // device bytes per chunk

struct HostPipe {
  hipStream_t st[kHostStreams] = {};
  DevBuf buf[kHostStreams];
  ~HostPipe() {
    for (auto& s : st)
      if (s) (void)hipStreamDestroy(s);
  }
};

struct rs_ctx {
  int k = 0, m = 0, device = 0, cu_count = 0;
  int blocks_per_cu = kDefaultBlocksPerCu;
  bool force_generic = false;
  bool bitsliced = false;  // generated encode XOR program matches enc (rs_create)
  std::string backend;
  Matrix enc;

  DevBuf d_enc_plan;              // encode plan (uniform)
  DevBuf d_plans, d_lut;          // eager all-pattern plans + LUT (k+m <= 16)
  uint32_t n_plans = 0;
  std::vector<uint32_t> h_lut;    // missing mask -> plan index
  bool have_lut = false;
  std::mutex plan_mu;             // uniform plans built on demand (k+m > 16 / data-only)
  std::unordered_map<uint64_t, std::unique_ptr<DevBuf>> plan_cache;

  DevBuf d_status, d_scratch;     // device status word (per-stripe calls); store sink
  PinnedBuf h_status;

  std::mutex lane_mu;
  std::condition_variable lane_cv;
  std::vector<std::unique_ptr<Lane>> lanes;
  std::vector<Lane*> free_lanes;
  int max_lanes = 8;

  std::mutex upload_mu;
  static constexpr size_t kUploadSlots = 4;
  UploadSlot uploads[kUploadSlots];
  size_t upload_next = 0;

  std::mutex host_mu;             // host-resident batches: one at a time per context
  HostPipe host_pipe;
  bool host_zero_copy = true;     // pinned host batches: kernel reads/writes them in place
  DevBuf d_bad;                   // zero-copy verify: per-stripe result before D2H
  std::atomic<const char*> last_host_path{"none"};

  std::atomic<const char*> last_kernel{"none"};

  ~rs_ctx() {
    for (auto& s : uploads)
      if (s.done) (void)hipEventDestroy(s.done);
    for (auto& l : lanes)
      if (l->stream) (void)hipStreamDestroy(l->stream);
  }
};

namespace {

rs::KernelArgs make_args(rs_ctx* c, const Layout& L, size_t S, size_t N) {
  rs::KernelArgs a{};
  a.data = L.data;
  a.parity = L.parity;
  a.data_sp = L.data_sp;
  a.parity_sp = L.parity_sp;
  a.shard_pitch = L.pitch;
  a.shard_len = static_cast<uint32_t>(S);
  a.n_stripes = static_cast<uint32_t>(N);
  a.blocks_per_stripe = static_cast<uint32_t>((round_up(S, 16) / 16 + 63) / 64);
  a.full_cols = static_cast<uint32_t>(S / 16);
  a.blocks_full = (a.full_cols + 63u) / 64u;
  a.k = c->k;
  a.m = c->m;
  a.full_mask = (c->k + c->m >= 32) ? 0xFFFFFFFFu : ((1u << (c->k + c->m)) - 1u);
  a.plan_bytes = rs::plan_stride(c->k, c->m);
  a.scratch = static_cast<uint8_t*>(c->d_scratch.p);
  a.status = static_cast<uint32_t*>(c->d_status.p);
  a.lut = static_cast<const uint32_t*>(c->d_lut.p);
  return a;
}

// e = outputs per stripe (m for encode, #missing for a uniform reconstruct, max
// #missing for per-stripe patterns).
int launch(rs_ctx* c, const rs::KernelArgs& args, int e, bool per_stripe, hipStream_t s) {
  if (args.n_stripes == 0 || args.shard_len == 0 || e <= 0) return RS_OK;
  rs::KernelArgs a = args;
  // the encode plan with a verified generated XOR program -> bitsliced kernel
  a.encode_net = (c->bitsliced && !per_stripe && a.plans == c->d_enc_plan.p) ? 1u : 0u;
  const int bpc = c->blocks_per_cu > 0 ? c->blocks_per_cu : default_blocks_per_cu(c->k, e);
  const char* name = rs::launch_apply(a, e, per_stripe, static_cast<uint32_t>(bpc),
                                      static_cast<uint32_t>(c->cu_count), s, c->force_generic);
  if (!name) return RS_ERR_DEVICE;
  c->last_kernel.store(name);
  RS_HIP(hipGetLastError());
  return RS_OK;
}

int launch_verify_args(rs_ctx* c, rs::KernelArgs& a, hipStream_t s) {
  a.plans = static_cast<const uint8_t*>(c->d_enc_plan.p);
  const int bpc = c->blocks_per_cu > 0 ? c->blocks_per_cu : default_blocks_per_cu(c->k, c->m);
  const char* name = rs::launch_verify(a, static_cast<uint32_t>(bpc), static_cast<uint32_t>(c->cu_count), s,
                                       c->force_generic);
  if (!name) return RS_ERR_DEVICE;
  c->last_kernel.store(name);
  RS_HIP(hipGetLastError());
  return RS_OK;
}

uint64_t full_mask64(int t) { return (t >= 64) ? ~0ull : ((1ull << t) - 1); }

// Device pointer of the plan for one erasure pattern (cached).
int uniform_plan(rs_ctx* c, uint64_t present, bool data_only, const uint8_t** plan_dev) {
  const int t = c->k + c->m;
  present &= full_mask64(t);
  if (__builtin_popcountll(present) < c->k) return RS_ERR_TOO_FEW_SHARDS;
  if (c->have_lut && !data_only) {
    const uint32_t missing = static_cast<uint32_t>(~present & full_mask64(t));
    const uint32_t pid = c->h_lut[missing];
    if (pid == rs::kPlanInvalid) return RS_ERR_TOO_FEW_SHARDS;
    *plan_dev = static_cast<const uint8_t*>(c->d_plans.p) + static_cast<size_t>(pid) * rs::plan_stride(c->k, c->m);
    return RS_OK;
  }
  const uint64_t key = present | (data_only ? (1ull << 63) : 0ull);
  std::lock_guard<std::mutex> g(c->plan_mu);
  auto it = c->plan_cache.find(key);
  if (it == c->plan_cache.end()) {
    std::vector<uint8_t> plan;
    int rc = make_decode_plan(c->k, c->m, c->enc, present, data_only, &plan);
    if (rc) return rc;
    auto buf = std::make_unique<DevBuf>();
    if (buf->ensure(plan.size())) return RS_ERR_DEVICE;
    RS_HIP(hipMemcpy(buf->p, plan.data(), plan.size(), hipMemcpyHostToDevice));
    it = c->plan_cache.emplace(key, std::move(buf)).first;
  }
  *plan_dev = static_cast<const uint8_t*>(it->second->p);
  return RS_OK;
}

// RAII lane checkout.
struct LaneGuard {
  rs_ctx* c;
  Lane* lane = nullptr;
  int rc = RS_OK;
  explicit LaneGuard(rs_ctx* ctx) : c(ctx) {
    std::unique_lock<std::mutex> g(c->lane_mu);
    if (c->free_lanes.empty() && static_cast<int>(c->lanes.size()) < c->max_lanes) {
      auto l = std::make_unique<Lane>();
      if (hipSetDevice(c->device) != hipSuccess ||
          hipStreamCreateWithFlags(&l->stream, hipStreamNonBlocking) != hipSuccess) {
        rc = RS_ERR_DEVICE;
        return;
      }
      c->free_lanes.push_back(l.get());
      c->lanes.push_back(std::move(l));
    }
    c->lane_cv.wait(g, [&] { return !c->free_lanes.empty(); });
    lane = c->free_lanes.back();
    c->free_lanes.pop_back();
  }
  ~LaneGuard() {
    if (!lane) return;
    std::lock_guard<std::mutex> g(c->lane_mu);
    c->free_lanes.push_back(lane);
    c->lane_cv.notify_one();
  }
};

// [upstream reedsolomon.go checkShards(shards, nilok)] + shardSize.
// One object through a lane: pack inputs into pinned staging, H2D, one kernel,
// D2H of the outputs, unpack.  in/out slots are shard indices into `shards`.
int run_object(rs_ctx* c, const uint8_t* plan_dev, const std::vector<int>& in_idx, const std::vector<int>& out_idx,
               uint8_t* const* shards, size_t S) {
  if (S > 0xFFFFFFF0u) return RS_ERR_INVALID_ARG;
  LaneGuard lg(c);
  if (lg.rc) return lg.rc;
  Lane* L = lg.lane;
  const int t = c->k + c->m;
  const size_t P = round_up(S, 256);  // 256-B slots: see batch.shard_pitch_for
  const size_t bytes = P * static_cast<size_t>(t);
  if (L->dev.ensure(bytes) || L->host.ensure(bytes)) return RS_ERR_DEVICE;
  uint8_t* h = static_cast<uint8_t*>(L->host.p);
  uint8_t* d = static_cast<uint8_t*>(L->dev.p);
  for (int s : in_idx) std::memcpy(h + static_cast<size_t>(s) * P, shards[s], S);
  const int lo = *std::min_element(in_idx.begin(), in_idx.end());
  const int hi = *std::max_element(in_idx.begin(), in_idx.end());
  RS_HIP(hipMemcpyAsync(d + lo * P, h + lo * P, (hi - lo + 1) * P, hipMemcpyHostToDevice, L->stream));
  const Layout dl{d, bytes, d + static_cast<size_t>(c->k) * P, bytes, P};
  rs::KernelArgs a = make_args(c, dl, S, 1);
  a.plans = plan_dev;
  int rc = launch(c, a, static_cast<int>(out_idx.size()), false, L->stream);
  if (rc) return rc;
  for (int s : out_idx)
    RS_HIP(hipMemcpyAsync(h + static_cast<size_t>(s) * P, d + static_cast<size_t>(s) * P, S, hipMemcpyDeviceToHost,
                          L->stream));
  RS_HIP(hipStreamSynchronize(L->stream));
  for (int s : out_idx) std::memcpy(shards[s], h + static_cast<size_t>(s) * P, S);
  return RS_OK;
}

int reconstruct_impl(rs_ctx* c, uint8_t* const* shards, size_t* lens, bool data_only) {
  if (!c || !shards || !lens) return RS_ERR_INVALID_ARG;
  const int t = c->k + c->m;
  size_t S = 0;
  int rc = check_shards(t, lens, true, &S);
  if (rc) return rc;
  uint64_t present = 0;
  int np = 0, data_present = 0;
  for (int i = 0; i < t; ++i)
    if (lens[i]) {
      present |= 1ull << i;
      ++np;
      if (i < c->k) ++data_present;
    }
  if (np == t || (data_only && data_present == c->k)) return RS_OK;
  if (np < c->k) return RS_ERR_TOO_FEW_SHARDS;
  std::vector<int> surv, miss;
  for (int i = 0; i < t; ++i) {
    if (lens[i]) {
      if (static_cast<int>(surv.size()) < c->k) surv.push_back(i);
    } else if (!data_only || i < c->k) {
      if (!shards[i]) return RS_ERR_INVALID_ARG;
      miss.push_back(i);
    }
  }
  const uint8_t* plan = nullptr;
  rc = uniform_plan(c, present, data_only, &plan);
  if (rc) return rc;
  rc = run_object(c, plan, surv, miss, shards, S);
  if (rc) return rc;
  for (int s : miss) lens[s] = S;
  return RS_OK;
}

// NULL = the HIP null stream (as in HIP's own APIs), so torch's default stream and
// the engine order against each other.
hipStream_t as_stream(void* s) { return static_cast<hipStream_t>(s); }

bool device_layout_ok(const Layout& L, int m, size_t S) {
  auto al = [](const void* p) { return reinterpret_cast<uintptr_t>(p) % 16 == 0; };
  return al(L.data) && (m == 0 || al(L.parity)) && L.data_sp % 16 == 0 && L.parity_sp % 16 == 0 &&
         L.pitch % 16 == 0 && L.pitch >= round_up(S, 16);
}

// Out-of-place outputs at out + i*out_sp + r*pitch (r < e) must not overlap:
// stripe-major (the e outputs of a stripe inside its out_sp) or plane-major
// (output r of every stripe in its own plane of N*out_sp bytes, the SoA layout).
bool out_layout_ok(size_t out_sp, size_t pitch, size_t S, size_t N, int e) {
  const size_t slot = round_up(S, 16);
  if (e <= 1) return out_sp >= slot || N == 1;
  return (out_sp >= static_cast<size_t>(e) * pitch && pitch >= slot) || (out_sp >= slot && pitch >= N * out_sp);
}

bool batch_sizes_ok(size_t S, size_t N, size_t pitch) {
  if (S > 0xFFFFFFF0u || N > 0xFFFFFFFFu || pitch < S) return false;
  const uint64_t cols = round_up(S, 16) / 16;
  return N * ((cols + 63) / 64) < 0xFFFFFFFFull;  // task ids fit 32 bits
}

hipError_t copy2d(void* dst, size_t dpitch, const void* src, size_t spitch, size_t width, size_t rows,
                  hipMemcpyKind kind, hipStream_t s) {
  if (rows == 0 || width == 0) return hipSuccess;
  if (dpitch == width && spitch == width) return hipMemcpyAsync(dst, src, width * rows, kind, s);
  return hipMemcpy2DAsync(dst, dpitch, src, spitch, width, rows, kind, s);
}

// Copies the listed slots of n stripes between two layouts.  Runs of consecutive
// slots that are back to back in one region of both layouts travel as one 2D copy.
int copy_slots(const Layout& dst, const Layout& src, int k, const std::vector<int>& slots, size_t s_dst0,
               size_t s_src0, size_t n, size_t S, hipMemcpyKind kind, hipStream_t st) {
  size_t i = 0;
  while (i < slots.size()) {
    size_t j = i + 1;
    while (j < slots.size() && slots[j] == slots[j - 1] + 1 && (slots[j] < k) == (slots[i] < k) && dst.pitch == S &&
           src.pitch == S)
      ++j;
    const int s0 = slots[i];
    RS_HIP(copy2d(dst.slot(k, s_dst0, s0), dst.stripe_pitch(k, s0), src.slot(k, s_src0, s0), src.stripe_pitch(k, s0),
                  S * (j - i), n, kind, st));
    i = j;
  }
  return RS_OK;
}

int upload_masks(rs_ctx* c, const uint32_t* masks, size_t n, hipStream_t s, const uint32_t** dev);

// GPU address of a pinned host range [p, p+bytes) (hipHostMalloc'ed or
// rs_host_register'ed), or nullptr if any part of it is pageable.
uint8_t* mapped(const void* p, size_t bytes) {
  if (!p || bytes == 0) return nullptr;
  hipPointerAttribute_t a{}, b{};
  if (hipPointerGetAttributes(&a, p) != hipSuccess || a.type != hipMemoryTypeHost || !a.devicePointer) {
    (void)hipGetLastError();
    return nullptr;
  }
  const void* last = static_cast<const uint8_t*>(p) + bytes - 1;
  if (hipPointerGetAttributes(&b, last) != hipSuccess || b.type != hipMemoryTypeHost || !b.devicePointer) {
    (void)hipGetLastError();
    return nullptr;
  }
  uint8_t* d = static_cast<uint8_t*>(a.devicePointer);
  if (static_cast<uint8_t*>(b.devicePointer) != d + (bytes - 1)) return nullptr;  // one linear mapping
  return d;
}

// Zero-copy host batch: with the shards in pinned host memory the kernel itself
// reads the K survivors and writes only the missing shards across PCIe, in place
// -- per stripe exactly the bytes the codec needs, no staging slab, no DMA of
// slots it does not touch (the staged pipeline must move every slot a stripe
// might use).  Returns RS_ERR_NOT_SUPPORTED when the layout does not qualify.
int host_zero_copy(rs_ctx* c, const Layout& hl, size_t S, size_t N, const uint8_t* plan_dev,
                   const uint32_t* masks_host, int e, uint32_t* bad_host) {
  const int k = c->k, m = c->m;
  const size_t dbytes = (N - 1) * hl.data_sp + static_cast<size_t>(k - 1) * hl.pitch + S;
  const size_t pbytes = m ? (N - 1) * hl.parity_sp + static_cast<size_t>(m - 1) * hl.pitch + S : 0;
  uint8_t* dd = mapped(hl.data, dbytes);
  uint8_t* pd = m ? mapped(hl.parity, pbytes) : nullptr;
  if (!dd || (m && !pd)) return RS_ERR_NOT_SUPPORTED;
  const Layout dl{dd, hl.data_sp, pd, hl.parity_sp, hl.pitch};
  if (!device_layout_ok(dl, m, S)) return RS_ERR_NOT_SUPPORTED;
  std::lock_guard<std::mutex> g(c->host_mu);
  HostPipe& pipe = c->host_pipe;
  if (!pipe.st[0]) RS_HIP(hipStreamCreateWithFlags(&pipe.st[0], hipStreamNonBlocking));
  hipStream_t st = pipe.st[0];
  rs::KernelArgs a = make_args(c, dl, S, N);
  a.plans = plan_dev;
  int rc;
  if (bad_host) {
    if (c->d_bad.ensure(N * 4)) return RS_ERR_DEVICE;
    a.bad = static_cast<uint32_t*>(c->d_bad.p);
    rc = launch_verify_args(c, a, st);
    if (rc) return rc;
    RS_HIP(hipMemcpyAsync(bad_host, a.bad, N * 4, hipMemcpyDeviceToHost, st));
  } else {
    if (masks_host) {
      const uint32_t* dm = nullptr;
      rc = upload_masks(c, masks_host, N, st, &dm);
      if (rc) return rc;
      a.present_masks = dm;
    }
    rc = launch(c, a, e, masks_host != nullptr, st);
    if (rc) return rc;
  }
  RS_HIP(hipStreamSynchronize(st));
  c->last_host_path.store("zero-copy");
  return RS_OK;
}

int host_batch(rs_ctx* c, const Layout& hl, const std::vector<int>& in_slots, const std::vector<int>& out_slots,
               size_t S, size_t N, const uint8_t* plan_dev, const uint32_t* masks_host, int e,
               uint32_t* bad_host = nullptr) {
  if (c->host_zero_copy) {
    const int rc = host_zero_copy(c, hl, S, N, plan_dev, masks_host, e, bad_host);
    if (rc != RS_ERR_NOT_SUPPORTED) return rc;
  }
  c->last_host_path.store("staged");
  const int k = c->k, m = c->m;
  const size_t P = round_up(S, 256);  // 256-B slots: see batch.shard_pitch_for
  const size_t per_stripe = P * static_cast<size_t>(k + m) + ((masks_host || bad_host) ? 4 : 0);
  const size_t chunk = std::min(N, std::max<size_t>(1, kHostChunkBytes / per_stripe));
  std::lock_guard<std::mutex> g(c->host_mu);
  HostPipe& pipe = c->host_pipe;
  for (int i = 0; i < kHostStreams; ++i) {
    if (!pipe.st[i]) RS_HIP(hipStreamCreateWithFlags(&pipe.st[i], hipStreamNonBlocking));
    // sized for a full chunk whatever N is, so a small call never leaves slabs that
    // a later large call has to reallocate
    if (pipe.buf[i].ensure(std::max(kHostChunkBytes, per_stripe) + per_stripe + 256)) return RS_ERR_DEVICE;
  }
  int j = 0;
  for (size_t s0 = 0; s0 < N; s0 += chunk, ++j) {
    const size_t n = std::min(chunk, N - s0);
    hipStream_t st = pipe.st[j % kHostStreams];
    uint8_t* d = static_cast<uint8_t*>(pipe.buf[j % kHostStreams].p);
    const Layout dl{d, P * k, d + chunk * P * k, P * m, P};
    int rc = copy_slots(dl, hl, k, in_slots, 0, s0, n, S, hipMemcpyHostToDevice, st);
    if (rc) return rc;
    rs::KernelArgs a = make_args(c, dl, S, n);
    a.plans = plan_dev;
    if (masks_host) {
      uint32_t* dm = reinterpret_cast<uint32_t*>(d + round_up(chunk * P * (k + m), 256));
      RS_HIP(hipMemcpyAsync(dm, masks_host + s0, n * 4, hipMemcpyHostToDevice, st));
      a.present_masks = dm;
    }
    if (bad_host) {
      uint32_t* db = reinterpret_cast<uint32_t*>(d + round_up(chunk * P * (k + m), 256));
      a.bad = db;
      rc = launch_verify_args(c, a, st);
      if (rc) return rc;
      RS_HIP(hipMemcpyAsync(bad_host + s0, db, n * 4, hipMemcpyDeviceToHost, st));
      continue;
    }
    rc = launch(c, a, e, masks_host != nullptr, st);
    if (rc) return rc;
    rc = copy_slots(hl, dl, k, out_slots, s0, 0, n, S, hipMemcpyDeviceToHost, st);
    if (rc) return rc;
  }
  for (int i = 0; i < kHostStreams; ++i) RS_HIP(hipStreamSynchronize(pipe.st[i]));
  return RS_OK;
}

int upload_masks(rs_ctx* c, const uint32_t* masks, size_t n, hipStream_t s, const uint32_t** dev) {
  std::lock_guard<std::mutex> g(c->upload_mu);
  UploadSlot& u = c->uploads[c->upload_next++ % rs_ctx::kUploadSlots];
  if (!u.done) RS_HIP(hipEventCreateWithFlags(&u.done, hipEventDisableTiming));
  if (u.used) RS_HIP(hipEventSynchronize(u.done));
  if (u.host.ensure(n * 4) || u.dev.ensure(n * 4)) return RS_ERR_DEVICE;
  std::memcpy(u.host.p, masks, n * 4);
  RS_HIP(hipMemcpyAsync(u.dev.p, u.host.p, n * 4, hipMemcpyHostToDevice, s));
  RS_HIP(hipEventRecord(u.done, s));
  u.used = true;
  *dev = static_cast<const uint32_t*>(u.dev.p);
  return RS_OK;
}

}  // namespace

// =============================================================================
extern "C" {

const char* rs_strerror(int code) {
  switch (code) {
    case RS_OK: return "ok";
    case RS_ERR_INV_SHARD_NUM:
      return "cannot create Encoder with less than one data shard or less than zero parity shards";
    case RS_ERR_MAX_SHARD_NUM: return "cannot create Encoder with more than 256 data+parity shards";
    case RS_ERR_TOO_FEW_SHARDS: return "too few shards given";
    case RS_ERR_SHARD_NO_DATA: return "no shard data";
    case RS_ERR_SHARD_SIZE: return "shard sizes do not match";
    case RS_ERR_SHORT_DATA: return "not enough data to fill the number of requested shards";
    case RS_ERR_SINGULAR: return "matrix is singular";
    case RS_ERR_INVALID_ARG: return "rsgpu: invalid argument or layout";
    case RS_ERR_NO_DEVICE: return "rsgpu: no usable GPU device";
    case RS_ERR_DEVICE: return "rsgpu: HIP runtime error";
    case RS_ERR_NOT_SUPPORTED: return "operation not supported";
    default: return "rsgpu: unknown error";
  }
}

int rs_create(int k, int m, int device, int flags, rs_ctx** out) {
  (void)flags;
  if (!out) return RS_ERR_INVALID_ARG;
  *out = nullptr;
  // [upstream reedsolomon.go New] argument checks, same order and sentinels.
  if (k <= 0 || m < 0) return RS_ERR_INV_SHARD_NUM;
  if (k + m > 256) return RS_ERR_MAX_SHARD_NUM;
  if (k > rs::kMaxK || m > rs::kMaxM || k + m > 32) return RS_ERR_NOT_SUPPORTED;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return RS_ERR_NO_DEVICE;
  if (device < 0 || device >= ndev) return RS_ERR_NO_DEVICE;
  if (hipSetDevice(device) != hipSuccess) return RS_ERR_DEVICE;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) return RS_ERR_DEVICE;
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) return RS_ERR_NO_DEVICE;

  auto c = std::make_unique<rs_ctx>();
  c->k = k;
  c->m = m;
  c->device = device;
  c->cu_count = prop.multiProcessorCount;
  c->enc = rs::build_encode_matrix(k, m);
  if (const char* e = std::getenv("RSGPU_BLOCKS_PER_CU")) c->blocks_per_cu = std::max(1, std::atoi(e));
  if (const char* e = std::getenv("RSGPU_FORCE_GENERIC")) c->force_generic = std::atoi(e) != 0;
  if (const char* e = std::getenv("RSGPU_HOST_ZERO_COPY")) c->host_zero_copy = std::atoi(e) != 0;
  if (const uint8_t* rows = rs::bitsliced_encode_rows(k, m)) {
    bool same = true;
    for (int r = 0; r < m; ++r)
      for (int q = 0; q < k; ++q) same = same && rows[r * k + q] == c->enc.at(k + r, q);
    c->bitsliced = same;
  }
  if (const char* e = std::getenv("RSGPU_BITSLICED")) c->bitsliced = c->bitsliced && std::atoi(e) != 0;
  char name[160];
  std::snprintf(name, sizeof(name), "hip:%s:%s:%dCU", prop.gcnArchName, prop.name, c->cu_count);
  c->backend = name;

  // Encode plan: in = data slots 0..k-1, out = parity slots k..k+m-1.
  {
    std::vector<int> in_idx(k), out_idx(m);
    for (int i = 0; i < k; ++i) in_idx[i] = i;
    for (int p = 0; p < m; ++p) out_idx[p] = k + p;
    std::vector<uint8_t> rows(static_cast<size_t>(m) * k);
    for (int p = 0; p < m; ++p)
      for (int i = 0; i < k; ++i) rows[p * k + i] = c->enc.at(k + p, i);
    std::vector<uint8_t> p0 = make_plan(k, m, in_idx, out_idx, rows);
    if (c->d_enc_plan.ensure(p0.size())) return RS_ERR_DEVICE;
    if (hipMemcpy(c->d_enc_plan.p, p0.data(), p0.size(), hipMemcpyHostToDevice) != hipSuccess) return RS_ERR_DEVICE;
  }
  // Eager all-pattern plans + LUT for k+m <= 16.  Plan 0 = nothing missing.
  const int t = k + m;
  if (t <= 16 && m > 0) {
    const uint32_t full = (1u << t) - 1u;
    c->h_lut.assign(size_t(1) << t, rs::kPlanInvalid);
    std::vector<uint8_t> all;
    {
      std::vector<int> in_idx(k), none;
      for (int i = 0; i < k; ++i) in_idx[i] = i;
      std::vector<uint8_t> p = make_plan(k, m, in_idx, none, {});
      all.insert(all.end(), p.begin(), p.end());
      c->h_lut[0] = 0;
    }
    uint32_t count = 1;
    bool ok = true;
    for (uint32_t missing = 1; missing <= full && ok; ++missing) {
      if (__builtin_popcount(missing) > m) continue;
      std::vector<uint8_t> p;
      if (make_decode_plan(k, m, c->enc, full & ~missing, false, &p) != RS_OK) continue;
      if (all.size() + p.size() > (size_t(64) << 20)) {
        ok = false;
        break;
      }
      all.insert(all.end(), p.begin(), p.end());
      c->h_lut[missing] = count++;
    }
    if (ok) {
      if (c->d_plans.ensure(all.size()) || c->d_lut.ensure(c->h_lut.size() * 4)) return RS_ERR_DEVICE;
      if (hipMemcpy(c->d_plans.p, all.data(), all.size(), hipMemcpyHostToDevice) != hipSuccess ||
          hipMemcpy(c->d_lut.p, c->h_lut.data(), c->h_lut.size() * 4, hipMemcpyHostToDevice) != hipSuccess)
        return RS_ERR_DEVICE;
      c->n_plans = count;
      c->have_lut = true;
    }
  }
  if (c->d_status.ensure(256) || c->h_status.ensure(256) || c->d_scratch.ensure(256 * 1024)) return RS_ERR_DEVICE;
  if (hipMemset(c->d_status.p, 0, 256) != hipSuccess) return RS_ERR_DEVICE;
  *out = c.release();
  return RS_OK;
}

void rs_destroy(rs_ctx* ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->device);
  (void)hipDeviceSynchronize();
  delete ctx;
}

int rs_data_shards(const rs_ctx* c) { return c ? c->k : 0; }
int rs_parity_shards(const rs_ctx* c) { return c ? c->m : 0; }
int rs_device(const rs_ctx* c) { return c ? c->device : -1; }
const char* rs_backend(const rs_ctx* c) { return c ? c->backend.c_str() : "none"; }
const char* rs_last_kernel(const rs_ctx* c) { return c ? c->last_kernel.load() : "none"; }

int rs_encode_matrix(const rs_ctx* c, uint8_t* out) {
  if (!c || !out) return RS_ERR_INVALID_ARG;
  std::memcpy(out, c->enc.a.data(), c->enc.a.size());
  return RS_OK;
}

size_t rs_shard_size(const rs_ctx* c, size_t len) {
  if (!c || len == 0) return 0;
  return (len + static_cast<size_t>(c->k) - 1) / static_cast<size_t>(c->k);
}

int rs_encode(rs_ctx* c, uint8_t* const* shards, const size_t* lens) {
  if (!c || !shards || !lens) return RS_ERR_INVALID_ARG;
  size_t S = 0;
  int rc = check_shards(c->k + c->m, lens, false, &S);
  if (rc) return rc;
  if (c->m == 0) return RS_OK;
  for (int i = 0; i < c->k + c->m; ++i)
    if (!shards[i]) return RS_ERR_INVALID_ARG;
  std::vector<int> in_idx(c->k), out_idx(c->m);
  for (int i = 0; i < c->k; ++i) in_idx[i] = i;
  for (int p = 0; p < c->m; ++p) out_idx[p] = c->k + p;
  return run_object(c, static_cast<const uint8_t*>(c->d_enc_plan.p), in_idx, out_idx, shards, S);
}

int rs_reconstruct(rs_ctx* c, uint8_t* const* shards, size_t* lens) { return reconstruct_impl(c, shards, lens, false); }
int rs_reconstruct_data(rs_ctx* c, uint8_t* const* shards, size_t* lens) {
  return reconstruct_impl(c, shards, lens, true);
}

// [upstream reedsolomon.go Verify]: recompute parity on the GPU into scratch and
// compare on the host against the caller's parity shards.
int rs_verify(rs_ctx* c, uint8_t* const* shards, const size_t* lens, int* ok) {
  if (!c || !shards || !lens || !ok) return RS_ERR_INVALID_ARG;
  size_t S = 0;
  int rc = check_shards(c->k + c->m, lens, false, &S);
  if (rc) return rc;
  *ok = 1;
  if (c->m == 0) return RS_OK;
  std::vector<std::vector<uint8_t>> tmp(c->m, std::vector<uint8_t>(S));
  std::vector<uint8_t*> view(shards, shards + c->k + c->m);
  for (int p = 0; p < c->m; ++p) view[c->k + p] = tmp[p].data();
  std::vector<int> in_idx(c->k), out_idx(c->m);
  for (int i = 0; i < c->k; ++i) in_idx[i] = i;
  for (int p = 0; p < c->m; ++p) out_idx[p] = c->k + p;
  rc = run_object(c, static_cast<const uint8_t*>(c->d_enc_plan.p), in_idx, out_idx, view.data(), S);
  if (rc) return rc;
  for (int p = 0; p < c->m; ++p)
    if (std::memcmp(tmp[p].data(), shards[c->k + p], S) != 0) *ok = 0;
  return RS_OK;
}

int rs_encode_batch(rs_ctx* c, const uint8_t* data, size_t data_sp, uint8_t* parity, size_t parity_sp,
                    size_t shard_pitch, size_t S, size_t N, int mem, void* stream) {
  if (!c || !data || !parity) return RS_ERR_INVALID_ARG;
  if (N == 0) return RS_OK;
  if (S == 0) return RS_ERR_SHARD_NO_DATA;
  if (!batch_sizes_ok(S, N, shard_pitch)) return RS_ERR_INVALID_ARG;
  if (c->m == 0) return RS_OK;
  (void)hipSetDevice(c->device);
  const Layout L{const_cast<uint8_t*>(data), data_sp, parity, parity_sp, shard_pitch};
  const uint8_t* plan = static_cast<const uint8_t*>(c->d_enc_plan.p);
  if (mem == RS_MEM_DEVICE) {
    if (!device_layout_ok(L, c->m, S)) return RS_ERR_INVALID_ARG;
    rs::KernelArgs a = make_args(c, L, S, N);
    a.plans = plan;
    return launch(c, a, c->m, false, as_stream(stream));
  }
  if (mem != RS_MEM_HOST) return RS_ERR_INVALID_ARG;
  std::vector<int> in_slots(c->k), out_slots(c->m);
  for (int i = 0; i < c->k; ++i) in_slots[i] = i;
  for (int p = 0; p < c->m; ++p) out_slots[p] = c->k + p;
  return host_batch(c, L, in_slots, out_slots, S, N, plan, nullptr, c->m);
}

int rs_reconstruct_batch(rs_ctx* c, uint8_t* data, size_t data_sp, uint8_t* parity, size_t parity_sp,
                         size_t shard_pitch, size_t S, size_t N, const uint32_t* masks, size_t n_masks, int mem,
                         void* stream) {
  if (!c || !data || (c->m > 0 && !parity) || !masks) return RS_ERR_INVALID_ARG;
  if (N == 0) return RS_OK;
  if (S == 0) return RS_ERR_SHARD_NO_DATA;
  if (!batch_sizes_ok(S, N, shard_pitch)) return RS_ERR_INVALID_ARG;
  if (n_masks != 1 && n_masks != N) return RS_ERR_INVALID_ARG;
  const int t = c->k + c->m;
  const uint32_t full = static_cast<uint32_t>(full_mask64(t));
  int max_missing = 0;
  for (size_t i = 0; i < n_masks; ++i) {
    const int np = __builtin_popcount(masks[i] & full);
    if (np < c->k) return RS_ERR_TOO_FEW_SHARDS;
    max_missing = std::max(max_missing, t - np);
  }
  if (max_missing == 0) return RS_OK;
  if (mem != RS_MEM_DEVICE && mem != RS_MEM_HOST) return RS_ERR_INVALID_ARG;
  const Layout L{data, data_sp, parity, parity_sp, shard_pitch};
  if (mem == RS_MEM_DEVICE && !device_layout_ok(L, c->m, S)) return RS_ERR_INVALID_ARG;
  (void)hipSetDevice(c->device);
  if (n_masks == 1) {
    const uint32_t present = masks[0] & full;
    const uint8_t* plan = nullptr;
    int rc = uniform_plan(c, present, false, &plan);
    if (rc) return rc;
    if (mem == RS_MEM_DEVICE) {
      rs::KernelArgs a = make_args(c, L, S, N);
      a.plans = plan;
      return launch(c, a, max_missing, false, as_stream(stream));
    }
    std::vector<int> in_slots, out_slots;
    for (int i = 0; i < t; ++i) {
      if ((present >> i) & 1u) {
        if (static_cast<int>(in_slots.size()) < c->k) in_slots.push_back(i);
      } else {
        out_slots.push_back(i);
      }
    }
    return host_batch(c, L, in_slots, out_slots, S, N, plan, nullptr, max_missing);
  }
  if (!c->have_lut) return RS_ERR_NOT_SUPPORTED;
  if (mem == RS_MEM_DEVICE) {
    hipStream_t s = as_stream(stream);
    const uint32_t* dm = nullptr;
    int rc = upload_masks(c, masks, N, s, &dm);
    if (rc) return rc;
    rs::KernelArgs a = make_args(c, L, S, N);
    a.plans = static_cast<const uint8_t*>(c->d_plans.p);
    a.present_masks = dm;
    return launch(c, a, max_missing, true, s);
  }
  // host, per-stripe patterns: every slot travels both ways (present slots come back
  // unchanged); selective copies per pattern are a later optimisation.
  std::vector<int> all(t);
  for (int i = 0; i < t; ++i) all[i] = i;
  return host_batch(c, L, all, all, S, N, static_cast<const uint8_t*>(c->d_plans.p), masks, max_missing);
}

int rs_reconstruct_batch_out(rs_ctx* c, const uint8_t* data, size_t data_sp, const uint8_t* parity, size_t parity_sp,
                             size_t shard_pitch, size_t S, size_t N, const uint32_t* masks, size_t n_masks,
                             int masks_on_device, uint8_t* out, size_t out_sp, void* stream) {
  if (!c || !data || (c->m > 0 && !parity) || !masks || !out) return RS_ERR_INVALID_ARG;
  if (N == 0) return RS_OK;
  if (S == 0) return RS_ERR_SHARD_NO_DATA;
  if (!batch_sizes_ok(S, N, shard_pitch)) return RS_ERR_INVALID_ARG;
  const Layout L{const_cast<uint8_t*>(data), data_sp, const_cast<uint8_t*>(parity), parity_sp, shard_pitch};
  if (!device_layout_ok(L, c->m, S) || reinterpret_cast<uintptr_t>(out) % 16 || out_sp % 16) return RS_ERR_INVALID_ARG;
  const int t = c->k + c->m;
  const uint32_t full = static_cast<uint32_t>(full_mask64(t));
  (void)hipSetDevice(c->device);
  hipStream_t s = as_stream(stream);
  rs::KernelArgs a = make_args(c, L, S, N);
  a.out = out;
  a.out_sp = out_sp;
  if (masks_on_device) {
    if (!c->have_lut) return RS_ERR_NOT_SUPPORTED;
    if (!out_layout_ok(out_sp, shard_pitch, S, N, c->m)) return RS_ERR_INVALID_ARG;
    a.plans = static_cast<const uint8_t*>(c->d_plans.p);
    a.present_masks = masks;
    return launch(c, a, c->m, true, s);
  }
  if (n_masks != 1 && n_masks != N) return RS_ERR_INVALID_ARG;
  int max_missing = 0;
  for (size_t i = 0; i < n_masks; ++i) {
    const int np = __builtin_popcount(masks[i] & full);
    if (np < c->k) return RS_ERR_TOO_FEW_SHARDS;
    max_missing = std::max(max_missing, t - np);
  }
  if (max_missing == 0) return RS_OK;
  if (!out_layout_ok(out_sp, shard_pitch, S, N, max_missing)) return RS_ERR_INVALID_ARG;
  if (n_masks == 1) {
    const uint8_t* plan = nullptr;
    int rc = uniform_plan(c, masks[0] & full, false, &plan);
    if (rc) return rc;
    a.plans = plan;
    return launch(c, a, max_missing, false, s);
  }
  if (!c->have_lut) return RS_ERR_NOT_SUPPORTED;
  const uint32_t* dm = nullptr;
  int rc = upload_masks(c, masks, N, s, &dm);
  if (rc) return rc;
  a.plans = static_cast<const uint8_t*>(c->d_plans.p);
  a.present_masks = dm;
  return launch(c, a, max_missing, true, s);
}

int rs_verify_batch(rs_ctx* c, const uint8_t* data, size_t data_sp, const uint8_t* parity, size_t parity_sp,
                    size_t shard_pitch, size_t S, size_t N, uint32_t* bad, int mem, void* stream) {
  if (!c || !data || (c->m > 0 && !parity) || !bad) return RS_ERR_INVALID_ARG;
  if (N == 0) return RS_OK;
  if (S == 0) return RS_ERR_SHARD_NO_DATA;
  if (!batch_sizes_ok(S, N, shard_pitch) || reinterpret_cast<uintptr_t>(bad) % 4) return RS_ERR_INVALID_ARG;
  if (mem != RS_MEM_DEVICE && mem != RS_MEM_HOST) return RS_ERR_INVALID_ARG;
  (void)hipSetDevice(c->device);
  if (c->m == 0) {  // nothing to verify
    if (mem == RS_MEM_HOST) {
      std::memset(bad, 0, N * 4);
      return RS_OK;
    }
    RS_HIP(hipMemsetAsync(bad, 0, N * 4, as_stream(stream)));
    return RS_OK;
  }
  const Layout L{const_cast<uint8_t*>(data), data_sp, const_cast<uint8_t*>(parity), parity_sp, shard_pitch};
  if (mem == RS_MEM_DEVICE) {
    if (!device_layout_ok(L, c->m, S)) return RS_ERR_INVALID_ARG;
    rs::KernelArgs a = make_args(c, L, S, N);
    a.bad = bad;
    return launch_verify_args(c, a, as_stream(stream));
  }
  std::vector<int> all(c->k + c->m), none;
  for (int i = 0; i < c->k + c->m; ++i) all[i] = i;
  return host_batch(c, L, all, none, S, N, nullptr, nullptr, c->m, bad);
}

int rs_reconstruct_batch_devmask(rs_ctx* c, uint8_t* data, size_t data_sp, uint8_t* parity, size_t parity_sp,
                                 size_t shard_pitch, size_t S, size_t N, const uint32_t* masks_dev, void* stream) {
  if (!c || !data || (c->m > 0 && !parity) || !masks_dev) return RS_ERR_INVALID_ARG;
  if (N == 0) return RS_OK;
  if (S == 0) return RS_ERR_SHARD_NO_DATA;
  if (!c->have_lut) return RS_ERR_NOT_SUPPORTED;
  const Layout L{data, data_sp, parity, parity_sp, shard_pitch};
  if (!batch_sizes_ok(S, N, shard_pitch) || !device_layout_ok(L, c->m, S)) return RS_ERR_INVALID_ARG;
  (void)hipSetDevice(c->device);
  rs::KernelArgs a = make_args(c, L, S, N);
  a.plans = static_cast<const uint8_t*>(c->d_plans.p);
  a.present_masks = masks_dev;
  return launch(c, a, c->m, true, as_stream(stream));
}

int rs_sync(rs_ctx* c, void* stream) {
  if (!c) return RS_ERR_INVALID_ARG;
  (void)hipSetDevice(c->device);
  hipStream_t s = as_stream(stream);
  RS_HIP(hipMemcpyAsync(c->h_status.p, c->d_status.p, 4, hipMemcpyDeviceToHost, s));
  RS_HIP(hipStreamSynchronize(s));
  const uint32_t st = *static_cast<uint32_t*>(c->h_status.p);
  if (st) {
    RS_HIP(hipMemsetAsync(c->d_status.p, 0, 4, s));
    RS_HIP(hipStreamSynchronize(s));
    return RS_ERR_TOO_FEW_SHARDS;
  }
  return RS_OK;
}

int rs_host_register(rs_ctx* c, void* ptr, size_t bytes) {
  if (!c || !ptr) return RS_ERR_INVALID_ARG;
  (void)hipSetDevice(c->device);
  RS_HIP(hipHostRegister(ptr, bytes, hipHostRegisterDefault));
  return RS_OK;
}

int rs_host_unregister(rs_ctx* c, void* ptr) {
  if (!c || !ptr) return RS_ERR_INVALID_ARG;
  (void)hipSetDevice(c->device);
  RS_HIP(hipHostUnregister(ptr));
  return RS_OK;
}

int rs_device_copy(rs_ctx* c, void* dst, const void* src, size_t bytes, void* stream) {
  if (!c || !dst || !src || bytes % 16 || reinterpret_cast<uintptr_t>(dst) % 16 ||
      reinterpret_cast<uintptr_t>(src) % 16)
    return RS_ERR_INVALID_ARG;
  (void)hipSetDevice(c->device);
  const uint32_t grid = static_cast<uint32_t>(
      std::max<uint64_t>(1, std::min<uint64_t>(static_cast<uint64_t>(c->cu_count) * 2, (bytes / 16 + 1023) / 1024)));
  rs::launch_copy(src, dst, bytes, grid, as_stream(stream));
  c->last_kernel.store("copy_kernel");
  RS_HIP(hipGetLastError());
  return RS_OK;
}

// Batched SHA-256 (the reference's cold_hash, writeservice.go:51-54): device-resident
// messages, asynchronous on `stream`.
int rs_sha256_batch(rs_ctx* c, const uint8_t* base, size_t stride, size_t len, size_t n, uint8_t* digests,
                    void* stream) {
  if (!c || (n && (!base || !digests)) || n > 0xFFFFFFFFu || (n > 1 && stride < len) ||
      reinterpret_cast<uintptr_t>(digests) % 4)
    return RS_ERR_INVALID_ARG;
  if (n == 0) return RS_OK;
  (void)hipSetDevice(c->device);
  const rs::Sha256Args a{base, stride, nullptr, nullptr, len, static_cast<uint32_t>(n), digests};
  if (rs::launch_sha256(a, as_stream(stream))) return RS_ERR_DEVICE;
  c->last_kernel.store("sha256_kernel");
  return RS_OK;
}

int rs_sha256_batch_var(rs_ctx* c, const uint8_t* base, const uint64_t* offsets, const uint64_t* lens, size_t n,
                        uint8_t* digests, void* stream) {
  if (!c || (n && (!base || !offsets || !lens || !digests)) || n > 0xFFFFFFFFu ||
      reinterpret_cast<uintptr_t>(digests) % 4)
    return RS_ERR_INVALID_ARG;
  if (n == 0) return RS_OK;
  (void)hipSetDevice(c->device);
  const rs::Sha256Args a{base, 0, offsets, lens, 0, static_cast<uint32_t>(n), digests};
  if (rs::launch_sha256(a, as_stream(stream))) return RS_ERR_DEVICE;
  c->last_kernel.store("sha256_kernel");
  return RS_OK;
}

int rs_set_host_zero_copy(rs_ctx* c, int enable) {
  if (!c) return RS_ERR_INVALID_ARG;
  c->host_zero_copy = enable != 0;
  return RS_OK;
}

const char* rs_last_host_path(const rs_ctx* c) { return c ? c->last_host_path.load() : "none"; }

int rs_set_blocks_per_cu(rs_ctx* c, int bpc) {
  if (!c || bpc < 0) return RS_ERR_INVALID_ARG;
  c->blocks_per_cu = bpc;  // 0 = by shape
  return RS_OK;
}

}  // extern "C"
