// rs_engine.cpp -- librsgpu.so: the C-ABI in include/rsgpu.h.
//
// Host runtime around the gfx950 kernels in rs_kernels.hip:
//   * encode matrix and per-erasure-pattern decode plans (the analogue of
//     klauspost's inversion_tree.go cache, [upstream reedsolomon.go reconstruct]),
//     built once per pattern and kept resident in HBM;
//   * for k+m <= 16 every pattern with 1..m erasures is precomputed at creation and
//     indexed by a dense missing-mask -> plan LUT, so a batch may carry a different
//     erasure pattern per stripe with no host work per stripe;
//   * one context spans one or several GPUs (one Engine each): per-object calls go
//     to the least-busy engine, host-resident batches split into contiguous stripe
//     ranges across the engines (independent objects, no
//     collective), device-resident batches run on the engine of the caller's
//     stream;
//   * per-object host calls (the IEcDriver drop-in: ec.go:54-61) run on a pool of
//     "lanes" (stream + pinned staging + device slab) per engine so concurrent
//     goroutines do not serialise on one stream;
//   * host-resident batches run zero-copy (kernel reads / writes pinned host memory
//     in place) or pipelined H2D -> kernel -> D2H over 4 streams.
// No CPU arithmetic path exists: every parity / reconstructed byte comes from a
// HIP kernel.
#include "rs_engine.hpp"

#include <hip/hip_runtime.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cctype>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <fstream>
#include <functional>
#include <memory>
#include <mutex>
#include <shared_mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/rsgpu.h"
#include "gf256.hpp"
#include "rs_host_util.hpp"
#include "rs_plan.hpp"
#include "rs_sha256.hpp"

// ---- pinned host memory ------------------------------------------------------------
namespace rs {

int device_numa_node(int device) {
  char bus[64] = {0};
  if (hipDeviceGetPCIBusId(bus, sizeof(bus), device) != hipSuccess) {
    (void)hipGetLastError();
    return -1;
  }
  std::string id(bus);
  for (char& ch : id) ch = static_cast<char>(std::tolower(static_cast<unsigned char>(ch)));
  std::ifstream f("/sys/bus/pci/devices/" + id + "/numa_node");
  int node = -1;
  if (!(f >> node)) return -1;
  return node;
}

void* pinned_alloc(size_t bytes, int node) {
  // Place the pages on `node`: the allocating thread's memory policy is set to
  // prefer that node around the allocation and hipHostMallocNumaUser makes the HIP
  // runtime follow it; restored afterwards.
  constexpr unsigned long kMaxNode = 1024;
  unsigned long saved[kMaxNode / 64] = {0};
  int saved_mode = 0;
  bool policy_set = false;
  unsigned flags = hipHostMallocPortable;  // one staging slab may serve any GPU
  if (node >= 0 && node < static_cast<int>(kMaxNode) &&
      syscall(SYS_get_mempolicy, &saved_mode, saved, kMaxNode, nullptr, 0) == 0) {
    unsigned long want[kMaxNode / 64] = {0};
    want[node / 64] = 1ul << (node % 64);
    if (syscall(SYS_set_mempolicy, 1 /* MPOL_PREFERRED */, want, kMaxNode) == 0) {
      policy_set = true;
      flags |= hipHostMallocNumaUser;
    }
  }
  void* p = nullptr;
  hipError_t err = hipHostMalloc(&p, bytes, flags);
  if (err != hipSuccess && policy_set) {  // runtime without NUMA-user support: plain pinned
    (void)hipGetLastError();
    err = hipHostMalloc(&p, bytes, hipHostMallocPortable);
  }
  if (policy_set) syscall(SYS_set_mempolicy, saved_mode, saved_mode ? saved : nullptr, kMaxNode);
  if (err != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  return p;
}

void pinned_free(void* p) {
  if (p) (void)hipHostFree(p);
}

}  // namespace rs

namespace {

using rs::check_shards;
using rs::DevBuf;
using rs::DeviceScope;
using rs::Matrix;
using rs::PinnedBuf;
using rs::round_up;

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

// rows: n_out x k coefficient matrix (row-major); in_idx = the first k shards of
// `present`, out_idx = the shards of `out_mask` missing from it (both in index order:
// the kernels re-derive them from the masks).
std::vector<uint8_t> make_plan(int k, int m, uint32_t present, uint32_t out_mask, const std::vector<int>& in_idx,
                               const std::vector<int>& out_idx, const std::vector<uint8_t>& rows) {
  std::vector<uint8_t> p(rs::plan_stride(k, m), 0);
  const uint32_t hdr[4] = {static_cast<uint32_t>(out_idx.size()), present, out_mask, 0u};
  std::memcpy(p.data(), hdr, sizeof(hdr));
  uint32_t* ii = reinterpret_cast<uint32_t*>(p.data() + 16);
  for (int c = 0; c < k; ++c) ii[c] = static_cast<uint32_t>(in_idx[c]);
  for (size_t r = 0; r < out_idx.size(); ++r) ii[k + r] = static_cast<uint32_t>(out_idx[r]);
  uint8_t* coef = p.data() + rs::plan_coef_offset(k, m);
  for (size_t r = 0; r < out_idx.size(); ++r)
    for (int c = 0; c < k; ++c) coef[r * rs::plan_coef_row(k) + c] = rows[r * k + c];
  uint32_t* tab = reinterpret_cast<uint32_t*>(p.data() + rs::plan_tab_offset(k, m));
  for (size_t r = 0; r < out_idx.size(); ++r)
    for (int c = 0; c < k; ++c) perm_tables(rows[r * k + c], tab + (c * m + r) * 5);
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
  const uint32_t full = static_cast<uint32_t>((t >= 32) ? ~0ull : ((1ull << t) - 1));
  const uint32_t data = static_cast<uint32_t>((1ull << k) - 1);
  *out = make_plan(k, m, static_cast<uint32_t>(present) & full, data_only ? data : full, surv, miss, rows);
  return RS_OK;
}

uint64_t full_mask64(int t) { return (t >= 64) ? ~0ull : ((1ull << t) - 1); }

// ---- buffers -------------------------------------------------------------------
// A lane serves one synchronous host call at a time.
struct Lane {
  hipStream_t stream = nullptr;
  DevBuf dev;
  PinnedBuf host;
};

// Staging for per-stripe masks passed in host memory to an asynchronous device
// call.  A slot is reused only after the kernel that READ it has finished: `done`
// is recorded on the launch stream after that kernel (~UploadGuard), and `busy`
// keeps a second caller off the slot between its upload and its launch.
struct UploadSlot {
  PinnedBuf host;
  void* host_dev = nullptr;  // GPU address of host (a portable mapping)
  DevBuf dev;
  hipEvent_t done = nullptr;
  bool used = false;
  bool busy = false;
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
  // the same layout starting at stripe s0
  Layout from(size_t s0) const {
    return Layout{data + s0 * data_sp, data_sp, parity ? parity + s0 * parity_sp : nullptr, parity_sp, pitch};
  }
};

// Host batch pipeline: chunks of stripes flow H2D -> kernel -> D2H on kHostStreams
// streams; each stream has its own device slab (split layout), so chunk j+1's
// copies overlap chunk j's kernel and D2H.  Kept in the engine: creating streams
// and slabs per call cost more than a small call's transfers.
constexpr int kHostStreams = 4;
constexpr size_t kHostChunkBytes = size_t(16) << 20;  // device bytes per chunk
constexpr size_t kUploadSlots = 8;
constexpr uint32_t kStatusChunk = 1024;  // per-stream deferred-error words per allocation
constexpr uint32_t kStatusChunks = 4096;  // at most 4 M streams with words at once per engine

// Device words the per-stripe kernels OR their errors into, and the pinned words
// rs_sync reads them back through.  Chunks are never freed before the engine, so a
// word's address stays valid for the kernels that hold it.
struct StatusChunk {
  DevBuf dev;
  PinnedBuf host;
};

// "What ran last" (measurement and fault diagnostics): context-wide, and per launch
// stream -- a device fault surfaces asynchronously, and only the stream's own record
// names the launch that preceded it when other threads launch on the context too.
// The per-stream record is sharded by stream handle (one
// context-wide mutex on every launch made concurrent launchers queue on it); a
// shard's entry stays until rs_stream_release(stream) forgets it.
struct Shared {
  static constexpr size_t kShards = 64;
  struct Shard {
    std::mutex mu;
    std::unordered_map<hipStream_t, const char*> by_stream;
  };
  std::atomic<const char*> last_kernel{"none"};
  std::atomic<const char*> last_host_path{"none"};
  Shard shards[kShards];
  Shard& shard(hipStream_t s) { return shards[(reinterpret_cast<uintptr_t>(s) >> 4) % kShards]; }
  void note(hipStream_t s, const char* name) {
    last_kernel.store(name, std::memory_order_relaxed);
    Shard& sh = shard(s);
    std::lock_guard<std::mutex> g(sh.mu);
    sh.by_stream[s] = name;
  }
  const char* on(hipStream_t s) {
    Shard& sh = shard(s);
    std::lock_guard<std::mutex> g(sh.mu);
    auto it = sh.by_stream.find(s);
    return it == sh.by_stream.end() ? "none" : it->second;
  }
  void forget(hipStream_t s) {
    Shard& sh = shard(s);
    std::lock_guard<std::mutex> g(sh.mu);
    sh.by_stream.erase(s);
  }
};

}  // namespace

// ---- one GPU ----------------------------------------------------------------------
namespace rs {

struct Engine {
  int k = 0, m = 0, device = 0, cu_count = 0, numa = -1;
  rs_ctx* ctx = nullptr;                  // owner (its rs_host_alloc'ed ranges)
  const Matrix* enc = nullptr;            // the context's
  const std::vector<uint32_t>* h_lut = nullptr;
  Shared* shared = nullptr;
  int blocks_per_cu = 0;                  // 0 = by shape
  int occ_cap = -1;                       // waves per SIMD: -1 = each kernel's tuned default
  bool bitsliced = false;                 // generated encode XOR program matches enc
  bool host_zero_copy = true;             // pinned host batches: kernel reads/writes in place
  bool parity_pad = false;                // encode may write parity padding to the next 128-B line
  bool out_pad = false;                   // out-of-place rows end on whole lines (rs_set_out_pad_writes)
  std::string name;

  DevBuf d_enc_plan;                      // encode plan (uniform)
  DevBuf d_plans, d_lut;                  // eager all-pattern plans + LUT (k+m <= 16)
  bool have_lut = false;
  std::mutex plan_mu;                     // uniform plans built on demand (k+m > 16 / data-only)
  std::unordered_map<uint64_t, std::unique_ptr<DevBuf>> plan_cache;

  // Deferred per-stripe errors (device-resident masks): one word per stream, so
  // rs_sync(stream) reports and clears exactly the errors of kernels on that stream.
  // rs_stream_release(stream) returns the stream's word to status_free.
  std::mutex status_mu;
  std::unordered_map<hipStream_t, uint32_t> status_idx;
  std::vector<uint32_t> status_free;
  std::unique_ptr<StatusChunk> status_chunks[kStatusChunks];  // fixed slots: read without the mutex
  uint32_t status_next = 0;  // words handed out from the chunks so far

  std::mutex lane_mu;
  std::condition_variable lane_cv;
  std::vector<std::unique_ptr<Lane>> lanes;
  std::vector<Lane*> free_lanes;
  int max_lanes = 8;

  std::mutex upload_mu;
  std::condition_variable upload_cv;
  UploadSlot uploads[kUploadSlots];
  size_t upload_next = 0;

  std::mutex host_mu;                     // host-resident batches: one at a time per engine
  hipStream_t pipe_st[kHostStreams] = {};
  DevBuf pipe_buf[kHostStreams];
  // staged per-stripe reconstruct: a ring of pinned D2H buffers of dense output rows
  // and the events that say when each holds its chunk (host_batch_ps)
  PinnedBuf scatter_host[2 * kHostStreams];
  hipEvent_t scatter_ev[2 * kHostStreams] = {};
  // ... and per pipeline stream the parity survivors gathered on the host, which
  // the kernel reads in place over PCIe (GPU address par_dev)
  PinnedBuf par_host[kHostStreams];
  uint8_t* par_dev[kHostStreams] = {};
  DevBuf d_bad;                           // zero-copy verify: per-stripe result before D2H

  std::atomic<int> inflight{0};           // calls running on this engine (dispatch)
  std::atomic<uint64_t> launches{0};      // codec kernels launched here (rs_device_launches)

  // One persistent host thread per engine runs its share of a multi-GPU host batch
  // (fan_out), started on first use.
  std::mutex work_mu;
  std::condition_variable work_cv;
  std::deque<std::function<void()>> work;
  std::thread worker;
  bool work_stop = false;

  // Queues fn on this engine's worker; false if the thread cannot be started.
  bool post(std::function<void()> fn) {
    std::lock_guard<std::mutex> g(work_mu);
    if (!worker.joinable()) {
      try {
        worker = std::thread([this] {
          std::unique_lock<std::mutex> lk(work_mu);
          for (;;) {
            work_cv.wait(lk, [this] { return work_stop || !work.empty(); });
            if (work.empty()) return;  // stopping, nothing queued
            std::function<void()> f = std::move(work.front());
            work.pop_front();
            lk.unlock();
            f();
            lk.lock();
          }
        });
      } catch (...) {
        return false;
      }
    }
    work.push_back(std::move(fn));
    work_cv.notify_one();
    return true;
  }

  ~Engine() {  // runs under the rs_ctx destructor's DeviceScope
    {
      std::lock_guard<std::mutex> g(work_mu);
      work_stop = true;
      work_cv.notify_all();
    }
    if (worker.joinable()) worker.join();
    (void)hipDeviceSynchronize();
    for (auto& s : uploads)
      if (s.done) (void)hipEventDestroy(s.done);
    for (auto& l : lanes)
      if (l->stream) (void)hipStreamDestroy(l->stream);
    for (auto& s : pipe_st)
      if (s) (void)hipStreamDestroy(s);
    for (auto& ev : scatter_ev)
      if (ev) (void)hipEventDestroy(ev);
  }
};

}  // namespace rs

using rs::Engine;

// A host range the context knows: rs_host_alloc'ed (owned: page-locked by the
// driver, GPU-mapped, eligible for in-place kernels) or rs_host_register'ed (caller
// memory: recorded only, never mapped into a GPU, always staged).
struct RegRange {
  uintptr_t lo = 0, hi = 0;  // [lo, hi)
  uint8_t* dev = nullptr;     // owned: GPU address of lo (portable mapping: every device)
  bool owned = false;         // rs_host_alloc'ed (freed by rs_host_free / rs_destroy)
};

struct rs_ctx {
  int k = 0, m = 0;
  Matrix enc;
  // known host ranges, sorted by lo, never overlapping (kernels address buffers that
  // lie inside an owned one in place instead of staging them)
  std::shared_mutex reg_mu;
  std::vector<RegRange> reg;
  std::atomic<uint32_t> n_owned{0};
  std::vector<uint32_t> h_lut;            // missing mask -> plan index (k+m <= 16)
  std::vector<std::unique_ptr<Engine>> engines;
  Shared shared;
  std::string backend;
  std::atomic<uint32_t> rr{0};
  ~rs_ctx() {
    for (auto& e : engines) {  // each engine's buffers and streams freed on its device
      DeviceScope ds(e->device);
      e.reset();
    }
  }
};

namespace {

struct InflightGuard {
  Engine* e;
  explicit InflightGuard(Engine* en) : e(en) { e->inflight.fetch_add(1, std::memory_order_relaxed); }
  ~InflightGuard() { e->inflight.fetch_sub(1, std::memory_order_relaxed); }
};

// Least-busy engine for a per-object call (round-robin among equals).
Engine* pick_engine(rs_ctx* c) {
  const size_t n = c->engines.size();
  if (n == 1) return c->engines[0].get();
  const uint32_t start = c->rr.fetch_add(1, std::memory_order_relaxed);
  Engine* best = nullptr;
  int best_load = 0;
  for (size_t i = 0; i < n; ++i) {
    Engine* e = c->engines[(start + i) % n].get();
    const int load = e->inflight.load(std::memory_order_relaxed);
    if (!best || load < best_load) {
      best = e;
      best_load = load;
    }
  }
  return best;
}

// Engine of a device-resident call: the device the caller's stream belongs to
// (the current device for the null stream).  Always the FIRST engine on that
// device, so the stream's deferred errors are found by rs_sync.  nullptr if the
// context does not span that device.
Engine* engine_for_stream(rs_ctx* c, hipStream_t s) {
  if (c->engines.size() == 1) return c->engines[0].get();
  int dev = -1;
  if (s) {
    if (hipStreamGetDevice(s, &dev) != hipSuccess) {
      (void)hipGetLastError();
      return nullptr;
    }
  } else if (hipGetDevice(&dev) != hipSuccess) {
    return nullptr;
  }
  for (auto& e : c->engines)
    if (e->device == dev) return e.get();
  return nullptr;
}

// Runs fn(engine, first_stripe, n_stripes) over contiguous near-equal stripe
// ranges, one per engine, in parallel: range 0 on the calling
// thread, the others on the engines' persistent worker threads.  Small batches stay
// on one engine: a share below ~8 MiB of user data is not worth a second device's
// launch.  Never throws (a range whose worker cannot run is run inline).
template <class Fn>
int fan_out(rs_ctx* c, size_t N, size_t user_bytes_per_stripe, Fn&& fn) {
  const size_t ne = c->engines.size();
  size_t use = 1;
  if (ne > 1) {
    const size_t want = N * user_bytes_per_stripe / (size_t(8) << 20);
    use = std::max<size_t>(1, std::min({ne, want, N}));
  }
  if (use == 1) {
    Engine* e = pick_engine(c);
    InflightGuard ig(e);
    DeviceScope ds(e->device);
    if (!ds.ok()) return RS_ERR_DEVICE;
    return fn(e, size_t(0), N);
  }
  const uint32_t start = c->rr.fetch_add(1, std::memory_order_relaxed);
  std::vector<int> rcs(use, RS_OK);
  auto run = [&](size_t j) {
    Engine* e = c->engines[(start + j) % ne].get();
    InflightGuard ig(e);
    DeviceScope ds(e->device);
    if (!ds.ok()) {
      rcs[j] = RS_ERR_DEVICE;
      return;
    }
    const size_t base = N / use, extra = N % use;
    const size_t s0 = j * base + std::min(j, extra);
    try {
      rcs[j] = fn(e, s0, base + (j < extra ? 1 : 0));
    } catch (...) {
      rcs[j] = RS_ERR_DEVICE;
    }
  };
  std::mutex mu;
  std::condition_variable cv;
  size_t left = use - 1;
  auto done_one = [&] {
    std::lock_guard<std::mutex> g(mu);
    if (--left == 0) cv.notify_all();
  };
  for (size_t j = 1; j < use; ++j) {
    Engine* e = c->engines[(start + j) % ne].get();
    bool posted = false;
    try {
      posted = e->post([&, j] {
        run(j);
        done_one();
      });
    } catch (...) {
    }
    if (!posted) {
      run(j);
      done_one();
    }
  }
  run(0);
  {
    std::unique_lock<std::mutex> lk(mu);
    cv.wait(lk, [&] { return left == 0; });
  }
  for (int rc : rcs)
    if (rc) return rc;
  return RS_OK;
}

uint32_t* status_dev(Engine* e, uint32_t idx) {
  return static_cast<uint32_t*>(e->status_chunks[idx / kStatusChunk]->dev.p) + idx % kStatusChunk;
}
uint32_t* status_host(Engine* e, uint32_t idx) {
  return static_cast<uint32_t*>(e->status_chunks[idx / kStatusChunk]->host.p) + idx % kStatusChunk;
}

// The deferred-error word of stream s (a new zeroed one on its first per-stripe
// launch), or nullptr if no memory is left for it.  Caller holds a DeviceScope.
uint32_t* status_word(Engine* e, hipStream_t s) {
  std::lock_guard<std::mutex> g(e->status_mu);
  auto it = e->status_idx.find(s);
  if (it != e->status_idx.end()) return status_dev(e, it->second);
  uint32_t idx;
  if (!e->status_free.empty()) {
    idx = e->status_free.back();  // zeroed when it was released
    e->status_free.pop_back();
  } else {
    idx = e->status_next;
    if (idx / kStatusChunk >= kStatusChunks) return nullptr;
    if (!e->status_chunks[idx / kStatusChunk]) {
      auto ch = std::make_unique<StatusChunk>();
      ch->host.numa = e->numa;
      // zeroed to completion before any kernel can use a word of it: hipMemset may
      // return before the fill has run, and a kernel on a non-blocking stream does not
      // wait for the null stream -- its deferred error then landed before the zeroing
      // and was lost (a fresh process's first per-stripe launch, round 6)
      if (ch->dev.ensure(kStatusChunk * 4) || ch->host.ensure(kStatusChunk * 4) ||
          hipMemsetAsync(ch->dev.p, 0, kStatusChunk * 4, nullptr) != hipSuccess ||
          hipStreamSynchronize(nullptr) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
      }
      e->status_chunks[idx / kStatusChunk] = std::move(ch);
    }
    ++e->status_next;
  }
  e->status_idx.emplace(s, idx);
  return status_dev(e, idx);
}

rs::KernelArgs make_args(Engine* e, const Layout& L, size_t S, size_t N) {
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
  a.k = e->k;
  a.m = e->m;
  a.full_mask = (e->k + e->m >= 32) ? 0xFFFFFFFFu : ((1u << (e->k + e->m)) - 1u);
  a.plan_bytes = rs::plan_stride(e->k, e->m);
  a.lut = static_cast<const uint32_t*>(e->d_lut.p);
  return a;
}

// e_out = outputs per stripe (m for encode, #missing for a uniform reconstruct, max
// #missing for per-stripe patterns).  own_out: the out-of-place rows are the
// engine's own scratch (a staging slab), so their padding may always be written.
int launch(Engine* e, const rs::KernelArgs& args, int e_out, bool per_stripe, hipStream_t s, bool own_out = false) {
  if (args.n_stripes == 0 || args.shard_len == 0 || e_out <= 0) return RS_OK;
  rs::KernelArgs a = args;
  // the encode plan with a verified generated XOR program -> bitsliced kernel
  a.encode_net = (e->bitsliced && !per_stripe && a.plans == e->d_enc_plan.p) ? 1u : 0u;
  a.data_inputs = (!per_stripe && a.plans == e->d_enc_plan.p) ? 1u : 0u;
  if (per_stripe && !(a.status = status_word(e, s))) return RS_ERR_DEVICE;
  if ((e->parity_pad && a.data_inputs && !a.out) || ((e->out_pad || own_out) && a.out)) {
    // rs_set_parity_pad_writes / rs_set_out_pad_writes / engine-owned out rows: run
    // over whole 128-B lines of the slot (inputs' padding read, the written rows'
    // padding written): every output row ends on a whole line, no partial columns
    // A written row's padding stays inside its own slot: within the shard pitch
    // (rows of one stripe) and within the stripe pitch of the written region
    // (stripes of a plane-major / SoA layout lie only that far apart).
    const uint64_t s_eff = std::min<uint64_t>(a.shard_pitch, round_up(static_cast<size_t>(a.shard_len), 128));
    const uint64_t row_sp = a.out ? a.out_sp : a.parity_sp;
    if (s_eff > a.shard_len && s_eff <= 0xFFFFFFF0u && (a.n_stripes <= 1 || s_eff <= row_sp)) {
      a.shard_len = static_cast<uint32_t>(s_eff);
      a.blocks_per_stripe = static_cast<uint32_t>((round_up(s_eff, 16) / 16 + 63) / 64);
      a.full_cols = static_cast<uint32_t>(s_eff / 16);
    }
  }
  // 0: each kernel's own default (rs::launch_apply)
  const uint32_t bpc = e->blocks_per_cu > 0 ? static_cast<uint32_t>(e->blocks_per_cu) : 0u;
  const char* name = rs::launch_apply(a, e_out, per_stripe, bpc, static_cast<uint32_t>(e->cu_count), s, e->occ_cap);
  if (!name) return RS_ERR_DEVICE;
  e->launches.fetch_add(1, std::memory_order_relaxed);
  e->shared->note(s, name);
  RS_HIP(hipGetLastError());
  return RS_OK;
}

int launch_verify_args(Engine* e, rs::KernelArgs& a, hipStream_t s) {
  a.plans = static_cast<const uint8_t*>(e->d_enc_plan.p);
  const int bpc = e->blocks_per_cu > 0 ? e->blocks_per_cu : static_cast<int>(rs::default_blocks_per_cu(e->k, e->m));
  const char* name =
      rs::launch_verify(a, static_cast<uint32_t>(bpc), static_cast<uint32_t>(e->cu_count), s);
  if (!name) return RS_ERR_DEVICE;
  e->launches.fetch_add(1, std::memory_order_relaxed);
  e->shared->note(s, name);
  RS_HIP(hipGetLastError());
  return RS_OK;
}

// Device pointer of the plan for one erasure pattern (cached).  Caller holds a
// DeviceScope for the engine.
int uniform_plan(Engine* e, uint64_t present, bool data_only, const uint8_t** plan_dev) {
  const int t = e->k + e->m;
  present &= full_mask64(t);
  if (__builtin_popcountll(present) < e->k) return RS_ERR_TOO_FEW_SHARDS;
  if (e->have_lut && !data_only) {
    const uint32_t missing = static_cast<uint32_t>(~present & full_mask64(t));
    const uint32_t pid = (*e->h_lut)[missing];
    if (pid == rs::kPlanInvalid) return RS_ERR_TOO_FEW_SHARDS;
    *plan_dev = static_cast<const uint8_t*>(e->d_plans.p) + static_cast<size_t>(pid) * rs::plan_stride(e->k, e->m);
    return RS_OK;
  }
  const uint64_t key = present | (data_only ? (1ull << 63) : 0ull);
  std::lock_guard<std::mutex> g(e->plan_mu);
  auto it = e->plan_cache.find(key);
  if (it == e->plan_cache.end()) {
    std::vector<uint8_t> plan;
    int rc = make_decode_plan(e->k, e->m, *e->enc, present, data_only, &plan);
    if (rc) return rc;
    auto buf = std::make_unique<DevBuf>();
    if (buf->ensure(plan.size())) return RS_ERR_DEVICE;
    RS_HIP(hipMemcpy(buf->p, plan.data(), plan.size(), hipMemcpyHostToDevice));
    it = e->plan_cache.emplace(key, std::move(buf)).first;
  }
  *plan_dev = static_cast<const uint8_t*>(it->second->p);
  return RS_OK;
}

// RAII lane checkout (caller holds a DeviceScope for the engine).
struct LaneGuard {
  Engine* e;
  Lane* lane = nullptr;
  int rc = RS_OK;
  explicit LaneGuard(Engine* en) : e(en) {
    std::unique_lock<std::mutex> g(e->lane_mu);
    if (e->free_lanes.empty() && static_cast<int>(e->lanes.size()) < e->max_lanes) {
      auto l = std::make_unique<Lane>();
      l->host.numa = e->numa;
      if (hipStreamCreateWithFlags(&l->stream, hipStreamNonBlocking) != hipSuccess) {
        rc = RS_ERR_DEVICE;
        return;
      }
      e->free_lanes.push_back(l.get());
      e->lanes.push_back(std::move(l));
    }
    e->lane_cv.wait(g, [&] { return !e->free_lanes.empty(); });
    lane = e->free_lanes.back();
    e->free_lanes.pop_back();
  }
  ~LaneGuard() {
    if (!lane) return;
    std::lock_guard<std::mutex> g(e->lane_mu);
    e->free_lanes.push_back(lane);
    e->lane_cv.notify_one();
  }
};

// One object through a lane: pack inputs into pinned staging, H2D, one kernel,
// D2H of the outputs, unpack.  in/out slots are shard indices into `shards`.
int run_object(Engine* e, const uint8_t* plan_dev, const std::vector<int>& in_idx, const std::vector<int>& out_idx,
               uint8_t* const* shards, size_t S) {
  if (S > 0xFFFFFFF0u) return RS_ERR_INVALID_ARG;
  LaneGuard lg(e);
  if (lg.rc) return lg.rc;
  Lane* L = lg.lane;
  const int t = e->k + e->m;
  const size_t P = round_up(S, 256);  // 256-B slots: see batch.shard_pitch_for
  const size_t bytes = P * static_cast<size_t>(t);
  if (L->dev.ensure(bytes) || L->host.ensure(bytes)) return RS_ERR_DEVICE;
  uint8_t* h = static_cast<uint8_t*>(L->host.p);
  uint8_t* d = static_cast<uint8_t*>(L->dev.p);
  for (int s : in_idx) std::memcpy(h + static_cast<size_t>(s) * P, shards[s], S);
  const int lo = *std::min_element(in_idx.begin(), in_idx.end());
  const int hi = *std::max_element(in_idx.begin(), in_idx.end());
  RS_HIP(hipMemcpyAsync(d + lo * P, h + lo * P, (hi - lo + 1) * P, hipMemcpyHostToDevice, L->stream));
  const Layout dl{d, bytes, d + static_cast<size_t>(e->k) * P, bytes, P};
  rs::KernelArgs a = make_args(e, dl, S, 1);
  a.plans = plan_dev;
  int rc = launch(e, a, static_cast<int>(out_idx.size()), false, L->stream);
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
  const int k = c->k, t = c->k + c->m;
  size_t S = 0;
  int rc = check_shards(t, lens, true, &S);
  if (rc) return rc;
  uint64_t present = 0;
  int np = 0, data_present = 0;
  for (int i = 0; i < t; ++i)
    if (lens[i]) {
      present |= 1ull << i;
      ++np;
      if (i < k) ++data_present;
    }
  if (np == t || (data_only && data_present == k)) return RS_OK;
  if (np < k) return RS_ERR_TOO_FEW_SHARDS;
  std::vector<int> surv, miss;
  for (int i = 0; i < t; ++i) {
    if (lens[i]) {
      if (static_cast<int>(surv.size()) < k) surv.push_back(i);
    } else if (!data_only || i < k) {
      if (!shards[i]) return RS_ERR_INVALID_ARG;
      miss.push_back(i);
    }
  }
  Engine* e = pick_engine(c);
  InflightGuard ig(e);
  DeviceScope ds(e->device);
  if (!ds.ok()) return RS_ERR_DEVICE;
  const uint8_t* plan = nullptr;
  rc = uniform_plan(e, present, data_only, &plan);
  if (rc) return rc;
  rc = run_object(e, plan, surv, miss, shards, S);
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
  const uint64_t cols = round_up(std::min<size_t>(S, rs::kColumnWindow), 16) / 16;
  return N * ((cols + 63) / 64) < 0xFFFFFFFFull;  // task ids of one launch fit 32 bits
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

// ---- per-stripe mask uploads ----------------------------------------------------
// upload_acquire copies n host masks into a free slot and enqueues their copy to the
// slot's device buffer on s;
// the caller launches the kernel that reads them, then the guard's release records
// the slot's event on s AFTER that kernel -- the slot (pinned and device buffer)
// cannot be rewritten or reallocated while any kernel still reads it.
struct UploadGuard {
  Engine* e = nullptr;
  UploadSlot* u = nullptr;
  hipStream_t s = nullptr;
  bool ev_set = false;  // the kernel launch itself updated u->done (rs::set_stop_event)
  ~UploadGuard() {
    if (!u) return;
    rs::set_stop_event(nullptr, nullptr);
    const bool rec = ev_set || hipEventRecord(u->done, s) == hipSuccess;
    std::lock_guard<std::mutex> g(e->upload_mu);
    u->used = rec;
    if (!rec) (void)hipStreamSynchronize(s);  // no event: make the slot safe the slow way
    u->busy = false;
    e->upload_cv.notify_one();
  }
};

// Round 6: the masks are copied into the slot's device buffer by a small kernel on
// the launch stream itself, which reads the pinned slot over PCIe -- no DMA engine,
// no second stream, no cross-stream event -- and the slot's `done` event carries no
// system-scope release (it only tells the host that the kernel stopped reading the
// slot).  Same-process A/B (profiles/r06b_ab_mask.log, profiles/r06a_ab_mask.log, 64 KiB
// objects, mixed 0..m erasures per stripe with host masks) against round 5's H2D on
// an upload stream + cross-stream event + a fenced done event: RS(4+2) 67.9 ->
// 72.7 %, RS(8+4) 69.1 -> 69.6 %, RS(10+4) 59.4 -> 59.9 % of 8 TB/s.  (An H2D on the
// launch stream lost 0.9-3.5 points, the kernel reading the pinned masks in place
// 8-11; the copy kernel on a second stream, overlapping the previous kernel, with a
// fence-free event: level, profiles/r06f_ab_side.log.)
// extra (optional): extra_n more host words copied the same way straight into
// extra_dst (device memory the caller owns), e.g. a packed batch's row offsets.
int upload_acquire(Engine* e, const uint32_t* masks, size_t n, hipStream_t s, UploadGuard* g,
                   const uint32_t** dev, const uint32_t* extra = nullptr, size_t extra_n = 0,
                   uint32_t* extra_dst = nullptr) {
  UploadSlot* u = nullptr;
  {
    std::unique_lock<std::mutex> lk(e->upload_mu);
    for (;;) {
      for (size_t i = 0; i < kUploadSlots && !u; ++i) {
        UploadSlot& c = e->uploads[(e->upload_next + i) % kUploadSlots];
        if (!c.busy) {
          u = &c;
          e->upload_next = (e->upload_next + i + 1) % kUploadSlots;
        }
      }
      if (u) break;
      e->upload_cv.wait(lk);
    }
    u->busy = true;
  }
  g->e = e;
  g->u = u;
  g->s = s;
  if (!u->done) RS_HIP(hipEventCreateWithFlags(&u->done, hipEventDisableTiming | hipEventDisableSystemFence));
  if (u->used) RS_HIP(hipEventSynchronize(u->done));  // the last kernel that read this slot is done
  u->host.numa = e->numa;
  const void* before = u->host.p;
  if (u->host.ensure((n + extra_n) * 4) || u->dev.ensure(n * 4)) return RS_ERR_DEVICE;
  if (u->host.p != before || !u->host_dev) {
    void* dp = nullptr;
    RS_HIP(hipHostGetDevicePointer(&dp, u->host.p, 0));
    u->host_dev = dp;
  }
  std::memcpy(u->host.p, masks, n * 4);
  if (extra_n) std::memcpy(static_cast<uint32_t*>(u->host.p) + n, extra, extra_n * 4);
  if (!rs::launch_words_copy(static_cast<const uint32_t*>(u->host_dev), static_cast<uint32_t*>(u->dev.p), n, s,
                             extra_n ? extra_dst : nullptr, extra_n))
    return RS_ERR_DEVICE;
  *dev = static_cast<const uint32_t*>(u->dev.p);
  // the reading kernel's own completion updates the slot's event (no marker packet
  // after it: host-mask launches +1.0 / +2.6 / +2.0 points for RS(10+4) / RS(8+4) /
  // RS(4+2) 64 KiB mixed scans without the marker, profiles/r06n_ab_hostdiag.log)
  rs::set_stop_event(u->done, &g->ev_set);
  return RS_OK;
}

int ensure_pipe_stream(Engine* e, int i) {
  if (!e->pipe_st[i]) RS_HIP(hipStreamCreateWithFlags(&e->pipe_st[i], hipStreamNonBlocking));
  return RS_OK;
}

// Zero-copy host batch: with the shards in the context's own page-locked memory
// (rs_host_alloc) the kernel itself reads the K survivors and writes only the
// missing shards across PCIe, in place -- per stripe exactly the bytes the codec
// needs, no staging slab, no DMA of slots it does not touch (the staged pipeline
// must move every slot a stripe might use).  Memory the library does not own --
// pageable, rs_host_register'ed or pinned by someone else -- never qualifies: a
// kernel never reads or writes pages whose lifetime and placement the library does
// not control (`HISTORY.md` §A.1).  Returns RS_ERR_NOT_SUPPORTED when the batch does
// not qualify.
int host_zero_copy(Engine* e, const Layout& hl, size_t S, size_t N, const uint8_t* plan_dev,
                   const uint32_t* masks_host, int e_out, uint32_t* bad_host) {
  const int k = e->k, m = e->m;
  const size_t dbytes = (N - 1) * hl.data_sp + static_cast<size_t>(k - 1) * hl.pitch + S;
  const size_t pbytes = m ? (N - 1) * hl.parity_sp + static_cast<size_t>(m - 1) * hl.pitch + S : 0;
  uint8_t* dd = rs::ctx_owned(e->ctx, hl.data, dbytes);
  uint8_t* pd = m ? rs::ctx_owned(e->ctx, hl.parity, pbytes) : nullptr;
  if (!dd || (m && !pd)) return RS_ERR_NOT_SUPPORTED;
  const Layout dl{dd, hl.data_sp, pd, hl.parity_sp, hl.pitch};
  if (!device_layout_ok(dl, m, S)) return RS_ERR_NOT_SUPPORTED;
  std::lock_guard<std::mutex> g(e->host_mu);
  int rc = ensure_pipe_stream(e, 0);
  if (rc) return rc;
  hipStream_t st = e->pipe_st[0];
  rs::KernelArgs a = make_args(e, dl, S, N);
  a.plans = plan_dev;
  if (bad_host) {
    if (e->d_bad.ensure(N * 4)) return RS_ERR_DEVICE;
    a.bad = static_cast<uint32_t*>(e->d_bad.p);
    rc = launch_verify_args(e, a, st);
    if (rc) return rc;
    RS_HIP(hipMemcpyAsync(bad_host, a.bad, N * 4, hipMemcpyDeviceToHost, st));
  } else {
    UploadGuard ug;
    if (masks_host) {
      const uint32_t* dm = nullptr;
      rc = upload_acquire(e, masks_host, N, st, &ug, &dm);
      if (rc) return rc;
      a.present_masks = dm;
    }
    rc = launch(e, a, e_out, masks_host != nullptr, st);
    if (rc) return rc;
  }
  RS_HIP(hipStreamSynchronize(st));
  e->shared->last_host_path.store("zero-copy");
  return RS_OK;
}

// The first k present shards of a mask: the survivors a per-stripe plan reads
// (klauspost's choice, make_decode_plan).
uint32_t first_present(uint32_t present, int k) {
  uint32_t r = 0;
  for (int c = 0; c < k && present; ++c) {
    r |= present & (0u - present);
    present &= present - 1u;
  }
  return r;
}

// Staged per-stripe reconstruct (round 5): only the bytes the codec needs cross
// PCIe, and the caller's present shards are never written.
//  * H2D: the data slots some stripe of the share reads (the union of every
//    stripe's first k present shards: normally all k, one contiguous copy per
//    stripe).  Parity survivors are needed only by stripes missing a data shard
//    (a third of a 50/50 encode / 1-erasure RS(4+2) mix): the host gathers exactly
//    those rows into the library's own page-locked slab, which the kernel reads in
//    place over PCIe -- no DMA of parity rows nobody reads.
//  * The kernel writes out of place into a dense slab, the r-th missing shard of
//    stripe i at row i*e_out + r (what the healer writes back, poller.go:288-302),
//    whole 128-B lines (the slab is the engine's own).
//  * D2H: that slab (e_out rows per stripe, not k+m) into a ring of pinned buffers,
//    from which scatter threads copy each row into the caller's missing slot while
//    later chunks are in flight (one thread cannot keep up with the link: a 4 KiB
//    RS(4+2) mix scatters ~1.5 KiB per 5 KiB of H2D).
// Round 4 moved every slot both ways and wrote the present ones back unchanged:
// config 5 (50/50 encode / 1-erasure) 25.7 GiB/s.
constexpr int kScatterRing = 2 * kHostStreams;  // pinned D2H buffers in flight or being scattered
constexpr int kScatterThreads = 3;

int host_batch_ps(Engine* e, const Layout& hl, size_t S, size_t N, const uint32_t* masks, int e_out) {
  const int k = e->k, m = e->m, t = k + m;
  const uint32_t full = static_cast<uint32_t>(full_mask64(t));  // t <= 16: per-stripe host masks need the LUT
  std::vector<uint8_t> seen(size_t(1) << t, 0);
  uint32_t need = 0;
  for (size_t i = 0; i < N; ++i) {
    const uint32_t pm = masks[i] & full;
    if (!seen[pm]) {
      seen[pm] = 1;
      need |= first_present(pm, k);
    }
  }
  std::vector<int> in_slots;  // data slots only: parity survivors are gathered
  for (int s = 0; s < k; ++s)
    if ((need >> s) & 1u) in_slots.push_back(s);
  const bool need_par = (need >> k) != 0u;
  const size_t P = round_up(S, 256);  // 256-B slots: see batch.shard_pitch_for
  const size_t slab = P * static_cast<size_t>(t), outb = P * static_cast<size_t>(e_out);
  const size_t per_stripe = slab + outb + 4;
  const size_t chunk = std::min(N, std::max<size_t>(1, kHostChunkBytes / per_stripe));
  const size_t in_bytes = round_up(chunk * slab, 256), out_bytes = round_up(chunk * outb, 256);
  const size_t host_bytes = chunk * static_cast<size_t>(e_out) * S;
  std::lock_guard<std::mutex> g(e->host_mu);
  for (int i = 0; i < kHostStreams; ++i) {
    int rc = ensure_pipe_stream(e, i);
    if (rc) return rc;
    if (e->pipe_buf[i].ensure(std::max(kHostChunkBytes, in_bytes + out_bytes + chunk * 4) + per_stripe + 256))
      return RS_ERR_DEVICE;
    if (need_par) {
      const void* before = e->par_host[i].p;
      e->par_host[i].numa = e->numa;
      if (e->par_host[i].ensure(chunk * P * static_cast<size_t>(m))) return RS_ERR_DEVICE;
      if (e->par_host[i].p != before || !e->par_dev[i]) {
        void* dev = nullptr;
        RS_HIP(hipHostGetDevicePointer(&dev, e->par_host[i].p, 0));
        e->par_dev[i] = static_cast<uint8_t*>(dev);
      }
    }
  }
  for (int b = 0; b < kScatterRing; ++b) {
    e->scatter_host[b].numa = e->numa;
    if (e->scatter_host[b].ensure(host_bytes)) return RS_ERR_DEVICE;
    if (!e->scatter_ev[b]) RS_HIP(hipEventCreateWithFlags(&e->scatter_ev[b], hipEventDisableTiming));
  }
  // rows of the chunk in ring buffer b into the caller's missing slots
  auto scatter = [&](size_t s0, size_t n, int b) {
    const uint8_t* h = static_cast<const uint8_t*>(e->scatter_host[b].p);
    for (size_t q = 0; q < n; ++q) {
      const size_t s = s0 + q;
      uint32_t miss = ~masks[s] & full;
      for (size_t r = 0; miss; ++r) {
        const int j = __builtin_ctz(miss);
        miss &= miss - 1u;
        std::memcpy(hl.slot(k, s, j), h + (q * static_cast<size_t>(e_out) + r) * S, S);
      }
    }
  };
  const size_t n_chunks = (N + chunk - 1) / chunk;
  // scatter threads (several chunks only): a queue of retired chunks; buffer b is
  // free again once done[b] counts its chunk
  struct Job {
    size_t s0, n;
    int b;
  };
  std::mutex qm;
  std::condition_variable qcv, dcv;
  std::deque<Job> q;
  bool stop = false;
  std::vector<size_t> done(kScatterRing, 0), want(kScatterRing, 0);  // chunks scattered / handed out per buffer
  std::vector<std::thread> pool;
  if (n_chunks > static_cast<size_t>(kHostStreams)) {
    try {
      for (int w = 0; w < kScatterThreads; ++w)
        pool.emplace_back([&] {
          std::unique_lock<std::mutex> lk(qm);
          for (;;) {
            qcv.wait(lk, [&] { return stop || !q.empty(); });
            if (q.empty()) return;
            const Job jb = q.front();
            q.pop_front();
            lk.unlock();
            scatter(jb.s0, jb.n, jb.b);
            lk.lock();
            ++done[jb.b];
            dcv.notify_all();
          }
        });
    } catch (...) {  // no threads: the calling thread scatters
    }
  }
  auto join_pool = [&] {
    {
      std::lock_guard<std::mutex> lk(qm);
      stop = true;
    }
    qcv.notify_all();
    for (auto& th : pool) th.join();
    pool.clear();
  };
  std::vector<Job> inflight;  // enqueued chunks not yet retired, oldest first
  int rc = RS_OK;
  auto retire = [&](const Job& jb) -> int {  // the chunk's rows are in host memory: scatter them
    RS_HIP(hipEventSynchronize(e->scatter_ev[jb.b]));
    if (pool.empty()) {
      scatter(jb.s0, jb.n, jb.b);
      std::lock_guard<std::mutex> lk(qm);
      ++done[jb.b];
      return RS_OK;
    }
    {
      std::lock_guard<std::mutex> lk(qm);
      q.push_back(jb);
    }
    qcv.notify_one();
    return RS_OK;
  };
  for (size_t j = 0; j < n_chunks && rc == RS_OK; ++j) {
    const size_t s0 = j * chunk, n = std::min(chunk, N - s0);
    const int i = static_cast<int>(j % kHostStreams), b = static_cast<int>(j % kScatterRing);
    hipStream_t st = e->pipe_st[i];
    // keep at most kHostStreams chunks queued on the device: retire the oldest first
    if (inflight.size() >= static_cast<size_t>(kHostStreams)) {
      rc = retire(inflight.front());
      inflight.erase(inflight.begin());
      if (rc) break;
    }
    {  // ring buffer b: its previous chunk must be scattered before the D2H reuses it
      std::unique_lock<std::mutex> lk(qm);
      dcv.wait(lk, [&] { return done[b] == want[b]; });
      ++want[b];
    }
    uint8_t* d = static_cast<uint8_t*>(e->pipe_buf[i].p);
    // data slots in the device slab; parity slots in the pinned gather slab, which
    // the retire of chunk j - kHostStreams (above) has freed from its last kernel
    const Layout dl{d, P * k, need_par ? e->par_dev[i] : d + chunk * P * k, P * m, P};
    rc = copy_slots(dl, hl, k, in_slots, 0, s0, n, S, hipMemcpyHostToDevice, st);
    if (rc) break;
    if (need_par) {
      uint8_t* ph = static_cast<uint8_t*>(e->par_host[i].p);
      for (size_t q = 0; q < n; ++q) {
        uint32_t pm = first_present(masks[s0 + q] & full, k) >> k;  // parity survivors of this stripe
        while (pm) {
          const int p = __builtin_ctz(pm);
          pm &= pm - 1u;
          std::memcpy(ph + (q * static_cast<size_t>(m) + p) * P, hl.slot(k, s0 + q, k + p), S);
        }
      }
    }
    uint8_t* o = d + in_bytes;
    uint32_t* aux = reinterpret_cast<uint32_t*>(o + out_bytes);
    if (hipMemcpyAsync(aux, masks + s0, n * 4, hipMemcpyHostToDevice, st) != hipSuccess) {
      rc = RS_ERR_DEVICE;
      break;
    }
    rs::KernelArgs a = make_args(e, dl, S, n);
    a.plans = static_cast<const uint8_t*>(e->d_plans.p);
    a.present_masks = aux;
    a.out = o;
    a.out_sp = outb;
    rc = launch(e, a, e_out, true, st, true);  // the slab's rows: whole-line writes
    if (rc) break;
    if (copy2d(e->scatter_host[b].p, S, o, P, S, n * static_cast<size_t>(e_out), hipMemcpyDeviceToHost, st) !=
            hipSuccess ||
        hipEventRecord(e->scatter_ev[b], st) != hipSuccess) {
      rc = RS_ERR_DEVICE;
      break;
    }
    inflight.push_back(Job{s0, n, b});
  }
  for (const Job& jb : inflight) {
    const int r2 = retire(jb);
    if (!rc) rc = r2;
  }
  join_pool();  // drains the queue first
  for (int i = 0; i < kHostStreams; ++i)
    if (hipStreamSynchronize(e->pipe_st[i]) != hipSuccess && !rc) rc = RS_ERR_DEVICE;
  return rc;
}

// One engine's share of a host-resident batch (caller holds its DeviceScope).
int host_batch(Engine* e, const Layout& hl, const std::vector<int>& in_slots, const std::vector<int>& out_slots,
               size_t S, size_t N, const uint8_t* plan_dev, const uint32_t* masks_host, int e_out,
               uint32_t* bad_host = nullptr) {
  if (N == 0) return RS_OK;
  if (e->host_zero_copy) {
    const int rc = host_zero_copy(e, hl, S, N, plan_dev, masks_host, e_out, bad_host);
    if (rc != RS_ERR_NOT_SUPPORTED) return rc;
  }
  e->shared->last_host_path.store("staged");
  if (masks_host && !bad_host) return host_batch_ps(e, hl, S, N, masks_host, e_out);
  const int k = e->k, m = e->m;
  const size_t P = round_up(S, 256);  // 256-B slots: see batch.shard_pitch_for
  const size_t per_stripe = P * static_cast<size_t>(k + m) + ((masks_host || bad_host) ? 4 : 0);
  const size_t chunk = std::min(N, std::max<size_t>(1, kHostChunkBytes / per_stripe));
  std::lock_guard<std::mutex> g(e->host_mu);
  for (int i = 0; i < kHostStreams; ++i) {
    int rc = ensure_pipe_stream(e, i);
    if (rc) return rc;
    // sized for a full chunk whatever N is, so a small call never leaves slabs that
    // a later large call has to reallocate
    if (e->pipe_buf[i].ensure(std::max(kHostChunkBytes, per_stripe) + per_stripe + 256)) return RS_ERR_DEVICE;
  }
  int j = 0;
  for (size_t s0 = 0; s0 < N; s0 += chunk, ++j) {
    const size_t n = std::min(chunk, N - s0);
    hipStream_t st = e->pipe_st[j % kHostStreams];
    uint8_t* d = static_cast<uint8_t*>(e->pipe_buf[j % kHostStreams].p);
    const Layout dl{d, P * k, d + chunk * P * k, P * m, P};
    int rc = copy_slots(dl, hl, k, in_slots, 0, s0, n, S, hipMemcpyHostToDevice, st);
    if (rc) return rc;
    rs::KernelArgs a = make_args(e, dl, S, n);
    a.plans = plan_dev;
    // masks / mismatch words live in the slab itself: stream-ordered with the chunk
    uint32_t* aux = reinterpret_cast<uint32_t*>(d + round_up(chunk * P * (k + m), 256));
    if (masks_host) {
      RS_HIP(hipMemcpyAsync(aux, masks_host + s0, n * 4, hipMemcpyHostToDevice, st));
      a.present_masks = aux;
    }
    if (bad_host) {
      a.bad = aux;
      rc = launch_verify_args(e, a, st);
      if (rc) return rc;
      RS_HIP(hipMemcpyAsync(bad_host + s0, aux, n * 4, hipMemcpyDeviceToHost, st));
      continue;
    }
    rc = launch(e, a, e_out, masks_host != nullptr, st);
    if (rc) return rc;
    rc = copy_slots(hl, dl, k, out_slots, s0, 0, n, S, hipMemcpyDeviceToHost, st);
    if (rc) return rc;
  }
  for (int i = 0; i < kHostStreams; ++i) RS_HIP(hipStreamSynchronize(e->pipe_st[i]));
  return RS_OK;
}

// ---- engine creation ----------------------------------------------------------------
struct PlanSet {
  std::vector<uint8_t> enc_plan, all_plans;
  bool have_lut = false;
};

int create_engine(rs_ctx* c, int device, const PlanSet& ps, std::unique_ptr<Engine>* out) {
  DeviceScope ds(device);
  if (!ds.ok()) return RS_ERR_DEVICE;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) return RS_ERR_DEVICE;
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) return RS_ERR_NO_DEVICE;
  auto e = std::make_unique<Engine>();
  e->ctx = c;
  e->k = c->k;
  e->m = c->m;
  e->device = device;
  e->cu_count = prop.multiProcessorCount;
  e->numa = rs::device_numa_node(device);
  e->enc = &c->enc;
  e->h_lut = &c->h_lut;
  e->shared = &c->shared;
  if (const uint8_t* rows = rs::bitsliced_encode_rows(c->k, c->m)) {
    bool same = true;
    for (int r = 0; r < c->m; ++r)
      for (int q = 0; q < c->k; ++q) same = same && rows[r * c->k + q] == c->enc.at(c->k + r, q);
    e->bitsliced = same;
  }
  char name[200];
  std::snprintf(name, sizeof(name), "hip:%s:%s:%dCU:dev%d:numa%d", prop.gcnArchName, prop.name, e->cu_count, device,
                e->numa);
  e->name = name;
  if (e->d_enc_plan.ensure(ps.enc_plan.size()) ||
      hipMemcpy(e->d_enc_plan.p, ps.enc_plan.data(), ps.enc_plan.size(), hipMemcpyHostToDevice) != hipSuccess)
    return RS_ERR_DEVICE;
  if (ps.have_lut) {
    if (e->d_plans.ensure(ps.all_plans.size()) || e->d_lut.ensure(c->h_lut.size() * 4)) return RS_ERR_DEVICE;
    if (hipMemcpy(e->d_plans.p, ps.all_plans.data(), ps.all_plans.size(), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(e->d_lut.p, c->h_lut.data(), c->h_lut.size() * 4, hipMemcpyHostToDevice) != hipSuccess)
      return RS_ERR_DEVICE;
    e->have_lut = true;
  }
  *out = std::move(e);
  return RS_OK;
}

// Host-side plans shared by every engine of a context.
PlanSet build_plans(rs_ctx* c) {
  const int k = c->k, m = c->m, t = k + m;
  PlanSet ps;
  // Encode plan: in = data slots 0..k-1, out = parity slots k..k+m-1.
  {
    std::vector<int> in_idx(k), out_idx(m);
    for (int i = 0; i < k; ++i) in_idx[i] = i;
    for (int p = 0; p < m; ++p) out_idx[p] = k + p;
    std::vector<uint8_t> rows(static_cast<size_t>(m) * k);
    for (int p = 0; p < m; ++p)
      for (int i = 0; i < k; ++i) rows[p * k + i] = c->enc.at(k + p, i);
    ps.enc_plan = make_plan(k, m, static_cast<uint32_t>((1ull << k) - 1), static_cast<uint32_t>(full_mask64(t)),
                            in_idx, out_idx, rows);
  }
  // Eager all-pattern plans + LUT for k+m <= 16.  Plan 0 = nothing missing.
  if (t <= 16 && m > 0) {
    const uint32_t full = (1u << t) - 1u;
    c->h_lut.assign(size_t(1) << t, rs::kPlanInvalid);
    {
      std::vector<int> in_idx(k), none;
      for (int i = 0; i < k; ++i) in_idx[i] = i;
      std::vector<uint8_t> p = make_plan(k, m, full, full, in_idx, none, {});
      ps.all_plans.insert(ps.all_plans.end(), p.begin(), p.end());
      c->h_lut[0] = 0;
    }
    uint32_t count = 1;
    bool ok = true;
    for (uint32_t missing = 1; missing <= full && ok; ++missing) {
      if (__builtin_popcount(missing) > m) continue;
      std::vector<uint8_t> p;
      if (make_decode_plan(k, m, c->enc, full & ~missing, false, &p) != RS_OK) continue;
      if (ps.all_plans.size() + p.size() > (size_t(64) << 20)) {
        ok = false;
        break;
      }
      ps.all_plans.insert(ps.all_plans.end(), p.begin(), p.end());
      c->h_lut[missing] = count++;
    }
    ps.have_lut = ok;
    if (!ok) c->h_lut.clear();
  }
  return ps;
}

}  // namespace

// ---- internal interface for the coalescer (rs_engine.hpp) ---------------------------
namespace rs {

int ctx_engine_count(const rs_ctx* c) { return c ? static_cast<int>(c->engines.size()) : 0; }

uint8_t* ctx_owned(rs_ctx* c, const void* p, size_t bytes) {
  if (!c || !p || bytes == 0 || c->n_owned.load(std::memory_order_acquire) == 0) return nullptr;
  const uintptr_t lo = reinterpret_cast<uintptr_t>(p);
  std::shared_lock<std::shared_mutex> g(c->reg_mu);
  auto it = std::upper_bound(c->reg.begin(), c->reg.end(), lo,
                             [](uintptr_t x, const RegRange& r) { return x < r.lo; });
  if (it == c->reg.begin()) return nullptr;
  --it;  // the last range starting at or before p
  if (!it->owned || lo >= it->hi || bytes > it->hi - lo) return nullptr;
  return it->dev + (lo - it->lo);
}
Engine* ctx_engine(rs_ctx* c, int i) { return c->engines[static_cast<size_t>(i)].get(); }
int engine_device(const Engine* e) { return e->device; }

int engine_encode_batch(Engine* e, const uint8_t* data, size_t data_sp, uint8_t* parity, size_t parity_sp,
                        size_t pitch, size_t S, size_t N, hipStream_t s) {
  if (N == 0 || e->m == 0) return RS_OK;
  const Layout L{const_cast<uint8_t*>(data), data_sp, parity, parity_sp, pitch};
  if (!batch_sizes_ok(S, N, pitch) || !device_layout_ok(L, e->m, S)) return RS_ERR_INVALID_ARG;
  rs::KernelArgs a = make_args(e, L, S, N);
  a.plans = static_cast<const uint8_t*>(e->d_enc_plan.p);
  return launch(e, a, e->m, false, s);
}

int engine_reconstruct_batch_out(Engine* e, const uint8_t* data, size_t data_sp, const uint8_t* parity,
                                 size_t parity_sp, size_t pitch, size_t S, size_t N, const uint32_t* masks,
                                 size_t n_masks, int masks_on_device, int max_missing, uint8_t* out, size_t out_sp,
                                 hipStream_t s) {
  if (N == 0) return RS_OK;
  if (S == 0) return RS_ERR_SHARD_NO_DATA;
  if (!batch_sizes_ok(S, N, pitch)) return RS_ERR_INVALID_ARG;
  const Layout L{const_cast<uint8_t*>(data), data_sp, const_cast<uint8_t*>(parity), parity_sp, pitch};
  if (!device_layout_ok(L, e->m, S) || reinterpret_cast<uintptr_t>(out) % 16 || out_sp % 16) return RS_ERR_INVALID_ARG;
  const int t = e->k + e->m;
  const uint32_t full = static_cast<uint32_t>(full_mask64(t));
  rs::KernelArgs a = make_args(e, L, S, N);
  a.out = out;
  a.out_sp = out_sp;
  if (masks_on_device) {
    if (!e->have_lut) return RS_ERR_NOT_SUPPORTED;
    if (max_missing < 0) return RS_ERR_INVALID_ARG;
    const int bound = max_missing > 0 ? std::min(max_missing, e->m) : e->m;
    if (!out_layout_ok(out_sp, pitch, S, N, bound)) return RS_ERR_INVALID_ARG;
    a.plans = static_cast<const uint8_t*>(e->d_plans.p);
    a.present_masks = masks;
    return launch(e, a, bound, true, s);
  }
  if (n_masks != 1 && n_masks != N) return RS_ERR_INVALID_ARG;
  int most = 0;
  for (size_t i = 0; i < n_masks; ++i) {
    const int np = __builtin_popcount(masks[i] & full);
    if (np < e->k) return RS_ERR_TOO_FEW_SHARDS;
    most = std::max(most, t - np);
  }
  if (most == 0) return RS_OK;
  if (!out_layout_ok(out_sp, pitch, S, N, most)) return RS_ERR_INVALID_ARG;
  if (n_masks == 1) {
    const uint8_t* plan = nullptr;
    int rc = uniform_plan(e, masks[0] & full, false, &plan);
    if (rc) return rc;
    a.plans = plan;
    return launch(e, a, most, false, s);
  }
  if (!e->have_lut) return RS_ERR_NOT_SUPPORTED;
  UploadGuard ug;
  const uint32_t* dm = nullptr;
  int rc = upload_acquire(e, masks, N, s, &ug, &dm);
  if (rc) return rc;
  a.plans = static_cast<const uint8_t*>(e->d_plans.p);
  a.present_masks = dm;
  return launch(e, a, most, true, s);
}

// Packed out-of-place reconstruct: the missing shards of the whole batch back to back,
// stripe i's from row row_offsets[i] (an exclusive prefix sum of the erasure counts,
// written here: N + 1 device words; a stripe with < k present takes none, so the batch
// needs at most N * m rows).  Device masks: a one-workgroup scan kernel ahead
// of the reconstruct on s; host masks: the offsets summed on the host and copied with
// the masks.
int engine_reconstruct_batch_packed(Engine* e, const uint8_t* data, size_t data_sp, const uint8_t* parity,
                                    size_t parity_sp, size_t pitch, size_t S, size_t N, const uint32_t* masks,
                                    int masks_on_device, uint8_t* out, uint32_t* row_offsets, hipStream_t s) {
  if (N == 0) return RS_OK;
  if (S == 0) return RS_ERR_SHARD_NO_DATA;
  if (!batch_sizes_ok(S, N, pitch) || N >= 0xFFFFFFFFull / 32u) return RS_ERR_INVALID_ARG;
  const Layout L{const_cast<uint8_t*>(data), data_sp, const_cast<uint8_t*>(parity), parity_sp, pitch};
  if (!device_layout_ok(L, e->m, S) || reinterpret_cast<uintptr_t>(out) % 16 ||
      reinterpret_cast<uintptr_t>(row_offsets) % 4)
    return RS_ERR_INVALID_ARG;
  if (!e->have_lut) return RS_ERR_NOT_SUPPORTED;
  const int t = e->k + e->m;
  const uint32_t full = static_cast<uint32_t>(full_mask64(t));
  rs::KernelArgs a = make_args(e, L, S, N);
  a.out = out;
  a.out_sp = pitch;  // each row owns one pitch: whole-line rows stay inside it
  a.row_offsets = row_offsets;
  a.plans = static_cast<const uint8_t*>(e->d_plans.p);
  if (masks_on_device) {
    if (!rs::launch_row_offsets(masks, full, static_cast<uint32_t>(e->m), row_offsets, N, s)) return RS_ERR_DEVICE;
    a.present_masks = masks;
    return launch(e, a, e->m, true, s);
  }
  int most = 0;
  std::vector<uint32_t> offs(N + 1);
  uint32_t rows = 0;
  for (size_t i = 0; i < N; ++i) {
    const int np = __builtin_popcount(masks[i] & full);
    if (np < e->k) return RS_ERR_TOO_FEW_SHARDS;
    offs[i] = rows;
    rows += static_cast<uint32_t>(t - np);
    most = std::max(most, t - np);
  }
  offs[N] = rows;
  UploadGuard ug;
  const uint32_t* dm = nullptr;
  int rc = upload_acquire(e, masks, N, s, &ug, &dm, offs.data(), N + 1, row_offsets);
  if (rc) return rc;
  if (most == 0) return RS_OK;  // the offsets are all 0 (copied above), nothing to compute
  a.present_masks = dm;
  return launch(e, a, most, true, s);
}

int engine_plan_for(Engine* e, uint64_t present, bool data_only, const uint8_t** plan) {
  DeviceScope ds(e->device);
  if (!ds.ok()) return RS_ERR_DEVICE;
  return uniform_plan(e, present, data_only, plan);
}

const uint8_t* engine_encode_plan(Engine* e) { return static_cast<const uint8_t*>(e->d_enc_plan.p); }

int engine_apply_batch_plans(Engine* e, const uint8_t* data, size_t data_sp, const uint8_t* parity,
                             size_t parity_sp, size_t pitch, size_t S, size_t N, const uint64_t* plans_dev,
                             uint8_t* out, size_t out_sp, hipStream_t s) {
  if (N == 0) return RS_OK;
  if (S == 0) return RS_ERR_SHARD_NO_DATA;
  if (!batch_sizes_ok(S, N, pitch)) return RS_ERR_INVALID_ARG;
  const Layout L{const_cast<uint8_t*>(data), data_sp, const_cast<uint8_t*>(parity), parity_sp, pitch};
  if (!device_layout_ok(L, e->m, S) || reinterpret_cast<uintptr_t>(out) % 16 || out_sp % 16 ||
      !out_layout_ok(out_sp, pitch, S, N, e->m))
    return RS_ERR_INVALID_ARG;
  rs::KernelArgs a = make_args(e, L, S, N);
  a.out = out;
  a.out_sp = out_sp;
  a.plans = static_cast<const uint8_t*>(e->d_enc_plan.p);  // unused: every stripe has its own
  a.stripe_plans = plans_dev;
  return launch(e, a, e->m, true, s);
}

int engine_apply_batch_ptrs(Engine* e, const uint64_t* shard_ptrs_dev, const uint32_t* masks_dev, size_t S,
                            size_t N, int max_missing, hipStream_t s) {
  if (N == 0) return RS_OK;
  if (S == 0) return RS_ERR_SHARD_NO_DATA;
  if (!e->have_lut || S > 0xFFFFFFF0u || N * ((round_up(S, 16) / 16 + 63) / 64) >= (1ull << 32))
    return RS_ERR_NOT_SUPPORTED;
  const int bound = max_missing > 0 ? std::min(max_missing, e->m) : e->m;
  const Layout L{nullptr, 0, nullptr, 0, round_up(S, 16)};
  rs::KernelArgs a = make_args(e, L, S, N);
  a.plans = static_cast<const uint8_t*>(e->d_plans.p);
  a.present_masks = masks_dev;
  a.shard_ptrs = shard_ptrs_dev;
  if (!(a.status = status_word(e, s))) return RS_ERR_DEVICE;
  const int bpc = e->blocks_per_cu > 0 ? e->blocks_per_cu : static_cast<int>(rs::default_blocks_per_cu(e->k, bound));
  const char* name = rs::launch_apply_ptrs(a, bound, static_cast<uint32_t>(bpc), static_cast<uint32_t>(e->cu_count), s);
  if (!name) return RS_ERR_NOT_SUPPORTED;
  e->launches.fetch_add(1, std::memory_order_relaxed);
  e->shared->note(s, name);
  RS_HIP(hipGetLastError());
  return RS_OK;
}

int engine_verify_batch(Engine* e, const uint8_t* data, size_t data_sp, const uint8_t* parity, size_t parity_sp,
                        size_t pitch, size_t S, size_t N, uint32_t* bad_dev, hipStream_t s) {
  if (N == 0) return RS_OK;
  if (e->m == 0) {
    RS_HIP(hipMemsetAsync(bad_dev, 0, N * 4, s));
    return RS_OK;
  }
  const Layout L{const_cast<uint8_t*>(data), data_sp, const_cast<uint8_t*>(parity), parity_sp, pitch};
  if (!batch_sizes_ok(S, N, pitch) || !device_layout_ok(L, e->m, S)) return RS_ERR_INVALID_ARG;
  rs::KernelArgs a = make_args(e, L, S, N);
  a.bad = bad_dev;
  return launch_verify_args(e, a, s);
}

}  // namespace rs

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
    case RS_ERR_BUSY: return "rsgpu: coalescer busy, reap completed calls and retry";
    default: return "rsgpu: unknown error";
  }
}

int rs_create_devices(int k, int m, const int* devices, int n_devices, int flags, rs_ctx** out) {
  (void)flags;
  if (!out) return RS_ERR_INVALID_ARG;
  *out = nullptr;
  // [upstream reedsolomon.go New] argument checks, same order and sentinels.
  if (k <= 0 || m < 0) return RS_ERR_INV_SHARD_NUM;
  if (k + m > 256) return RS_ERR_MAX_SHARD_NUM;
  if (k > rs::kMaxK || m > rs::kMaxM || k + m > 32) return RS_ERR_NOT_SUPPORTED;
  if (!devices || n_devices <= 0 || n_devices > 64) return RS_ERR_INVALID_ARG;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
    (void)hipGetLastError();
    return RS_ERR_NO_DEVICE;
  }
  for (int i = 0; i < n_devices; ++i)
    if (devices[i] < 0 || devices[i] >= ndev) return RS_ERR_NO_DEVICE;

  auto c = std::make_unique<rs_ctx>();
  c->k = k;
  c->m = m;
  c->enc = rs::build_encode_matrix(k, m);
  const PlanSet ps = build_plans(c.get());
  for (int i = 0; i < n_devices; ++i) {
    std::unique_ptr<Engine> e;
    const int rc = create_engine(c.get(), devices[i], ps, &e);
    if (rc) return rc;
    c->engines.push_back(std::move(e));
  }
  c->backend = c->engines[0]->name;
  if (n_devices > 1) {
    c->backend += " x" + std::to_string(n_devices) + " [devices";
    for (int i = 0; i < n_devices; ++i) c->backend += " " + std::to_string(devices[i]);
    c->backend += "]";
  }
  *out = c.release();
  return RS_OK;
}

int rs_create(int k, int m, int device, int flags, rs_ctx** out) {
  return rs_create_devices(k, m, &device, 1, flags, out);
}

int rs_create_multi(int k, int m, uint64_t device_mask, int flags, rs_ctx** out) {
  if (!out) return RS_ERR_INVALID_ARG;
  *out = nullptr;
  if (k <= 0 || m < 0) return RS_ERR_INV_SHARD_NUM;
  if (k + m > 256) return RS_ERR_MAX_SHARD_NUM;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
    (void)hipGetLastError();
    return RS_ERR_NO_DEVICE;
  }
  std::vector<int> devs;
  for (int d = 0; d < std::min(ndev, 64); ++d) {
    if (device_mask && !((device_mask >> d) & 1u)) continue;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, d) != hipSuccess) return RS_ERR_DEVICE;
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
      if (device_mask) return RS_ERR_NO_DEVICE;  // an explicitly named device must be usable
      continue;
    }
    devs.push_back(d);
  }
  if (ndev < 64 && (device_mask >> ndev)) return RS_ERR_NO_DEVICE;  // names a device that does not exist
  if (devs.empty()) return RS_ERR_NO_DEVICE;
  return rs_create_devices(k, m, devs.data(), static_cast<int>(devs.size()), flags, out);
}

void rs_destroy(rs_ctx* ctx) {
  if (!ctx) return;
  std::vector<void*> owned;  // rs_host_alloc'ed memory never freed by the caller
  for (const RegRange& r : ctx->reg)
    if (r.owned) owned.push_back(reinterpret_cast<void*>(r.lo));
  // engines first: each joins its worker and synchronises its device, so no queued
  // kernel still reads or writes an arena when it is freed
  delete ctx;
  for (void* p : owned) rs::pinned_free(p);
}

int rs_data_shards(const rs_ctx* c) { return c ? c->k : 0; }
int rs_parity_shards(const rs_ctx* c) { return c ? c->m : 0; }
int rs_device(const rs_ctx* c) { return c ? c->engines[0]->device : -1; }
int rs_device_count(const rs_ctx* c) { return c ? static_cast<int>(c->engines.size()) : 0; }
int rs_device_at(const rs_ctx* c, int i) {
  return (c && i >= 0 && i < static_cast<int>(c->engines.size())) ? c->engines[static_cast<size_t>(i)]->device : -1;
}
int rs_device_launches(const rs_ctx* c, int i, uint64_t* launches) {
  if (!c || !launches || i < 0 || i >= static_cast<int>(c->engines.size())) return RS_ERR_INVALID_ARG;
  *launches = c->engines[static_cast<size_t>(i)]->launches.load(std::memory_order_relaxed);
  return RS_OK;
}
const char* rs_backend(const rs_ctx* c) { return c ? c->backend.c_str() : "none"; }
const char* rs_last_kernel(const rs_ctx* c) { return c ? c->shared.last_kernel.load() : "none"; }
const char* rs_last_kernel_on(rs_ctx* c, void* stream) { return c ? c->shared.on(as_stream(stream)) : "none"; }

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
  Engine* e = pick_engine(c);
  InflightGuard ig(e);
  DeviceScope ds(e->device);
  if (!ds.ok()) return RS_ERR_DEVICE;
  return run_object(e, static_cast<const uint8_t*>(e->d_enc_plan.p), in_idx, out_idx, shards, S);
}

int rs_reconstruct(rs_ctx* c, uint8_t* const* shards, size_t* lens) { return reconstruct_impl(c, shards, lens, false); }
int rs_reconstruct_data(rs_ctx* c, uint8_t* const* shards, size_t* lens) {
  return reconstruct_impl(c, shards, lens, true);
}

// [upstream reedsolomon.go Verify]: recompute parity on the GPU into temporary
// shards and compare on the host against the caller's parity shards.
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
  Engine* e = pick_engine(c);
  InflightGuard ig(e);
  DeviceScope ds(e->device);
  if (!ds.ok()) return RS_ERR_DEVICE;
  rc = run_object(e, static_cast<const uint8_t*>(e->d_enc_plan.p), in_idx, out_idx, view.data(), S);
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
  const Layout L{const_cast<uint8_t*>(data), data_sp, parity, parity_sp, shard_pitch};
  if (mem == RS_MEM_DEVICE) {
    Engine* e = engine_for_stream(c, as_stream(stream));
    if (!e) return RS_ERR_INVALID_ARG;
    DeviceScope ds(e->device);
    return rs::engine_encode_batch(e, data, data_sp, parity, parity_sp, shard_pitch, S, N, as_stream(stream));
  }
  if (mem != RS_MEM_HOST) return RS_ERR_INVALID_ARG;
  std::vector<int> in_slots(c->k), out_slots(c->m);
  for (int i = 0; i < c->k; ++i) in_slots[i] = i;
  for (int p = 0; p < c->m; ++p) out_slots[p] = c->k + p;
  return fan_out(c, N, static_cast<size_t>(c->k) * S, [&](Engine* e, size_t s0, size_t n) {
    return host_batch(e, L.from(s0), in_slots, out_slots, S, n, static_cast<const uint8_t*>(e->d_enc_plan.p),
                      nullptr, c->m);
  });
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
  if (n_masks != 1 && c->h_lut.empty()) return RS_ERR_NOT_SUPPORTED;
  if (mem == RS_MEM_DEVICE) {
    hipStream_t s = as_stream(stream);
    Engine* e = engine_for_stream(c, s);
    if (!e) return RS_ERR_INVALID_ARG;
    DeviceScope ds(e->device);
    rs::KernelArgs a = make_args(e, L, S, N);
    if (n_masks == 1) {
      int rc = uniform_plan(e, masks[0] & full, false, &a.plans);
      if (rc) return rc;
      return launch(e, a, max_missing, false, s);
    }
    UploadGuard ug;
    const uint32_t* dm = nullptr;
    int rc = upload_acquire(e, masks, N, s, &ug, &dm);
    if (rc) return rc;
    a.plans = static_cast<const uint8_t*>(e->d_plans.p);
    a.present_masks = dm;
    return launch(e, a, max_missing, true, s);
  }
  std::vector<int> in_slots, out_slots;
  if (n_masks == 1) {
    const uint32_t present = masks[0] & full;
    for (int i = 0; i < t; ++i) {
      if ((present >> i) & 1u) {
        if (static_cast<int>(in_slots.size()) < c->k) in_slots.push_back(i);
      } else {
        out_slots.push_back(i);
      }
    }
  }  // per-stripe patterns: host_batch_ps picks the slots from the masks
  return fan_out(c, N, static_cast<size_t>(c->k) * S, [&](Engine* e, size_t s0, size_t n) {
    const uint8_t* plan = static_cast<const uint8_t*>(e->d_plans.p);
    const uint32_t* mk = nullptr;
    if (n_masks == 1) {
      int rc = uniform_plan(e, masks[0] & full, false, &plan);
      if (rc) return rc;
    } else {
      mk = masks + s0;
    }
    return host_batch(e, L.from(s0), in_slots, out_slots, S, n, plan, mk, max_missing);
  });
}

int rs_reconstruct_batch_out(rs_ctx* c, const uint8_t* data, size_t data_sp, const uint8_t* parity, size_t parity_sp,
                             size_t shard_pitch, size_t S, size_t N, const uint32_t* masks, size_t n_masks,
                             int masks_on_device, uint8_t* out, size_t out_sp, void* stream) {
  if (!c || !data || (c->m > 0 && !parity) || !masks || !out) return RS_ERR_INVALID_ARG;
  if (N == 0) return RS_OK;
  Engine* e = engine_for_stream(c, as_stream(stream));
  if (!e) return RS_ERR_INVALID_ARG;
  DeviceScope ds(e->device);
  return rs::engine_reconstruct_batch_out(e, data, data_sp, parity, parity_sp, shard_pitch, S, N, masks, n_masks,
                                          masks_on_device, 0, out, out_sp, as_stream(stream));
}

int rs_reconstruct_batch_out_devmask(rs_ctx* c, const uint8_t* data, size_t data_sp, const uint8_t* parity,
                                     size_t parity_sp, size_t shard_pitch, size_t S, size_t N,
                                     const uint32_t* masks_dev, int max_missing, uint8_t* out, size_t out_sp,
                                     void* stream) {
  if (!c || !data || (c->m > 0 && !parity) || !masks_dev || !out) return RS_ERR_INVALID_ARG;
  if (N == 0) return RS_OK;
  Engine* e = engine_for_stream(c, as_stream(stream));
  if (!e) return RS_ERR_INVALID_ARG;
  DeviceScope ds(e->device);
  return rs::engine_reconstruct_batch_out(e, data, data_sp, parity, parity_sp, shard_pitch, S, N, masks_dev, N, 1,
                                          max_missing, out, out_sp, as_stream(stream));
}

int rs_reconstruct_batch_out_packed(rs_ctx* c, const uint8_t* data, size_t data_sp, const uint8_t* parity,
                                    size_t parity_sp, size_t shard_pitch, size_t S, size_t N, const uint32_t* masks,
                                    int masks_on_device, uint8_t* out, uint32_t* row_offsets, void* stream) {
  if (!c || !data || (c->m > 0 && !parity) || !masks || !out || !row_offsets) return RS_ERR_INVALID_ARG;
  if (N == 0) return RS_OK;
  Engine* e = engine_for_stream(c, as_stream(stream));
  if (!e) return RS_ERR_INVALID_ARG;
  DeviceScope ds(e->device);
  return rs::engine_reconstruct_batch_packed(e, data, data_sp, parity, parity_sp, shard_pitch, S, N, masks,
                                             masks_on_device, out, row_offsets, as_stream(stream));
}

int rs_verify_batch(rs_ctx* c, const uint8_t* data, size_t data_sp, const uint8_t* parity, size_t parity_sp,
                    size_t shard_pitch, size_t S, size_t N, uint32_t* bad, int mem, void* stream) {
  if (!c || !data || (c->m > 0 && !parity) || !bad) return RS_ERR_INVALID_ARG;
  if (N == 0) return RS_OK;
  if (S == 0) return RS_ERR_SHARD_NO_DATA;
  if (!batch_sizes_ok(S, N, shard_pitch) || reinterpret_cast<uintptr_t>(bad) % 4) return RS_ERR_INVALID_ARG;
  if (mem != RS_MEM_DEVICE && mem != RS_MEM_HOST) return RS_ERR_INVALID_ARG;
  if (mem == RS_MEM_DEVICE) {
    Engine* e = engine_for_stream(c, as_stream(stream));
    if (!e) return RS_ERR_INVALID_ARG;
    DeviceScope ds(e->device);
    return rs::engine_verify_batch(e, data, data_sp, parity, parity_sp, shard_pitch, S, N, bad, as_stream(stream));
  }
  if (c->m == 0) {  // nothing to verify
    std::memset(bad, 0, N * 4);
    return RS_OK;
  }
  const Layout L{const_cast<uint8_t*>(data), data_sp, const_cast<uint8_t*>(parity), parity_sp, shard_pitch};
  std::vector<int> all(c->k + c->m), none;
  for (int i = 0; i < c->k + c->m; ++i) all[i] = i;
  return fan_out(c, N, static_cast<size_t>(c->k) * S, [&](Engine* e, size_t s0, size_t n) {
    return host_batch(e, L.from(s0), all, none, S, n, nullptr, nullptr, c->m, bad + s0);
  });
}

int rs_reconstruct_batch_devmask(rs_ctx* c, uint8_t* data, size_t data_sp, uint8_t* parity, size_t parity_sp,
                                 size_t shard_pitch, size_t S, size_t N, const uint32_t* masks_dev, void* stream) {
  if (!c || !data || (c->m > 0 && !parity) || !masks_dev) return RS_ERR_INVALID_ARG;
  if (N == 0) return RS_OK;
  if (S == 0) return RS_ERR_SHARD_NO_DATA;
  if (c->h_lut.empty()) return RS_ERR_NOT_SUPPORTED;
  const Layout L{data, data_sp, parity, parity_sp, shard_pitch};
  if (!batch_sizes_ok(S, N, shard_pitch) || !device_layout_ok(L, c->m, S)) return RS_ERR_INVALID_ARG;
  Engine* e = engine_for_stream(c, as_stream(stream));
  if (!e) return RS_ERR_INVALID_ARG;
  DeviceScope ds(e->device);
  rs::KernelArgs a = make_args(e, L, S, N);
  a.plans = static_cast<const uint8_t*>(e->d_plans.p);
  a.present_masks = masks_dev;
  return launch(e, a, c->m, true, as_stream(stream));
}

// Waits for stream s; returns and clears its deferred per-stripe errors (bit 0: a
// stripe with < k present, bit 1: a stripe beyond the launch's erasure bound).
// release: also gives the stream's word back (rs_stream_release).
static int sync_stream(rs_ctx* c, void* stream, bool release) {
  if (!c) return RS_ERR_INVALID_ARG;
  hipStream_t s = as_stream(stream);
  Engine* e = engine_for_stream(c, s);
  if (!e) return RS_ERR_INVALID_ARG;
  DeviceScope ds(e->device);
  uint32_t idx;
  {
    std::lock_guard<std::mutex> g(e->status_mu);
    auto it = e->status_idx.find(s);
    if (it == e->status_idx.end()) {  // no per-stripe launch on this stream yet
      RS_HIP(hipStreamSynchronize(s));
      return RS_OK;
    }
    idx = it->second;
  }
  uint32_t* dw = status_dev(e, idx);
  volatile uint32_t* hw = status_host(e, idx);
  RS_HIP(hipMemcpyAsync(const_cast<uint32_t*>(hw), dw, 4, hipMemcpyDeviceToHost, s));
  RS_HIP(hipStreamSynchronize(s));
  const uint32_t word = *hw;
  if (word) {
    RS_HIP(hipMemsetAsync(dw, 0, 4, s));
    RS_HIP(hipStreamSynchronize(s));
  }
  if (release) {  // the word is zero and no kernel of s holds it any more
    std::lock_guard<std::mutex> g(e->status_mu);
    e->status_idx.erase(s);
    e->status_free.push_back(idx);
  }
  if (release) c->shared.forget(s);
  if (word & 1u) return RS_ERR_TOO_FEW_SHARDS;
  if (word & 2u) return RS_ERR_INVALID_ARG;
  return RS_OK;
}

int rs_sync(rs_ctx* c, void* stream) { return sync_stream(c, stream, false); }
int rs_stream_release(rs_ctx* c, void* stream) { return sync_stream(c, stream, true); }

namespace {
uint32_t count_owned(const rs_ctx* c) {
  uint32_t n = 0;
  for (const RegRange& r : c->reg) n += r.owned ? 1u : 0u;
  return n;
}

// Inserts r unless it overlaps a known range (false then).
bool reg_insert(rs_ctx* c, const RegRange& r) {
  std::unique_lock<std::shared_mutex> g(c->reg_mu);
  if (r.owned) {
    // Memory the allocator just handed out cannot be live caller memory: a caller
    // range recorded over it is stale (freed without rs_host_unregister -- harmless
    // since round 4, nothing is pinned) and gives way instead of failing the
    // allocation.
    c->reg.erase(std::remove_if(c->reg.begin(), c->reg.end(),
                                [&](const RegRange& q) { return !q.owned && q.lo < r.hi && r.lo < q.hi; }),
                 c->reg.end());
  }
  auto it = std::lower_bound(c->reg.begin(), c->reg.end(), r.lo,
                             [](const RegRange& a, uintptr_t lo) { return a.lo < lo; });
  if (it != c->reg.end() && it->lo < r.hi) return false;
  if (it != c->reg.begin() && std::prev(it)->hi > r.lo) return false;
  c->reg.insert(it, r);
  c->n_owned.store(count_owned(c), std::memory_order_release);
  return true;
}

// Removes the range starting at ptr if its ownership matches; false if none does.
bool reg_erase(rs_ctx* c, void* ptr, bool owned) {
  std::unique_lock<std::shared_mutex> g(c->reg_mu);
  const uintptr_t lo = reinterpret_cast<uintptr_t>(ptr);
  auto it = std::find_if(c->reg.begin(), c->reg.end(), [&](const RegRange& r) { return r.lo == lo; });
  if (it == c->reg.end() || it->owned != owned) return false;
  c->reg.erase(it);
  c->n_owned.store(count_owned(c), std::memory_order_release);
  return true;
}
}  // namespace

// Caller memory is recorded, not pinned or mapped (round 4).  amdgpu maps
// hipHostRegister'ed pageable memory as a user-pointer range whose pages the kernel
// may still migrate, compact or collapse into huge pages under a running kernel;
// the round-3 records show lost in-place writes and a late-reported illegal address
// right after the only tests that ran GPU work on such ranges (`HISTORY.md` §A.1).  So no
// kernel and no DMA of this library touches caller pages in place: calls on
// registered buffers are staged through the library's own page-locked memory, and
// in-place work needs rs_host_alloc.
int rs_host_register(rs_ctx* c, void* ptr, size_t bytes) {
  if (!c || !ptr || bytes == 0 || reinterpret_cast<uintptr_t>(ptr) + bytes < reinterpret_cast<uintptr_t>(ptr))
    return RS_ERR_INVALID_ARG;
  const uintptr_t lo = reinterpret_cast<uintptr_t>(ptr);
  return reg_insert(c, RegRange{lo, lo + bytes, nullptr, false}) ? RS_OK : RS_ERR_INVALID_ARG;
}

int rs_host_unregister(rs_ctx* c, void* ptr) {
  if (!c || !ptr) return RS_ERR_INVALID_ARG;
  return reg_erase(c, ptr, false) ? RS_OK : RS_ERR_INVALID_ARG;  // rs_host_alloc's are rs_host_free's
}

int rs_host_alloc(rs_ctx* c, size_t bytes, void** out) {
  if (!c || !out || bytes == 0) return RS_ERR_INVALID_ARG;
  *out = nullptr;
  Engine* e = c->engines[0].get();
  DeviceScope ds(e->device);
  if (!ds.ok()) return RS_ERR_DEVICE;
  const size_t n = round_up(bytes, 4096);
  void* p = rs::pinned_alloc(n, e->numa);
  if (!p) return RS_ERR_DEVICE;
  void* dev = nullptr;
  if (hipHostGetDevicePointer(&dev, p, 0) != hipSuccess || !dev) {
    (void)hipGetLastError();
    rs::pinned_free(p);
    return RS_ERR_DEVICE;
  }
  if (!reg_insert(c, RegRange{reinterpret_cast<uintptr_t>(p), reinterpret_cast<uintptr_t>(p) + n,
                              static_cast<uint8_t*>(dev), true})) {
    rs::pinned_free(p);  // overlaps a live owned range: the allocator's bookkeeping is broken
    return RS_ERR_INVALID_ARG;
  }
  *out = p;
  return RS_OK;
}

int rs_host_free(rs_ctx* c, void* ptr) {
  if (!c || !ptr) return RS_ERR_INVALID_ARG;
  if (!reg_erase(c, ptr, true)) return RS_ERR_INVALID_ARG;
  DeviceScope ds(c->engines[0]->device);
  rs::pinned_free(ptr);
  return RS_OK;
}

int rs_device_copy(rs_ctx* c, void* dst, const void* src, size_t bytes, void* stream) {
  if (!c || !dst || !src || bytes % 16 || reinterpret_cast<uintptr_t>(dst) % 16 ||
      reinterpret_cast<uintptr_t>(src) % 16)
    return RS_ERR_INVALID_ARG;
  Engine* e = engine_for_stream(c, as_stream(stream));
  if (!e) return RS_ERR_INVALID_ARG;
  DeviceScope ds(e->device);
  // one workgroup per CU, 4 KiB wave tasks: the best of tools/copy_probe.hip's sweep
  // (task shape x loads in flight x store policy x 1..16 workgroups per CU)
  const uint32_t grid = static_cast<uint32_t>(
      std::max<uint64_t>(1, std::min<uint64_t>(static_cast<uint64_t>(e->cu_count), (bytes + 16383) / 16384)));
  rs::launch_copy(src, dst, bytes, grid, as_stream(stream));
  c->shared.note(as_stream(stream), "copy_kernel");
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
  Engine* e = engine_for_stream(c, as_stream(stream));
  if (!e) return RS_ERR_INVALID_ARG;
  DeviceScope ds(e->device);
  const rs::Sha256Args a{base, stride, nullptr, nullptr, len, static_cast<uint32_t>(n), digests};
  if (rs::launch_sha256(a, as_stream(stream))) return RS_ERR_DEVICE;
  c->shared.note(as_stream(stream), "sha256_kernel");
  return RS_OK;
}

int rs_sha256_batch_var(rs_ctx* c, const uint8_t* base, const uint64_t* offsets, const uint64_t* lens, size_t n,
                        uint8_t* digests, void* stream) {
  if (!c || (n && (!base || !offsets || !lens || !digests)) || n > 0xFFFFFFFFu ||
      reinterpret_cast<uintptr_t>(digests) % 4)
    return RS_ERR_INVALID_ARG;
  if (n == 0) return RS_OK;
  Engine* e = engine_for_stream(c, as_stream(stream));
  if (!e) return RS_ERR_INVALID_ARG;
  DeviceScope ds(e->device);
  const rs::Sha256Args a{base, 0, offsets, lens, 0, static_cast<uint32_t>(n), digests};
  if (rs::launch_sha256(a, as_stream(stream))) return RS_ERR_DEVICE;
  c->shared.note(as_stream(stream), "sha256_kernel");
  return RS_OK;
}

int rs_set_host_zero_copy(rs_ctx* c, int enable) {
  if (!c) return RS_ERR_INVALID_ARG;
  for (auto& e : c->engines) e->host_zero_copy = enable != 0;
  return RS_OK;
}

const char* rs_last_host_path(const rs_ctx* c) { return c ? c->shared.last_host_path.load() : "none"; }

int rs_set_parity_pad_writes(rs_ctx* c, int enable) {
  if (!c) return RS_ERR_INVALID_ARG;
  for (auto& e : c->engines) e->parity_pad = enable != 0;
  return RS_OK;
}

int rs_set_out_pad_writes(rs_ctx* c, int enable) {
  if (!c) return RS_ERR_INVALID_ARG;
  for (auto& e : c->engines) e->out_pad = enable != 0;
  return RS_OK;
}

int rs_set_occupancy_cap(rs_ctx* c, int waves_per_simd) {
  if (!c || waves_per_simd < -1 || waves_per_simd > 32) return RS_ERR_INVALID_ARG;
  for (auto& e : c->engines) e->occ_cap = waves_per_simd;
  return RS_OK;
}

int rs_set_blocks_per_cu(rs_ctx* c, int bpc) {
  if (!c || bpc < 0) return RS_ERR_INVALID_ARG;
  for (auto& e : c->engines) e->blocks_per_cu = bpc;  // 0 = by shape
  return RS_OK;
}

}  // extern "C"
