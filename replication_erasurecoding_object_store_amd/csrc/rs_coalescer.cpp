// rs_coalescer.cpp -- batch coalescer behind the per-object IEcDriver calls
// (SURVEY.md §8f rank 1).
//
// The reference calls Encode / Reconstruct once per object from a goroutine per
// HTTP request (writeservice.go:218-222,382-386; readservice.go:144,285; healer
// workers poller.go:282).  One object is a few KiB to a few MiB -- far too little
// to fill an MI355X, and each call alone pays a full H2D -> kernel -> D2H round
// trip.  The coalescer keeps the per-object contract (same arguments, same checks
// and error codes as rs_encode / rs_reconstruct / rs_reconstruct_data / rs_verify)
// but parks concurrent calls with the same shard length in one staging batch and
// runs the batch as ONE device launch:
//
//   caller i:  validate -> reserve slot i of the open batch for its S -> copy its
//              shards into the batch's pinned staging (callers copy in parallel)
//   leader  :  the batch's first caller waits until the batch is full or
//              max_wait_us has passed, closes it, then moves it:
//              H2D (data [n,K,P] (+ parity [n,M,P] if a reconstruct needs it) +
//              masks) -> rs_reconstruct_batch_out with per-stripe masks (an encode
//              is the pattern "all parity missing") or rs_verify_batch -> D2H
//   caller i:  copies its outputs out of the staging batch and returns.
//
// Up to `inflight` batches exist at once (each with its own stream, pinned and
// device slab), so one batch's transfers overlap the next batch's filling.  All
// arithmetic is the device kernels'; the host only moves bytes.
//
// A context spanning several GPUs (rs_create_multi) gives each GPU its own
// batches: batch i belongs to engine i % n_engines, with its pinned staging on that
// GPU's NUMA node and its stream / slab on that GPU.  A new batch is opened on the
// engine with the fewest batches open or executing, so concurrent callers spread
// over every GPU while a lone caller still sees one batch at a time.
#include <hip/hip_runtime.h>
#include <linux/futex.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <climits>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <thread>
#include <utility>
#include <vector>

#include "../../include/rsgpu.h"
#include "rs_engine.hpp"
#include "rs_host_util.hpp"

namespace {

using Clock = std::chrono::steady_clock;

enum class Kind : int { kApply = 0, kVerify = 1 };

// Slot reservation is one CAS on `ticket` = [generation:24 | closed:1 | count:39].
// A batch is opened (generation bumped, count 0) under rs_coalescer::mu; from then
// on callers of its shard length reserve slots WITHOUT the mutex (through
// rs_coalescer::hot or the open map) until it is closed -- full, or by its leader.
// With callers outnumbering cores, a reservation mutex convoys: a preempted holder
// stalls every caller behind it.
constexpr uint64_t kClosedBit = 1ull << 39;
constexpr uint64_t kCountMask = kClosedBit - 1;
constexpr int kGenShift = 40;

struct Batch {
  int index = 0;               // position in rs_coalescer::batches (the hot-slot id)
  int engine = 0;              // the GPU (engine index in the context) this batch runs on
  bool free = true;            // guarded by rs_coalescer::mu
  uint32_t gen = 0;            // generation of the current / last open period (mu)
  Kind kind = Kind::kApply;
  size_t S = 0, P = 0;
  std::atomic<size_t> cap{0};
  std::atomic<int> key_kind{-1};      // (kind, S) of the current generation, published
  std::atomic<uint64_t> key_S{0};     //   before `ticket` (read racily by the fast path)
  std::atomic<uint64_t> ticket{kClosedBit};
  std::atomic<uint32_t> parity_in{0};  // some slot needs its parity shards uploaded
  size_t n_final = 0;          // slots of the closed batch (published by done_gen)
  int rc = RS_OK;              // published by done_gen
  Clock::time_point deadline;
  // Lock-free completion: callers stage, wait and drain without the mutex, so a
  // finished batch of n callers does not turn into a convoy of n lock handoffs.
  std::atomic<uint32_t> filled{0};    // slots staged
  std::atomic<uint32_t> released{0};  // slots drained
  std::atomic<uint32_t> done_gen{0};  // bumped (and futex-woken) when a run finishes
  hipStream_t stream = nullptr;
  rs::PinnedBuf host;
  rs::DevBuf dev;
  // region offsets (same in host staging and device slab)
  size_t o_data = 0, o_parity = 0, o_out = 0, o_masks = 0, o_bad = 0, bytes = 0;
};

// Reserves up to `want` consecutive slots of batch b in generation gen.
// Returns the number taken (0: closed, full or another generation).
size_t try_reserve(Batch* b, uint32_t gen, size_t want, size_t* slot0) {
  uint64_t t = b->ticket.load(std::memory_order_acquire);
  for (;;) {
    const size_t cap = b->cap.load(std::memory_order_relaxed);
    const size_t cnt = static_cast<size_t>(t & kCountMask);
    if (static_cast<uint32_t>(t >> kGenShift) != (gen & 0xFFFFFFu) || (t & kClosedBit) || cnt >= cap) return 0;
    const size_t take = std::min(want, cap - cnt);
    if (b->ticket.compare_exchange_weak(t, t + take, std::memory_order_acq_rel, std::memory_order_acquire)) {
      *slot0 = cnt;
      return take;
    }
  }
}

static_assert(sizeof(std::atomic<uint32_t>) == sizeof(uint32_t), "futex word");

void futex_wait(std::atomic<uint32_t>* w, uint32_t expected) {
  syscall(SYS_futex, reinterpret_cast<uint32_t*>(w), FUTEX_WAIT_PRIVATE, expected, nullptr, nullptr, 0);
}
void futex_wake_all(std::atomic<uint32_t>* w) {
  syscall(SYS_futex, reinterpret_cast<uint32_t*>(w), FUTEX_WAKE_PRIVATE, INT_MAX, nullptr, nullptr, 0);
}
// Waits until *w != v: a brief spin, then sleeps (callers may far outnumber cores,
// so spinning long would steal the CPU the stragglers need to stage their shards).
void wait_change(std::atomic<uint32_t>* w, uint32_t v) {
  for (int i = 0; i < 64; ++i) {
    if (w->load(std::memory_order_acquire) != v) return;
    __builtin_ia32_pause();
  }
  while (w->load(std::memory_order_acquire) == v) futex_wait(w, v);
}

}  // namespace

struct rs_coalescer {
  rs_ctx* ctx = nullptr;
  int k = 0, m = 0;
  bool per_stripe = false;  // k+m <= 16: per-stripe masks (reconstruct coalesces)
  size_t max_batch = 0, max_bytes = 0;
  std::chrono::microseconds max_wait{0};

  int max_exec = 2;   // batches on one device at once
  bool zero_copy = true;

  std::mutex mu;
  std::condition_variable free_cv;    // a batch became free (or opened)
  std::condition_variable leader_cv;  // batch full / an execution slot freed
  std::vector<std::unique_ptr<Batch>> batches;
  std::vector<Batch*> free_list;
  std::vector<int> engine_load;   // batches open or executing per engine (mu)
  std::vector<int> engine_exec;   // batches executing per engine (mu)
  std::map<std::pair<int, size_t>, Batch*> open;  // (kind, S) -> batch accepting slots (mu)
  std::atomic<uint64_t> hot{0};  // last opened batch: hot_word(gen, index); 0 = none

  std::atomic<uint64_t> calls{0}, n_batches{0}, stripes{0}, max_seen{0};

  ~rs_coalescer() {
    for (auto& b : batches) {
      rs::DeviceScope ds(rs::engine_device(rs::ctx_engine(ctx, b->engine)));
      if (b->stream) (void)hipStreamDestroy(b->stream);
      b.reset();  // slabs freed on their device
    }
  }
};

namespace {

using rs::round_up;

uint8_t* host_at(Batch* b, size_t off) { return static_cast<uint8_t*>(b->host.p) + off; }
uint8_t* dev_at(Batch* b, size_t off) { return static_cast<uint8_t*>(b->dev.p) + off; }

// Lays out a batch for (kind, S) and makes sure its buffers are large enough.
int prepare(rs_coalescer* co, Batch* b, Kind kind, size_t S) {
  const size_t k = co->k, m = co->m;
  b->kind = kind;
  b->S = S;
  b->P = round_up(S, 16);  // kernel contract: 16-B aligned slots
  rs::DeviceScope ds(rs::engine_device(rs::ctx_engine(co->ctx, b->engine)));
  const size_t per = b->P * (k + 2 * m) + 8;
  const size_t cap = std::max<size_t>(1, std::min(co->max_batch, co->max_bytes / per));
  b->cap.store(cap, std::memory_order_relaxed);
  b->o_data = 0;
  b->o_parity = round_up(cap * k * b->P, 256);
  b->o_out = b->o_parity + round_up(cap * m * b->P, 256);
  b->o_masks = b->o_out + round_up(cap * m * b->P, 256);
  b->o_bad = b->o_masks + round_up(cap * 4, 256);
  b->bytes = b->o_bad + round_up(cap * 4, 256);
  if (!b->stream) RS_HIP(hipStreamCreateWithFlags(&b->stream, hipStreamNonBlocking));
  if (b->host.ensure(b->bytes) || b->dev.ensure(b->bytes)) return RS_ERR_DEVICE;
  b->filled.store(0, std::memory_order_relaxed);
  b->released.store(0, std::memory_order_relaxed);
  b->parity_in.store(0, std::memory_order_relaxed);
  b->rc = RS_OK;
  b->free = false;
  b->deadline = Clock::now() + co->max_wait;
  b->gen = (b->gen + 1) & 0xFFFFFFu;
  b->key_kind.store(static_cast<int>(kind), std::memory_order_relaxed);
  b->key_S.store(S, std::memory_order_relaxed);
  b->ticket.store(static_cast<uint64_t>(b->gen) << kGenShift, std::memory_order_release);  // open, count 0
  return RS_OK;
}

// Runs a closed batch of n slots on its engine's stream and waits for the outputs.
int execute(rs_coalescer* co, Batch* b, size_t n) {
  const size_t k = co->k, m = co->m, P = b->P;
  rs::Engine* eng = rs::ctx_engine(co->ctx, b->engine);
  rs::DeviceScope ds(rs::engine_device(eng));
  hipStream_t st = b->stream;
  // Zero-copy (default): the staging is pinned host memory the GPU can address, so
  // the kernel reads the staged shards and writes its outputs there directly --
  // one launch + one sync per batch instead of 3-4 DMA round trips.
  void* hd = nullptr;
  const bool zc = co->zero_copy && hipHostGetDevicePointer(&hd, b->host.p, 0) == hipSuccess && hd;
  if (!zc) (void)hipGetLastError();
  uint8_t* base = zc ? static_cast<uint8_t*>(hd) : static_cast<uint8_t*>(b->dev.p);
  auto at = [&](size_t off) { return base + off; };
  if (!zc) {
    RS_HIP(hipMemcpyAsync(dev_at(b, b->o_data), host_at(b, b->o_data), n * k * P, hipMemcpyHostToDevice, st));
    if (b->parity_in.load(std::memory_order_relaxed) || b->kind == Kind::kVerify)
      RS_HIP(hipMemcpyAsync(dev_at(b, b->o_parity), host_at(b, b->o_parity), n * m * P, hipMemcpyHostToDevice, st));
    if (b->kind == Kind::kApply && co->per_stripe)
      RS_HIP(hipMemcpyAsync(dev_at(b, b->o_masks), host_at(b, b->o_masks), n * 4, hipMemcpyHostToDevice, st));
  }
  int rc;
  if (b->kind == Kind::kVerify) {
    // the mismatch words are OR-ed atomically: keep them in HBM, copy them back
    rc = rs::engine_verify_batch(eng, at(b->o_data), k * P, at(b->o_parity), m * P, P, b->S, n,
                                 reinterpret_cast<uint32_t*>(dev_at(b, b->o_bad)), st);
    if (rc) return rc;
    RS_HIP(hipMemcpyAsync(host_at(b, b->o_bad), dev_at(b, b->o_bad), n * 4, hipMemcpyDeviceToHost, st));
  } else {
    if (co->per_stripe) {
      rc = rs::engine_reconstruct_batch_out(eng, at(b->o_data), k * P, at(b->o_parity), m * P, P, b->S, n,
                                            reinterpret_cast<const uint32_t*>(at(b->o_masks)), n, 1, at(b->o_out),
                                            m * P, st);
    } else {  // encode-only batches (k+m > 16): parity straight into the out region
      rc = rs::engine_encode_batch(eng, at(b->o_data), k * P, at(b->o_out), m * P, P, b->S, n, st);
    }
    if (rc) return rc;
    if (!zc)
      RS_HIP(hipMemcpyAsync(host_at(b, b->o_out), dev_at(b, b->o_out), n * m * P, hipMemcpyDeviceToHost, st));
  }
  RS_HIP(hipStreamSynchronize(st));
  return RS_OK;  // every mask was checked (>= k present) before it was staged
}

// One call through the coalescer.  fill(b, slot) stages the inputs, drain(b, slot)
// copies the outputs back; both run outside the lock, in the caller's thread.
//
// Batching is group commit: a batch's leader starts it as soon as an execution slot
// is free (at most max_exec batches on the device at once) and max_wait has passed
// since the batch opened (default 0).  Callers that arrive while earlier batches
// are on the device pile into the open batch, so batches grow with the load and a
// lone caller pays no timer.
uint64_t hot_word(uint32_t gen, int index) {
  return (static_cast<uint64_t>(gen) << 16) | static_cast<uint64_t>(index + 1);
}

// Takes batch b (generation gen) out of the open map / hot slot (under mu).
void unpublish(rs_coalescer* co, Batch* b, uint32_t gen) {
  const auto key = std::make_pair(static_cast<int>(b->kind), b->S);
  auto it = co->open.find(key);
  if (it != co->open.end() && it->second == b) co->open.erase(it);
  uint64_t h = co->hot.load(std::memory_order_relaxed);
  const uint64_t mine = hot_word(gen, b->index);
  if (h == mine) co->hot.compare_exchange_strong(h, 0, std::memory_order_relaxed);
}

template <class Fill, class Drain>
int submit_many(rs_coalescer* co, Kind kind, size_t S, size_t count, bool parity_in, Fill&& fill, Drain&& drain) {
  const auto key = std::make_pair(static_cast<int>(kind), S);
  int result = RS_OK;
  size_t done_items = 0;
  while (done_items < count) {
    const size_t want = count - done_items;
    Batch* b = nullptr;
    uint32_t gen = 0;
    size_t slot0 = 0, take = 0;
    // fast path: the most recently opened batch, no mutex
    if (const uint64_t h = co->hot.load(std::memory_order_acquire)) {
      Batch* hb = co->batches[(h & 0xFFFF) - 1].get();
      const uint32_t hg = static_cast<uint32_t>(h >> 16);
      if (hb->key_kind.load(std::memory_order_relaxed) == key.first &&
          hb->key_S.load(std::memory_order_relaxed) == key.second && (take = try_reserve(hb, hg, want, &slot0))) {
        b = hb;
        gen = hg;
      }
    }
    std::unique_lock<std::mutex> lk(co->mu, std::defer_lock);
    if (!b) {
      lk.lock();
      for (;;) {
        auto it = co->open.find(key);
        if (it != co->open.end()) {
          Batch* ob = it->second;
          if ((take = try_reserve(ob, ob->gen, want, &slot0))) {
            b = ob;
            gen = ob->gen;
            break;
          }
          co->open.erase(it);  // closed or full: stop offering it
          continue;
        }
        if (!co->free_list.empty()) {
          // the free batch of the least-loaded engine (the most recently freed one
          // among equals: its staging is warm)
          size_t pick = co->free_list.size() - 1;
          for (size_t i = co->free_list.size(); i-- > 0;)
            if (co->engine_load[co->free_list[i]->engine] < co->engine_load[co->free_list[pick]->engine]) pick = i;
          Batch* nb = co->free_list[pick];
          co->free_list.erase(co->free_list.begin() + static_cast<std::ptrdiff_t>(pick));
          const int rc = prepare(co, nb, kind, S);
          if (rc) {
            nb->free = true;
            co->free_list.push_back(nb);
            co->free_cv.notify_all();
            return rc;
          }
          ++co->engine_load[nb->engine];
          take = try_reserve(nb, nb->gen, want, &slot0);  // slot 0: this caller leads
          b = nb;
          gen = nb->gen;
          co->open[key] = nb;
          co->hot.store(hot_word(gen, nb->index), std::memory_order_release);
          co->free_cv.notify_all();  // waiters for this S may join it
          break;
        }
        co->free_cv.wait(lk);  // every batch is in flight: back-pressure
      }
      lk.unlock();
    }
    const bool leader = slot0 == 0;
    const uint32_t dgen = b->done_gen.load(std::memory_order_relaxed);
    if (parity_in) b->parity_in.store(1, std::memory_order_relaxed);
    if (slot0 + take == b->cap.load(std::memory_order_relaxed)) {  // took the last slot: close it
      b->ticket.fetch_or(kClosedBit, std::memory_order_acq_rel);
      lk.lock();
      unpublish(co, b, gen);
      co->leader_cv.notify_all();
      lk.unlock();
    }
    for (size_t j = 0; j < take; ++j) fill(b, slot0 + j, done_items + j);
    b->filled.fetch_add(static_cast<uint32_t>(take), std::memory_order_release);
    if (leader) {
      lk.lock();
      // gather: until full, or (an execution slot is free and the linger is over)
      int& exec = co->engine_exec[b->engine];
      for (;;) {
        if (b->ticket.load(std::memory_order_acquire) & kClosedBit) break;
        const bool slot_free = exec < co->max_exec;
        if (slot_free && Clock::now() >= b->deadline) break;
        if (slot_free)
          co->leader_cv.wait_until(lk, b->deadline);
        else
          co->leader_cv.wait(lk);
      }
      const uint64_t t = b->ticket.fetch_or(kClosedBit, std::memory_order_acq_rel);
      const size_t n = static_cast<size_t>(t & kCountMask);
      unpublish(co, b, gen);
      while (exec >= co->max_exec) co->leader_cv.wait(lk);
      ++exec;
      lk.unlock();
      while (b->filled.load(std::memory_order_acquire) < n) std::this_thread::yield();  // stragglers staging
      b->n_final = n;
      const int rc = execute(co, b, n);
      co->n_batches.fetch_add(1, std::memory_order_relaxed);
      co->stripes.fetch_add(n, std::memory_order_relaxed);
      uint64_t seen = co->max_seen.load(std::memory_order_relaxed);
      while (n > seen && !co->max_seen.compare_exchange_weak(seen, n)) {
      }
      lk.lock();
      --exec;
      co->leader_cv.notify_all();  // an execution slot is free
      lk.unlock();
      b->rc = rc;
      b->done_gen.fetch_add(1, std::memory_order_release);
      futex_wake_all(&b->done_gen);
    } else {
      wait_change(&b->done_gen, dgen);
    }
    const int rc = b->rc;
    const size_t n = b->n_final;  // published by done_gen
    if (rc == RS_OK)
      for (size_t j = 0; j < take; ++j) drain(b, slot0 + j, done_items + j);
    else if (result == RS_OK)
      result = rc;
    if (b->released.fetch_add(static_cast<uint32_t>(take), std::memory_order_acq_rel) + take == n) {
      lk.lock();
      b->free = true;
      --co->engine_load[b->engine];
      co->free_list.push_back(b);
      co->free_cv.notify_all();
      lk.unlock();
    }
    done_items += take;
  }
  return result;
}

// One object (the per-call IEcDriver entry points).
template <class Fill, class Drain>
int submit(rs_coalescer* co, Kind kind, size_t S, bool parity_in, Fill&& fill, Drain&& drain) {
  co->calls.fetch_add(1, std::memory_order_relaxed);
  return submit_many(
      co, kind, S, 1, parity_in, [&](Batch* b, size_t slot, size_t) { fill(b, slot); },
      [&](Batch* b, size_t slot, size_t) { drain(b, slot); });
}

// Reconstruct / ReconstructData through the coalescer; semantics of
// reconstruct_impl in rs_engine.cpp ([upstream reedsolomon.go reconstruct]).
struct RecItem {
  uint8_t* const* shards = nullptr;
  size_t* lens = nullptr;
  size_t S = 0;
  uint32_t present = 0;
  bool parity_used = false;  // a parity shard is among the k survivors
};

// Checks one object; *need = false when there is nothing to do (rc RS_OK).
int rec_check(const rs_coalescer* co, uint8_t* const* shards, size_t* lens, bool data_only, RecItem* it,
              bool* need) {
  const int k = co->k, m = co->m, t = k + m;
  *need = false;
  if (!shards || !lens) return RS_ERR_INVALID_ARG;
  size_t S = 0;
  int rc = rs::check_shards(t, lens, true, &S);
  if (rc) return rc;
  uint32_t present = 0;
  int np = 0, data_present = 0;
  for (int i = 0; i < t; ++i)
    if (lens[i]) {
      present |= 1u << i;
      ++np;
      if (i < k) ++data_present;
    }
  if (np == t || (data_only && data_present == k)) return RS_OK;
  if (np < k) return RS_ERR_TOO_FEW_SHARDS;
  if (S > 0xFFFFFFF0u) return RS_ERR_INVALID_ARG;
  for (int i = 0; i < t; ++i)
    if (!lens[i] && (!data_only || i < k) && !shards[i]) return RS_ERR_INVALID_ARG;
  it->shards = shards;
  it->lens = lens;
  it->S = S;
  it->present = present;
  it->parity_used = false;
  for (int i = 0, used = 0; i < t && used < k; ++i)  // survivors = first k present
    if (lens[i]) {
      ++used;
      if (i >= k) it->parity_used = true;
    }
  (void)m;
  *need = true;
  return RS_OK;
}

void rec_fill(const rs_coalescer* co, Batch* b, size_t slot, const RecItem& it) {
  const int k = co->k, m = co->m, t = k + m;
  const size_t P = b->P;
  for (int i = 0, staged = 0; i < t && staged < k; ++i) {  // the k survivors only
    if (!it.lens[i]) continue;
    ++staged;
    uint8_t* dst = i < k ? host_at(b, b->o_data + (slot * k + i) * P) : host_at(b, b->o_parity + (slot * m + (i - k)) * P);
    std::memcpy(dst, it.shards[i], it.S);
  }
  reinterpret_cast<uint32_t*>(host_at(b, b->o_masks))[slot] = it.present;
}

void rec_drain(const rs_coalescer* co, Batch* b, size_t slot, const RecItem& it, bool data_only) {
  const int k = co->k, m = co->m, t = k + m;
  int r = 0;  // r-th missing shard (index order, data before parity) = out slot r
  for (int i = 0; i < t; ++i) {
    if (it.lens[i]) continue;
    if (!data_only || i < k) {
      std::memcpy(it.shards[i], host_at(b, b->o_out + (slot * m + r) * b->P), it.S);
      it.lens[i] = it.S;
    }
    ++r;
  }
}

int co_reconstruct(rs_coalescer* co, uint8_t* const* shards, size_t* lens, bool data_only) {
  if (!co || !shards || !lens) return RS_ERR_INVALID_ARG;
  if (!co->per_stripe)
    return data_only ? rs_reconstruct_data(co->ctx, shards, lens) : rs_reconstruct(co->ctx, shards, lens);
  RecItem it;
  bool need = false;
  const int rc = rec_check(co, shards, lens, data_only, &it, &need);
  if (rc || !need) return rc;
  return submit(
      co, Kind::kApply, it.S, it.parity_used, [&](Batch* b, size_t slot) { rec_fill(co, b, slot, it); },
      [&](Batch* b, size_t slot) { rec_drain(co, b, slot, it, data_only); });
}

}  // namespace

extern "C" {

int rs_coalescer_create(rs_ctx* ctx, const rs_coalescer_opts* opts, rs_coalescer** out) {
  if (!ctx || !out) return RS_ERR_INVALID_ARG;
  *out = nullptr;
  const int ne = rs::ctx_engine_count(ctx);
  rs_coalescer_opts o{4096, 0, std::max(16, 8 * ne), size_t(32) << 20, 2, 0};
  if (opts) {
    if (opts->max_batch) o.max_batch = opts->max_batch;
    o.max_wait_us = opts->max_wait_us;
    if (opts->inflight > 0) o.inflight = opts->inflight;
    if (opts->max_batch_bytes) o.max_batch_bytes = opts->max_batch_bytes;
    if (opts->max_exec > 0) o.max_exec = opts->max_exec;
    o.staged_dma = opts->staged_dma;
  }
  if (o.inflight > 256 || o.max_exec > o.inflight || o.inflight < ne) return RS_ERR_INVALID_ARG;
  auto co = std::make_unique<rs_coalescer>();
  co->ctx = ctx;
  co->k = rs_data_shards(ctx);
  co->m = rs_parity_shards(ctx);
  co->per_stripe = co->k + co->m <= 16;
  co->max_batch = o.max_batch;
  co->max_bytes = o.max_batch_bytes;
  co->max_wait = std::chrono::microseconds(o.max_wait_us);
  co->max_exec = o.max_exec;
  co->zero_copy = o.staged_dma == 0;
  co->engine_load.assign(static_cast<size_t>(ne), 0);
  co->engine_exec.assign(static_cast<size_t>(ne), 0);
  for (int i = 0; i < o.inflight; ++i) {
    co->batches.push_back(std::make_unique<Batch>());
    Batch* b = co->batches.back().get();
    b->index = i;
    b->engine = i % ne;
    b->host.numa = rs::device_numa_node(rs::engine_device(rs::ctx_engine(ctx, b->engine)));
    co->free_list.push_back(b);
  }
  *out = co.release();
  return RS_OK;
}

void rs_coalescer_destroy(rs_coalescer* co) { delete co; }

int rs_co_encode(rs_coalescer* co, uint8_t* const* shards, const size_t* lens) {
  if (!co || !shards || !lens) return RS_ERR_INVALID_ARG;
  const int k = co->k, m = co->m;
  size_t S = 0;
  int rc = rs::check_shards(k + m, lens, false, &S);
  if (rc) return rc;
  if (m == 0) return RS_OK;
  for (int i = 0; i < k + m; ++i)
    if (!shards[i]) return RS_ERR_INVALID_ARG;
  if (S > 0xFFFFFFF0u) return RS_ERR_INVALID_ARG;
  const uint32_t data_mask = (1u << k) - 1u;  // parity all missing -> encode rows
  auto fill = [&](Batch* b, size_t slot) {
    for (int c = 0; c < k; ++c) std::memcpy(host_at(b, b->o_data + (slot * k + c) * b->P), shards[c], S);
    reinterpret_cast<uint32_t*>(host_at(b, b->o_masks))[slot] = data_mask;
  };
  auto drain = [&](Batch* b, size_t slot) {
    for (int r = 0; r < m; ++r) std::memcpy(shards[k + r], host_at(b, b->o_out + (slot * m + r) * b->P), S);
  };
  return submit(co, Kind::kApply, S, false, fill, drain);
}

int rs_co_reconstruct(rs_coalescer* co, uint8_t* const* shards, size_t* lens) {
  return co_reconstruct(co, shards, lens, false);
}

int rs_co_reconstruct_data(rs_coalescer* co, uint8_t* const* shards, size_t* lens) {
  return co_reconstruct(co, shards, lens, true);
}

int rs_co_verify(rs_coalescer* co, uint8_t* const* shards, const size_t* lens, int* ok) {
  if (!co || !shards || !lens || !ok) return RS_ERR_INVALID_ARG;
  const int k = co->k, m = co->m;
  size_t S = 0;
  int rc = rs::check_shards(k + m, lens, false, &S);
  if (rc) return rc;
  *ok = 1;
  if (m == 0) return RS_OK;
  for (int i = 0; i < k + m; ++i)
    if (!shards[i]) return RS_ERR_INVALID_ARG;
  if (S > 0xFFFFFFF0u) return RS_ERR_INVALID_ARG;
  auto fill = [&](Batch* b, size_t slot) {
    for (int c = 0; c < k; ++c) std::memcpy(host_at(b, b->o_data + (slot * k + c) * b->P), shards[c], S);
    for (int r = 0; r < m; ++r) std::memcpy(host_at(b, b->o_parity + (slot * m + r) * b->P), shards[k + r], S);
  };
  auto drain = [&](Batch* b, size_t slot) { *ok = reinterpret_cast<uint32_t*>(host_at(b, b->o_bad))[slot] == 0; };
  return submit(co, Kind::kVerify, S, true, fill, drain);
}

// Batched healer repair: the objects a scan found damaged
// (poller.go:227-309 audits one object per goroutine, 10 at a time) go through in
// as few device batches as their shard lengths allow.  Per object exactly
// rs_reconstruct's contract; its code lands in rcs[i].
int rs_co_reconstruct_many(rs_coalescer* co, size_t n_objects, uint8_t* const* shards, size_t* lens, int* rcs) {
  if (!co || (n_objects && (!shards || !lens || !rcs))) return RS_ERR_INVALID_ARG;
  const size_t t = static_cast<size_t>(co->k + co->m);
  co->calls.fetch_add(n_objects, std::memory_order_relaxed);
  if (!co->per_stripe) {
    for (size_t i = 0; i < n_objects; ++i) rcs[i] = rs_reconstruct(co->ctx, shards + i * t, lens + i * t);
    return RS_OK;
  }
  std::vector<RecItem> items(n_objects);
  std::map<size_t, std::vector<size_t>> by_len;
  for (size_t i = 0; i < n_objects; ++i) {
    bool need = false;
    rcs[i] = rec_check(co, shards + i * t, lens + i * t, false, &items[i], &need);
    if (need) by_len[items[i].S].push_back(i);
  }
  for (auto& g : by_len) {
    const std::vector<size_t>& idx = g.second;
    bool parity_in = false;
    for (size_t i : idx) parity_in |= items[i].parity_used;
    const int rc = submit_many(
        co, Kind::kApply, g.first, idx.size(), parity_in,
        [&](Batch* b, size_t slot, size_t j) { rec_fill(co, b, slot, items[idx[j]]); },
        [&](Batch* b, size_t slot, size_t j) { rec_drain(co, b, slot, items[idx[j]], false); });
    if (rc) {
      for (size_t i : idx)
        if (rcs[i] == RS_OK) rcs[i] = rc;  // device failure: the whole group
      return rc;
    }
  }
  return RS_OK;
}

// Bulk encode of many objects (e.g. a batch of writes): per object rs_encode's
// contract, results in rcs[i].
int rs_co_encode_many(rs_coalescer* co, size_t n_objects, uint8_t* const* shards, const size_t* lens, int* rcs) {
  if (!co || (n_objects && (!shards || !lens || !rcs))) return RS_ERR_INVALID_ARG;
  const int k = co->k, m = co->m;
  const size_t t = static_cast<size_t>(k + m);
  co->calls.fetch_add(n_objects, std::memory_order_relaxed);
  std::vector<size_t> Ss(n_objects, 0);
  std::map<size_t, std::vector<size_t>> by_len;
  for (size_t i = 0; i < n_objects; ++i) {
    size_t S = 0;
    int rc = rs::check_shards(k + m, lens + i * t, false, &S);
    for (size_t j = 0; rc == RS_OK && j < t; ++j)
      if (!shards[i * t + j]) rc = RS_ERR_INVALID_ARG;
    if (rc == RS_OK && S > 0xFFFFFFF0u) rc = RS_ERR_INVALID_ARG;
    rcs[i] = rc;
    Ss[i] = S;
    if (rc == RS_OK && m > 0) by_len[S].push_back(i);
  }
  const uint32_t data_mask = (1u << k) - 1u;
  for (auto& g : by_len) {
    const std::vector<size_t>& idx = g.second;
    const size_t S = g.first;
    const int rc = submit_many(
        co, Kind::kApply, S, idx.size(), false,
        [&](Batch* b, size_t slot, size_t j) {
          uint8_t* const* sh = shards + idx[j] * t;
          for (int c = 0; c < k; ++c) std::memcpy(host_at(b, b->o_data + (slot * k + c) * b->P), sh[c], S);
          reinterpret_cast<uint32_t*>(host_at(b, b->o_masks))[slot] = data_mask;
        },
        [&](Batch* b, size_t slot, size_t j) {
          uint8_t* const* sh = shards + idx[j] * t;
          for (int r = 0; r < m; ++r) std::memcpy(sh[k + r], host_at(b, b->o_out + (slot * m + r) * b->P), S);
        });
    if (rc) {
      for (size_t i : idx) rcs[i] = rc;
      return rc;
    }
  }
  return RS_OK;
}

int rs_co_stats(rs_coalescer* co, uint64_t* calls, uint64_t* batches, uint64_t* stripes, uint64_t* max_batch) {
  if (!co) return RS_ERR_INVALID_ARG;
  if (calls) *calls = co->calls.load();
  if (batches) *batches = co->n_batches.load();
  if (stripes) *stripes = co->stripes.load();
  if (max_batch) *max_batch = co->max_seen.load();
  return RS_OK;
}

}  // extern "C"
