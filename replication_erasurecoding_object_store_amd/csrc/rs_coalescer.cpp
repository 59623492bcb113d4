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
//              -> sleep on the batch's completion word
//   launcher:  (one thread per GPU) closes an open batch once fewer than max_exec
//              of its GPU's batches are executing (group commit; optional
//              max_wait_us linger) or it is full, and enqueues it: kernel on the
//              pinned staging in place (zero-copy) or H2D -> kernel -> D2H
//   completer: (one thread per GPU) waits for each launched batch and wakes its
//              callers, who copy their outputs out of the staging and return.
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
#include <sched.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <climits>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <thread>
#include <type_traits>
#include <utility>
#include <vector>

#include "../../include/rsgpu.h"
#include "rs_engine.hpp"
#include "rs_host_util.hpp"
#include "rs_sha256.hpp"

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

struct Batch;

// How one reservation is staged, published in its slots right after the slots are
// reserved: if the caller is descheduled before it has staged them, the launcher
// stages them itself (the caller's buffers stay valid -- it is blocked in the call
// until its batch completes) instead of holding the whole batch for it.  Both may
// copy the same bytes into the same slot; the per-slot state decides who counts it.
struct FillReq {
  void (*fn)(const void* ctx, Batch* b, size_t slot, size_t item);
  const void* ctx;
  size_t slot0, item0;  // the reservation's first slot and item index
};
constexpr uint32_t kSlotReserved = 0;   // reserved, FillReq not yet published
constexpr uint32_t kSlotPublished = 1;  // FillReq published, not yet staged
constexpr uint32_t kSlotStaged = 2;     // staged by its caller
constexpr uint32_t kSlotTaken = 3;      // staged by the launcher

constexpr int kMaxAsyncOut = 16;  // m <= 16 (rs_create)

// Where an asynchronous call's outputs go (its shard buffers, kept valid by the
// caller until rs_co_reap reports its tag).
struct AsyncRec {
  uint64_t tag = 0;
  uint32_t slot = 0;           // the call's slot in its batch
  uint32_t n_out = 0;          // outputs: out slot r of the batch -> out[r]
  uint8_t* out[kMaxAsyncOut] = {};
  uint8_t* digest = nullptr;   // encode + hash: 32 bytes
};

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
  std::atomic<uint32_t> fill_err{0};   // a slot's plan could not be resolved (plan mode)
  std::atomic<uint32_t> max_missing{0};  // most shards any slot fills: the launch's erasure bound
  std::atomic<uint32_t> hash_in{0};      // some slot wants the SHA-256 of its value (cold_hash)
  std::atomic<uint32_t> direct_in{0};    // some slot is addressed in place in the caller's rs_host_alloc'ed buffers
  uint8_t* host_dev = nullptr;           // zero-copy: GPU address of the pinned staging
  // asynchronous calls of the current run: their records, how many were made, how
  // many have been handed to reapers (under rs_coalescer::done_mu)
  std::unique_ptr<AsyncRec[]> arec;
  size_t arec_cap = 0;
  std::atomic<uint32_t> n_async{0};
  uint32_t async_cursor = 0;
  size_t n_final = 0;          // slots of the closed batch (published by the group words)
  int rc = RS_OK;              // published by the group words
  Clock::time_point deadline;
  // Lock-free completion: callers stage, wait and drain without the mutex, so a
  // finished batch of n callers does not turn into a convoy of n lock handoffs.
  std::atomic<uint32_t> filled{0};    // slots staged
  std::atomic<uint32_t> released{0};  // slots drained
  // Completion words, one per group of kGroup slots, each holding the epoch of the
  // last batch run that finished for that group.  A caller sleeps on its first
  // slot's group word until it reaches the caller's epoch (and marks the group as
  // having a waiter of that epoch).  Groups are woken in order from `wake`
  // ([epoch:32 | next group:32]): the completer wakes until two groups with
  // waiters are up, then every woken caller does the same, so waking a batch of n
  // callers costs the completer two groups' wake-ups instead of n and the rest fan
  // out over the woken threads.  Groups nobody sleeps on (slots of a multi-object
  // call) are advanced in passing and never end the chain.
  //
  // Everything is epoch-tagged because a waker may still be in the chain when the
  // batch has drained, been recycled and reopened: a claim on `wake` succeeds only
  // in the waker's own epoch, and group words only move forward, so a late waker
  // can neither wake callers of a newer run early nor move a word back.
  static constexpr uint32_t kGroup = 8;
  uint32_t epoch = 0;                 // of the current open period (set in prepare, mu)
  uint32_t n_groups_alloc = 0;        // fixed at creation: ceil(max cap / kGroup)
  std::unique_ptr<std::atomic<uint32_t>[]> grp;
  std::unique_ptr<std::atomic<uint32_t>[]> has_waiter;
  // per slot (reset to kSlotReserved by the launcher once the batch is staged)
  std::unique_ptr<std::atomic<uint32_t>[]> slot_state;
  std::unique_ptr<std::atomic<const FillReq*>[]> slot_req;
  std::atomic<uint64_t> wake{0};
  std::atomic<uint32_t> wake_groups{0};
  hipStream_t stream = nullptr;
  hipEvent_t done_ev = nullptr;       // recorded after the batch's last device op
  rs::PinnedBuf host;
  rs::DevBuf dev;
  // region offsets (same in host staging and device slab)
  size_t o_data = 0, o_parity = 0, o_out = 0, o_masks = 0, o_plans = 0, o_bad = 0, o_hoff = 0, o_hlen = 0,
         o_digest = 0, o_ptrs = 0, bytes = 0;
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
void futex_wake(std::atomic<uint32_t>* w, int n) {
  syscall(SYS_futex, reinterpret_cast<uint32_t*>(w), FUTEX_WAKE_PRIVATE, n, nullptr, nullptr, 0);
}
// Epochs compare modulo 2^32 (prepare() keeps every live word within 2^30).
bool epoch_reached(uint32_t word, uint32_t epoch) { return static_cast<int32_t>(word - epoch) >= 0; }

// Moves a group word forward to `epoch` (never back).
void advance_epoch(std::atomic<uint32_t>* w, uint32_t epoch) {
  uint32_t cur = w->load(std::memory_order_relaxed);
  while (!epoch_reached(cur, epoch) &&
         !w->compare_exchange_weak(cur, epoch, std::memory_order_release, std::memory_order_relaxed)) {
  }
}

// Waits until *w reaches `epoch`.  A caller holding one of the `spin_slots`
// (rs_coalescer_opts.spin_waiters, default none) spins for up to 200 us before it
// sleeps; the others sleep after a brief spin (callers may far outnumber cores, and
// spinning steals the CPU the launcher, the completer and straggling callers need).
void wait_epoch(std::atomic<uint32_t>* w, uint32_t epoch, std::atomic<int>* spinners, int spin_slots) {
  if (spinners->fetch_add(1, std::memory_order_acq_rel) < spin_slots) {
    const auto t0 = Clock::now();
    for (uint32_t i = 0;; ++i) {
      if (epoch_reached(w->load(std::memory_order_acquire), epoch)) {
        spinners->fetch_sub(1, std::memory_order_acq_rel);
        return;
      }
      __builtin_ia32_pause();
      if ((i & 255u) == 255u && Clock::now() - t0 > std::chrono::microseconds(200)) break;
    }
  } else {
    for (int i = 0; i < 64; ++i) {
      if (epoch_reached(w->load(std::memory_order_acquire), epoch)) {
        spinners->fetch_sub(1, std::memory_order_acq_rel);
        return;
      }
      __builtin_ia32_pause();
    }
  }
  spinners->fetch_sub(1, std::memory_order_acq_rel);
  for (;;) {
    const uint32_t v = w->load(std::memory_order_acquire);
    if (epoch_reached(v, epoch)) return;
    futex_wait(w, v);
  }
}

// Per-GPU dispatch: a launcher thread closes open batches and launches them (at
// most max_exec executing), a completer thread waits for each launched batch and
// wakes its callers.  Callers only reserve, stage and sleep -- no caller thread is
// on the launch critical path, so a descheduled caller never holds up a batch
// (round 1's leader-caller design collapsed past ~256 callers on 16 cores:
// profiles/r01_coalesce_hi.log).
struct Dispatcher {
  int engine = 0;
  std::thread launcher, completer;
  std::atomic<uint32_t> work{0};      // bumped on every event the launcher may act on
  std::atomic<bool> launcher_idle{false};
  // Set before the launcher sleeps: true if a newly staged slot could start a batch
  // (an execution slot was free), false if only a completion can (then callers
  // skip the wake-up syscall: with callers outnumbering cores that was one futex
  // wake per call while the launcher waited for the device).
  std::atomic<bool> launcher_wants_callers{true};
  std::atomic<int> executing{0};
  std::mutex run_mu;
  std::condition_variable run_cv;
  std::deque<Batch*> running;         // launched, completion pending (launch order)
  std::vector<Batch*> mine;           // this engine's batches
};

// Wakes the launcher if it sleeps.  The handshake with launcher_loop's sleep
// (idle = true, then re-read work) is store -> load on both sides, so both are
// sequentially consistent: with acquire / release alone x86 may reorder each
// side's load before its store and both miss (a lost wake-up).  A caller's poke
// (from_caller) wakes the launcher only if it went to sleep able to start a batch;
// completions and shutdown always wake it.
void poke(Dispatcher* d, bool from_caller = false) {
  d->work.fetch_add(1, std::memory_order_seq_cst);
  if (d->launcher_idle.load(std::memory_order_seq_cst) &&
      (!from_caller || d->launcher_wants_callers.load(std::memory_order_seq_cst)))
    futex_wake(&d->work, 1);
}

// CPUs this process may run on: the cgroup v2 quota (cpu.max "quota period") when
// one is set, else the affinity mask (a container's quota is usually far below the
// host CPUs its mask shows).
int usable_cpus() {
  int n = 0;
  cpu_set_t set;
  if (sched_getaffinity(0, sizeof(set), &set) == 0) n = CPU_COUNT(&set);
  if (FILE* f = std::fopen("/sys/fs/cgroup/cpu.max", "r")) {
    char q[32] = {0};
    long long period = 0;
    if (std::fscanf(f, "%31s %lld", q, &period) == 2 && std::strcmp(q, "max") != 0 && period > 0) {
      const long long quota = std::atoll(q);
      const int qc = static_cast<int>(std::max(1LL, quota / period));
      if (n <= 0 || qc < n) n = qc;
    }
    std::fclose(f);
  }
  return n > 0 ? n : 1;
}

}  // namespace

struct rs_coalescer {
  rs_ctx* ctx = nullptr;
  int k = 0, m = 0;
  // k+m <= 16: a mask per slot, resolved by the kernel through the all-pattern LUT;
  // else a plan address per slot (resolved at staging from the engine's plan cache)
  bool per_stripe = false;
  size_t max_batch = 0, max_bytes = 0;
  std::chrono::microseconds max_wait{0};

  int max_exec = 2;   // batches on one device at once
  bool zero_copy = true;
  bool nt_copy = true;  // streaming stores in the staging copies (opts.plain_copy = 0)
  // objects whose shards lie in rs_host_alloc'ed memory run in place (zero-copy
  // staging, k+m <= 16, a pointer-table kernel for (k, m))
  bool direct_ok = false;
  // callers that may spin-wait for their batch at once (opts.spin_waiters, capped at
  // the CPUs this process may use minus the launcher and completer threads)
  int spin_slots = 0;
  std::atomic<int> spinners{0};
  std::atomic<bool> stop{false};

  std::mutex mu;
  std::condition_variable free_cv;    // a batch became free (back-pressure)
  int free_waiters = 0;               // callers blocked on free_cv (mu)
  std::vector<std::unique_ptr<Batch>> batches;
  std::vector<Batch*> free_list;
  std::vector<int> engine_load;   // batches open or executing per engine (mu)
  std::map<std::pair<int, size_t>, Batch*> open;  // (kind, S) -> batch accepting slots (mu)
  std::atomic<uint64_t> hot{0};  // last opened batch: hot_word(gen, index); 0 = none
  std::vector<std::unique_ptr<Dispatcher>> disp;  // one per engine
  // finished batches with asynchronous calls not yet reaped (rs_co_reap)
  std::mutex done_mu;
  std::condition_variable done_cv;
  std::deque<Batch*> done;

  std::atomic<uint64_t> calls{0}, n_batches{0}, stripes{0}, max_seen{0};
  // diagnostics (rs_co_timing)
  std::atomic<uint64_t> straggle_ns{0}, exec_ns{0}, free_waits{0}, launches_idle{0}, launch_ns{0};

  ~rs_coalescer() {
    stop.store(true, std::memory_order_release);
    {
      std::lock_guard<std::mutex> g(done_mu);  // a reaper waiting without a timeout returns 0
      done_cv.notify_all();
    }
    for (auto& d : disp) {
      poke(d.get());
      d->launcher_idle.store(true);
      futex_wake(&d->work, INT_MAX);
      {
        std::lock_guard<std::mutex> g(d->run_mu);
        d->run_cv.notify_all();
      }
      if (d->launcher.joinable()) d->launcher.join();
      if (d->completer.joinable()) d->completer.join();
    }
    for (auto& b : batches) {
      rs::DeviceScope ds(rs::engine_device(rs::ctx_engine(ctx, b->engine)));
      if (b->done_ev) (void)hipEventDestroy(b->done_ev);
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
  const size_t per = b->P * (k + 2 * m) + 64 + 8 * (k + m);  // shards + out + mask + plan + bad + hash + digest + ptrs
  const size_t cap = std::max<size_t>(
      1, std::min({co->max_batch, co->max_bytes / per, size_t(b->n_groups_alloc) * Batch::kGroup}));
  b->cap.store(cap, std::memory_order_relaxed);
  b->o_data = 0;
  b->o_parity = round_up(cap * k * b->P, 256);
  b->o_out = b->o_parity + round_up(cap * m * b->P, 256);
  b->o_masks = b->o_out + round_up(cap * m * b->P, 256);
  b->o_plans = b->o_masks + round_up(cap * 4, 256);
  b->o_bad = b->o_plans + round_up(cap * 8, 256);
  b->o_hoff = b->o_bad + round_up(cap * 4, 256);
  b->o_hlen = b->o_hoff + round_up(cap * 8, 256);
  b->o_digest = b->o_hlen + round_up(cap * 8, 256);
  b->o_ptrs = b->o_digest + round_up(cap * 32, 256);
  b->bytes = b->o_ptrs + round_up(cap * 8 * (k + m), 256);
  if (!b->stream) RS_HIP(hipStreamCreateWithFlags(&b->stream, hipStreamNonBlocking));
  if (!b->done_ev) RS_HIP(hipEventCreateWithFlags(&b->done_ev, hipEventDisableTiming));
  if (b->host.ensure(b->bytes) || b->dev.ensure(b->bytes)) return RS_ERR_DEVICE;
  b->host_dev = nullptr;
  if (co->direct_ok) {
    void* hd = nullptr;
    if (hipHostGetDevicePointer(&hd, b->host.p, 0) == hipSuccess) b->host_dev = static_cast<uint8_t*>(hd);
    else (void)hipGetLastError();
  }
  b->epoch += 1;
  // Words of groups unused for ~2^30 runs would read as "reached" once the epoch
  // wraps half-way round: pull them along (loads only, almost always).
  const uint32_t groups = static_cast<uint32_t>((cap + Batch::kGroup - 1) / Batch::kGroup);
  for (uint32_t g = 0; g < groups; ++g)
    if (static_cast<uint32_t>(b->epoch - b->grp[g].load(std::memory_order_relaxed)) > (1u << 30))
      advance_epoch(&b->grp[g], b->epoch - 1);
  b->filled.store(0, std::memory_order_relaxed);
  b->released.store(0, std::memory_order_relaxed);
  b->parity_in.store(0, std::memory_order_relaxed);
  b->fill_err.store(0, std::memory_order_relaxed);
  b->max_missing.store(0, std::memory_order_relaxed);
  b->hash_in.store(0, std::memory_order_relaxed);
  b->direct_in.store(0, std::memory_order_relaxed);
  b->n_async.store(0, std::memory_order_relaxed);
  b->async_cursor = 0;
  if (b->arec_cap < cap) {  // the batch is free: nobody reads the old records
    b->arec.reset(new AsyncRec[cap]);
    b->arec_cap = cap;
  }
  b->rc = RS_OK;
  b->free = false;
  b->deadline = Clock::now() + co->max_wait;
  b->gen = (b->gen + 1) & 0xFFFFFFu;
  b->key_kind.store(static_cast<int>(kind), std::memory_order_relaxed);
  b->key_S.store(S, std::memory_order_relaxed);
  b->ticket.store(static_cast<uint64_t>(b->gen) << kGenShift, std::memory_order_release);  // open, count 0
  return RS_OK;
}

// Enqueues a closed batch of n slots on its engine's stream (H2D / kernel / D2H as
// the staging mode needs) and records its completion event.  Asynchronous.
int launch_batch(rs_coalescer* co, Batch* b, size_t n) {
  const size_t k = co->k, m = co->m, P = b->P;
  rs::Engine* eng = rs::ctx_engine(co->ctx, b->engine);
  rs::DeviceScope ds(rs::engine_device(eng));
  hipStream_t st = b->stream;
  // Zero-copy (default): the staging is pinned host memory the GPU can address, so
  // the kernel reads the staged shards and writes its outputs there directly --
  // one launch per batch instead of 3-4 DMA round trips.
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
    if (b->kind == Kind::kApply && !co->per_stripe)
      RS_HIP(hipMemcpyAsync(dev_at(b, b->o_plans), host_at(b, b->o_plans), n * 8, hipMemcpyHostToDevice, st));
    if (b->hash_in.load(std::memory_order_relaxed)) {
      RS_HIP(hipMemcpyAsync(dev_at(b, b->o_hoff), host_at(b, b->o_hoff), n * 8, hipMemcpyHostToDevice, st));
      RS_HIP(hipMemcpyAsync(dev_at(b, b->o_hlen), host_at(b, b->o_hlen), n * 8, hipMemcpyHostToDevice, st));
    }
  }
  int rc;
  if (b->kind == Kind::kVerify) {
    // the mismatch words are OR-ed atomically: keep them in HBM, copy them back
    rc = rs::engine_verify_batch(eng, at(b->o_data), k * P, at(b->o_parity), m * P, P, b->S, n,
                                 reinterpret_cast<uint32_t*>(dev_at(b, b->o_bad)), st);
    if (rc) return rc;
    RS_HIP(hipMemcpyAsync(host_at(b, b->o_bad), dev_at(b, b->o_bad), n * 4, hipMemcpyDeviceToHost, st));
  } else {
    if (b->fill_err.load(std::memory_order_acquire)) return RS_ERR_DEVICE;
    if (co->per_stripe && b->direct_in.load(std::memory_order_acquire)) {
      // some slot is addressed in place in the caller's rs_host_alloc'ed buffers: every slot
      // through its row of the pointer table (staged slots point into the staging)
      if (!zc || !b->host_dev || at(0) != b->host_dev) return RS_ERR_DEVICE;
      const int bound = static_cast<int>(b->max_missing.load(std::memory_order_acquire));
      rc = rs::engine_apply_batch_ptrs(eng, reinterpret_cast<const uint64_t*>(at(b->o_ptrs)),
                                       reinterpret_cast<const uint32_t*>(at(b->o_masks)), b->S, n, bound, st);
    } else if (co->per_stripe) {
      // erasure bound = the most any slot misses (an encode slot: m): a batch of
      // 1-2 erasure repairs runs the E = 1 / 2 kernels
      const int bound = static_cast<int>(b->max_missing.load(std::memory_order_acquire));
      rc = rs::engine_reconstruct_batch_out(eng, at(b->o_data), k * P, at(b->o_parity), m * P, P, b->S, n,
                                            reinterpret_cast<const uint32_t*>(at(b->o_masks)), n, 1, bound,
                                            at(b->o_out), m * P, st);
    } else {  // k+m > 16: every slot names its plan (encode, reconstruct or ReconstructData)
      rc = rs::engine_apply_batch_plans(eng, at(b->o_data), k * P, at(b->o_parity), m * P, P, b->S, n,
                                        reinterpret_cast<const uint64_t*>(at(b->o_plans)), at(b->o_out), m * P,
                                        st);
    }
    if (rc) return rc;
    if (b->hash_in.load(std::memory_order_relaxed)) {
      // cold_hash of every slot that asked for it, over the same staged data shards
      // (value byte o in data shard o / S of the slot, offset o % S)
      rs::Sha256Args ha{at(b->o_data), 0, reinterpret_cast<const uint64_t*>(at(b->o_hoff)),
                        reinterpret_cast<const uint64_t*>(at(b->o_hlen)), 0, static_cast<uint32_t>(n),
                        at(b->o_digest), b->S, P};
      if (rs::launch_sha256(ha, st)) return RS_ERR_DEVICE;
      if (!zc)
        RS_HIP(hipMemcpyAsync(host_at(b, b->o_digest), dev_at(b, b->o_digest), n * 32, hipMemcpyDeviceToHost, st));
    }
    if (!zc)
      RS_HIP(hipMemcpyAsync(host_at(b, b->o_out), dev_at(b, b->o_out), n * m * P, hipMemcpyDeviceToHost, st));
  }
  RS_HIP(hipEventRecord(b->done_ev, st));
  return RS_OK;  // every mask was checked (>= k present) before it was staged
}

// Raises a batch's erasure bound to at least e (a slot's missing-shard count).
void note_missing(Batch* b, uint32_t e) {
  uint32_t cur = b->max_missing.load(std::memory_order_relaxed);
  while (cur < e && !b->max_missing.compare_exchange_weak(cur, e, std::memory_order_release, std::memory_order_relaxed)) {
  }
}

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

// Wakes the next groups of run `epoch` of a finished batch until `limit` groups
// with waiters are up (or none is left).  A no-op once the batch has moved on.
void wake_more(Batch* b, uint32_t epoch, int limit) {
  int woken = 0;
  while (woken < limit) {
    uint64_t w = b->wake.load(std::memory_order_acquire);
    if (static_cast<uint32_t>(w >> 32) != epoch) return;
    const uint32_t g = static_cast<uint32_t>(w);
    if (g >= b->wake_groups.load(std::memory_order_acquire)) return;
    if (!b->wake.compare_exchange_weak(w, w + 1, std::memory_order_acq_rel, std::memory_order_acquire)) continue;
    advance_epoch(&b->grp[g], epoch);
    if (b->has_waiter[g].load(std::memory_order_acquire) == epoch) {
      futex_wake(&b->grp[g], INT_MAX);
      ++woken;
    }
  }
}

// Publishes a finished batch to its callers.
void complete(rs_coalescer* co, Dispatcher* d, Batch* b, int rc) {
  b->rc = rc;
  co->n_batches.fetch_add(1, std::memory_order_relaxed);
  co->stripes.fetch_add(b->n_final, std::memory_order_relaxed);
  uint64_t seen = co->max_seen.load(std::memory_order_relaxed);
  while (b->n_final > seen && !co->max_seen.compare_exchange_weak(seen, b->n_final)) {
  }
  const uint32_t epoch = b->epoch;
  b->wake_groups.store(static_cast<uint32_t>((b->n_final + Batch::kGroup - 1) / Batch::kGroup),
                       std::memory_order_relaxed);
  b->wake.store(static_cast<uint64_t>(epoch) << 32, std::memory_order_release);
  d->executing.fetch_sub(1, std::memory_order_acq_rel);
  poke(d);  // an execution slot is free: the next batch may start before the wake-ups
  if (b->n_async.load(std::memory_order_relaxed)) {  // staged before the launch (acquired there)
    std::lock_guard<std::mutex> g(co->done_mu);
    co->done.push_back(b);
    co->done_cv.notify_all();
  }
  wake_more(b, epoch, 2);
}

// One pass over a closed batch's n slots: stages the slots whose callers published
// their FillReq but have not started staging (a descheduled caller, common with
// callers far outnumbering cores).  Slots a caller is copying are left to it.
void stage_published(Batch* b, size_t n) {
  for (size_t s = 0; s < n; ++s) {
    uint32_t st = b->slot_state[s].load(std::memory_order_acquire);
    if (st != kSlotPublished) continue;
    const FillReq* r = b->slot_req[s].load(std::memory_order_relaxed);
    if (!b->slot_state[s].compare_exchange_strong(st, kSlotTaken, std::memory_order_acq_rel)) continue;
    r->fn(r->ctx, b, s, r->item0 + (s - r->slot0));
    b->filled.fetch_add(1, std::memory_order_release);
  }
}

// A closed batch waiting for its callers' staging copies before it may launch.
struct Closing {
  Batch* b;
  size_t n;
  Clock::time_point closed;
};

// How long the launcher lets a closed batch's callers finish their own staging
// copies before it stages published slots itself.
constexpr auto kStraggleGrace = std::chrono::microseconds(100);

// Launcher: batching is group commit -- an open batch closes when full, or when
// max_wait has passed since it opened (default 0) and the device has room for it;
// callers arriving meanwhile pile into it, so batches grow with the load and a lone
// caller waits for no timer.  A closed batch launches once every reserved slot is
// staged and fewer than max_exec batches of this GPU are executing.  Round 3: the
// launcher no longer waits on a closed batch's staging copies before it can look
// at other batches -- with 1.5 MB objects those copies took 41 % of its time while
// the device idled between batches (rs_co_timing straggle_ns).  The last caller to
// stage into a closed batch always wakes the launcher.
void launcher_loop(rs_coalescer* co, Dispatcher* d) {
  std::vector<Closing> closing;
  for (;;) {
    const uint32_t w = d->work.load(std::memory_order_acquire);
    if (co->stop.load(std::memory_order_acquire)) return;
    const auto now = Clock::now();
    Clock::time_point wake_at = Clock::time_point::max();
    // 1. launch fully staged closed batches, oldest first, while the device has room
    for (size_t i = 0; i < closing.size() && d->executing.load(std::memory_order_acquire) < co->max_exec;) {
      Closing& c = closing[i];
      if (c.b->filled.load(std::memory_order_acquire) < c.n && now - c.closed >= kStraggleGrace) {
        const auto ts0 = Clock::now();
        stage_published(c.b, c.n);
        co->straggle_ns.fetch_add(std::chrono::duration_cast<std::chrono::nanoseconds>(Clock::now() - ts0).count(),
                                  std::memory_order_relaxed);
      }
      if (c.b->filled.load(std::memory_order_acquire) < c.n) {
        // before the grace ends: wake then to stage published slots; after it, the
        // slots left are being copied by their callers, and the last one wakes us
        if (now - c.closed < kStraggleGrace) wake_at = std::min(wake_at, c.closed + kStraggleGrace);
        ++i;
        continue;
      }
      Batch* b = c.b;
      const size_t n = c.n;
      closing.erase(closing.begin() + static_cast<std::ptrdiff_t>(i));
      for (size_t s = 0; s < n; ++s) b->slot_state[s].store(kSlotReserved, std::memory_order_relaxed);
      b->n_final = n;
      d->executing.fetch_add(1, std::memory_order_acq_rel);
      const auto tl0 = Clock::now();
      const int rc = launch_batch(co, b, n);
      co->launch_ns.fetch_add(std::chrono::duration_cast<std::chrono::nanoseconds>(Clock::now() - tl0).count(),
                              std::memory_order_relaxed);
      if (rc) {
        complete(co, d, b, rc);
        continue;
      }
      std::lock_guard<std::mutex> g(d->run_mu);
      d->running.push_back(b);
      d->run_cv.notify_one();
    }
    // 2. close open batches: a full one at once (it cannot grow), one past its
    // linger only if the device would have room for it next to the closed ones
    const int busy = d->executing.load(std::memory_order_acquire) + static_cast<int>(closing.size());
    const bool slot = busy < co->max_exec;
    Batch* pick = nullptr;
    for (Batch* b : d->mine) {
      const uint64_t t = b->ticket.load(std::memory_order_acquire);
      const size_t cnt = static_cast<size_t>(t & kCountMask);
      if ((t & kClosedBit) || cnt == 0) continue;  // free, closed, or nobody in it yet
      const bool full = cnt >= b->cap.load(std::memory_order_relaxed);
      if (full || (slot && now >= b->deadline)) {
        if (!pick || full) pick = b;
        if (full) break;
      } else if (slot) {
        wake_at = std::min(wake_at, b->deadline);
      }
    }
    if (pick) {
      const uint64_t t = pick->ticket.fetch_or(kClosedBit, std::memory_order_acq_rel);
      {
        std::lock_guard<std::mutex> g(co->mu);
        unpublish(co, pick, static_cast<uint32_t>(t >> kGenShift));
      }
      closing.push_back(Closing{pick, static_cast<size_t>(t & kCountMask), Clock::now()});
      continue;  // its callers may all have staged already
    }
    // nothing to do now: sleep until a caller stages, a slot frees, a linger or a
    // straggler grace ends.  A staging caller wakes the launcher only if that can
    // start something (a free slot for an open batch); the last stager of a closed
    // batch and completions always wake it.
    d->launcher_wants_callers.store(slot, std::memory_order_seq_cst);
    d->launcher_idle.store(true, std::memory_order_seq_cst);
    if (d->work.load(std::memory_order_seq_cst) == w && !co->stop.load(std::memory_order_acquire)) {
      if (wake_at != Clock::time_point::max()) {
        const auto ns = std::chrono::duration_cast<std::chrono::nanoseconds>(wake_at - Clock::now()).count();
        if (ns > 0) {
          timespec ts{static_cast<time_t>(ns / 1000000000), static_cast<long>(ns % 1000000000)};
          syscall(SYS_futex, reinterpret_cast<uint32_t*>(&d->work), FUTEX_WAIT_PRIVATE, w, &ts, nullptr, 0);
        }
      } else {
        futex_wait(&d->work, w);
      }
    }
    d->launcher_idle.store(false, std::memory_order_release);
  }
}

// Completer: waits for each launched batch in launch order and wakes its callers.
void completer_loop(rs_coalescer* co, Dispatcher* d) {
  rs::DeviceScope ds(rs::engine_device(rs::ctx_engine(co->ctx, d->engine)));
  for (;;) {
    Batch* b = nullptr;
    {
      std::unique_lock<std::mutex> lk(d->run_mu);
      d->run_cv.wait(lk, [&] { return !d->running.empty() || co->stop.load(std::memory_order_acquire); });
      if (d->running.empty()) return;  // stopping with nothing in flight
      b = d->running.front();
      d->running.pop_front();
    }
    const auto t0 = Clock::now();
    const int rc = hipEventSynchronize(b->done_ev) == hipSuccess ? RS_OK : RS_ERR_DEVICE;
    co->exec_ns.fetch_add(std::chrono::duration_cast<std::chrono::nanoseconds>(Clock::now() - t0).count(),
                          std::memory_order_relaxed);
    complete(co, d, b, rc);
  }
}

// Reserves up to `want` consecutive slots of an open batch for (kind, S), opening
// one if needed.  With every batch in flight a blocking caller waits for one to
// free (back-pressure); a non-blocking one gets RS_ERR_BUSY.  Returns RS_OK with
// *take >= 1 slots from *slot0 of *bp.
int reserve_slots(rs_coalescer* co, Kind kind, size_t S, size_t want, bool block, Batch** bp, size_t* slot0,
                  size_t* take) {
  const auto key = std::make_pair(static_cast<int>(kind), S);
  // fast path: the most recently opened batch, no mutex
  if (const uint64_t h = co->hot.load(std::memory_order_acquire)) {
    Batch* hb = co->batches[(h & 0xFFFF) - 1].get();
    const uint32_t hg = static_cast<uint32_t>(h >> 16);
    if (hb->key_kind.load(std::memory_order_relaxed) == key.first &&
        hb->key_S.load(std::memory_order_relaxed) == key.second && (*take = try_reserve(hb, hg, want, slot0))) {
      *bp = hb;
      return RS_OK;
    }
  }
  std::unique_lock<std::mutex> lk(co->mu);
  for (;;) {
    auto it = co->open.find(key);
    if (it != co->open.end()) {
      Batch* ob = it->second;
      if ((*take = try_reserve(ob, ob->gen, want, slot0))) {
        *bp = ob;
        return RS_OK;
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
        if (co->free_waiters) co->free_cv.notify_one();
        return rc;
      }
      ++co->engine_load[nb->engine];
      *take = try_reserve(nb, nb->gen, want, slot0);
      *bp = nb;
      co->open[key] = nb;
      co->hot.store(hot_word(nb->gen, nb->index), std::memory_order_release);
      return RS_OK;
    }
    if (!block) return RS_ERR_BUSY;
    ++co->free_waiters;  // every batch is in flight: back-pressure
    co->free_waits.fetch_add(1, std::memory_order_relaxed);
    co->free_cv.wait(lk);
    --co->free_waiters;
  }
}

// `count` slots of batch b have been drained: the last one hands the batch back.
void release_slots(rs_coalescer* co, Batch* b, size_t count) {
  if (b->released.fetch_add(static_cast<uint32_t>(count), std::memory_order_acq_rel) + count == b->n_final) {
    std::lock_guard<std::mutex> g(co->mu);
    b->free = true;
    --co->engine_load[b->engine];
    co->free_list.push_back(b);
    if (co->free_waiters) co->free_cv.notify_one();
  }
}

// One call through the coalescer.  fill(b, slot, item) stages the inputs,
// drain(b, slot, item) copies the outputs back; both run in the caller's thread,
// outside any lock.
template <class Fill, class Drain>
int submit_many(rs_coalescer* co, Kind kind, size_t S, size_t count, bool parity_in, Fill&& fill, Drain&& drain) {
  int result = RS_OK;
  size_t done_items = 0;
  while (done_items < count) {
    Batch* b = nullptr;
    size_t slot0 = 0, take = 0;
    const int rrc = reserve_slots(co, kind, S, count - done_items, true, &b, &slot0, &take);
    if (rrc) return rrc;
    // the epoch was set before the ticket opened (acquired by the reservation)
    const uint32_t epoch = b->epoch;
    const uint32_t grp = static_cast<uint32_t>(slot0 / Batch::kGroup);
    b->has_waiter[grp].store(epoch, std::memory_order_release);  // before `filled`: seen by the waker
    if (parity_in) b->parity_in.store(1, std::memory_order_relaxed);
    // publish how to stage these slots (the launcher may do it if we are descheduled)
    const FillReq fr{[](const void* c, Batch* bb, size_t slot, size_t item) {
                       (*static_cast<const std::remove_reference_t<Fill>*>(c))(bb, slot, item);
                     },
                     &fill, slot0, done_items};
    for (size_t j = 0; j < take; ++j) {
      b->slot_req[slot0 + j].store(&fr, std::memory_order_relaxed);
      b->slot_state[slot0 + j].store(kSlotPublished, std::memory_order_release);
    }
    uint32_t staged = 0;
    for (size_t j = 0; j < take; ++j) {
      uint32_t st = kSlotPublished;
      if (b->slot_state[slot0 + j].load(std::memory_order_acquire) != st) continue;  // the launcher took it
      fill(b, slot0 + j, done_items + j);
      if (b->slot_state[slot0 + j].compare_exchange_strong(st, kSlotStaged, std::memory_order_acq_rel)) ++staged;
    }
    bool last = false;  // this caller completed the staging of a closed batch
    if (staged) {
      const size_t filled = b->filled.fetch_add(staged, std::memory_order_acq_rel) + staged;
      const uint64_t t = b->ticket.load(std::memory_order_acquire);
      last = (t & kClosedBit) && filled >= static_cast<size_t>(t & kCountMask);
    }
    poke(co->disp[static_cast<size_t>(b->engine)].get(), !last);
    wait_epoch(&b->grp[grp], epoch, &co->spinners, co->spin_slots);
    wake_more(b, epoch, 2);
    const int rc = b->rc;  // published by the group word (release / acquire), as n_final
    if (rc == RS_OK)
      for (size_t j = 0; j < take; ++j) drain(b, slot0 + j, done_items + j);
    else if (result == RS_OK)
      result = rc;
    release_slots(co, b, take);
    done_items += take;
  }
  return result;
}

// An asynchronous call (rs_co_submit_*): reserve one slot, stage it here, record
// where its outputs go, and return without waiting -- rs_co_reap drains it once
// its batch has run.  Never blocks: with every batch in flight RS_ERR_BUSY tells
// the caller to reap first.  The slot's FillReq is never published (the caller
// stages before it returns, so the launcher never runs a fill on its stack).
template <class Fill>
int submit_async(rs_coalescer* co, Kind kind, size_t S, bool parity_in, Fill&& fill, const AsyncRec& rec) {
  Batch* b = nullptr;
  size_t slot = 0, take = 0;
  const int rrc = reserve_slots(co, kind, S, 1, false, &b, &slot, &take);
  if (rrc) return rrc;
  co->calls.fetch_add(1, std::memory_order_relaxed);
  if (parity_in) b->parity_in.store(1, std::memory_order_relaxed);
  fill(b, slot);
  const uint32_t ai = b->n_async.fetch_add(1, std::memory_order_relaxed);
  b->arec[ai] = rec;
  b->arec[ai].slot = static_cast<uint32_t>(slot);
  const size_t filled = b->filled.fetch_add(1, std::memory_order_acq_rel) + 1;  // publishes the slot and its record
  const uint64_t t = b->ticket.load(std::memory_order_acquire);
  poke(co->disp[static_cast<size_t>(b->engine)].get(), !((t & kClosedBit) && filled >= (t & kCountMask)));
  return RS_OK;
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
  bool direct = false;       // every shard it reads or writes is rs_host_alloc'ed: addressed in place
  uint64_t dev[32] = {};     // direct: GPU address of every shard (rs_host_alloc'ed)
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

// Plan mode (k+m > 16): slot's plan address on the batch's engine.
void set_plan(const rs_coalescer* co, Batch* b, size_t slot, uint64_t present, bool data_only, bool encode) {
  rs::Engine* eng = rs::ctx_engine(co->ctx, b->engine);
  const uint8_t* plan = nullptr;
  if (encode)
    plan = rs::engine_encode_plan(eng);
  else if (rs::engine_plan_for(eng, present, data_only, &plan) != RS_OK)
    plan = nullptr;
  if (!plan) b->fill_err.store(1, std::memory_order_release);
  reinterpret_cast<uint64_t*>(host_at(b, b->o_plans))[slot] = reinterpret_cast<uint64_t>(plan);
}

// Per-slot cold_hash request: the first value_len bytes of the slot's k data
// shards (offsets relative to the data region), or kSha256Skip for none.
void set_hash(Batch* b, int k, size_t slot, uint64_t value_len) {
  reinterpret_cast<uint64_t*>(host_at(b, b->o_hlen))[slot] = value_len;
  reinterpret_cast<uint64_t*>(host_at(b, b->o_hoff))[slot] = static_cast<uint64_t>(slot) * k * b->P;
  if (value_len != rs::kSha256Skip) b->hash_in.store(1, std::memory_order_relaxed);
}

// A slot's row of the pointer table (GPU addresses of its k+m shards), used when
// the batch runs the pointer-table kernel (some slot is direct).
uint64_t* ptr_row(const rs_coalescer* co, Batch* b, size_t slot) {
  return reinterpret_cast<uint64_t*>(host_at(b, b->o_ptrs)) + slot * static_cast<size_t>(co->k + co->m);
}

// Row of a staged slot: present shards at their staging copies, missing ones at the
// slot's output rows (the r-th missing shard -> out row r), all in the staging's
// GPU mapping.  Written for every staged slot, so a direct slot may join any batch.
void stage_ptrs(const rs_coalescer* co, Batch* b, size_t slot, uint32_t present) {
  if (!co->direct_ok || !b->host_dev) return;
  const size_t k = co->k, m = co->m, P = b->P;
  uint64_t* row = ptr_row(co, b, slot);
  auto at = [&](size_t off) { return reinterpret_cast<uint64_t>(b->host_dev + off); };
  for (size_t s = 0, r = 0; s < k + m; ++s) {
    if ((present >> s) & 1u)
      row[s] = s < k ? at(b->o_data + (slot * k + s) * P) : at(b->o_parity + (slot * m + (s - k)) * P);
    else
      row[s] = at(b->o_out + (slot * m + r++) * P);
  }
}

// GPU addresses of a call's shards when every one the kernel touches lies in
// rs_host_alloc'ed memory (the context's own page-locked pages), 16-B aligned: `touched` bit s = shard s is read (one of
// the first k present) or written (an output).  Other entries repeat the first
// touched address (never dereferenced).  False: the call is staged.
bool direct_ptrs(rs_coalescer* co, uint8_t* const* shards, size_t S, uint32_t touched, uint64_t* dev) {
  if (!co->direct_ok) return false;
  const int t = co->k + co->m;
  uint64_t first = 0;
  for (int s = 0; s < t; ++s) {
    dev[s] = 0;
    if (!((touched >> s) & 1u)) continue;
    if (!shards[s] || reinterpret_cast<uintptr_t>(shards[s]) % 16) return false;
    uint8_t* d = rs::ctx_owned(co->ctx, shards[s], S);
    if (!d || reinterpret_cast<uintptr_t>(d) % 16) return false;
    dev[s] = reinterpret_cast<uint64_t>(d);
    if (!first) first = dev[s];
  }
  for (int s = 0; s < t; ++s)
    if (!dev[s]) dev[s] = first;
  return first != 0;
}

// cold_hash of a direct encode reads the value in place: possible when the data
// shards holding its first value_len bytes are contiguous (shard c at shard 0 + c*S,
// as Split carves them from one body; with 16-B aligned shards S is then a multiple
// of 16, so the hash kernel's shard pitch b->P equals S).
bool hash_in_place_ok(uint8_t* const* shards, size_t S, uint64_t value_len) {
  const uint64_t n = (value_len + S - 1) / S;
  for (uint64_t c = 1; c < n; ++c)
    if (shards[c] != shards[0] + c * S) return false;
  return true;
}

// The hash request of a direct slot: its value starts at the GPU address dev0 (the
// kernel adds the offset to the batch's data base in 64-bit wrap-around arithmetic).
void set_hash_direct(Batch* b, size_t slot, uint64_t value_len, uint64_t dev0) {
  reinterpret_cast<uint64_t*>(host_at(b, b->o_hlen))[slot] = value_len;
  reinterpret_cast<uint64_t*>(host_at(b, b->o_hoff))[slot] = dev0 - reinterpret_cast<uint64_t>(b->host_dev + b->o_data);
  b->hash_in.store(1, std::memory_order_relaxed);
}

// A direct slot: its row = the caller's buffers; nothing is copied.
void direct_fill(const rs_coalescer* co, Batch* b, size_t slot, const uint64_t* dev, uint32_t present) {
  const int t = co->k + co->m;
  std::memcpy(ptr_row(co, b, slot), dev, static_cast<size_t>(t) * 8);
  set_hash(b, co->k, slot, rs::kSha256Skip);
  reinterpret_cast<uint32_t*>(host_at(b, b->o_masks))[slot] = present;
  note_missing(b, static_cast<uint32_t>(t - __builtin_popcount(present)));
  b->direct_in.store(1, std::memory_order_relaxed);
}

// One encode slot (rs_co_encode / _hash / _submit_encode / _many): in place through
// the caller's addresses when `dev` is set, else its data shards staged, its mask
// (or plan) and pointer row written -- every staged slot needs the row, since an
// in-place slot may make the batch run the pointer-table kernel.  value_len:
// kSha256Skip for no cold_hash.
void encode_fill(const rs_coalescer* co, Batch* b, size_t slot, uint8_t* const* shards, size_t S,
                 const uint64_t* dev, uint64_t value_len) {
  const int k = co->k, m = co->m;
  const uint32_t data_mask = (1u << k) - 1u;  // parity all missing -> encode rows
  if (dev) {
    direct_fill(co, b, slot, dev, data_mask);
    if (value_len != rs::kSha256Skip) set_hash_direct(b, slot, value_len, dev[0]);
    return;
  }
  for (int c = 0; c < k; ++c) rs::stage_copy(host_at(b, b->o_data + (slot * k + c) * b->P), shards[c], S, co->nt_copy);
  set_hash(b, k, slot, value_len);
  if (co->per_stripe) {
    reinterpret_cast<uint32_t*>(host_at(b, b->o_masks))[slot] = data_mask;
    note_missing(b, static_cast<uint32_t>(m));
    stage_ptrs(co, b, slot, data_mask);
  } else {
    set_plan(co, b, slot, data_mask, false, true);
  }
}

// Decides whether a reconstruct runs in place (Reconstruct only: ReconstructData
// leaves missing parity unwritten and may pass no buffer for it).
void rec_direct(rs_coalescer* co, RecItem* it, bool data_only) {
  it->direct = false;
  if (data_only) return;
  const int k = co->k, t = k + co->m;
  uint32_t touched = 0;
  for (int i = 0, used = 0; i < t; ++i) {
    if (it->lens[i] && used < k) {
      touched |= 1u << i;
      ++used;
    } else if (!it->lens[i]) {
      touched |= 1u << i;
    }
  }
  it->direct = direct_ptrs(co, it->shards, it->S, touched, it->dev);
}

void rec_fill(const rs_coalescer* co, Batch* b, size_t slot, const RecItem& it, bool data_only) {
  const int k = co->k, m = co->m, t = k + m;
  const size_t P = b->P;
  if (it.direct) {
    direct_fill(co, b, slot, it.dev, it.present);
    return;
  }
  set_hash(b, k, slot, rs::kSha256Skip);
  for (int i = 0, staged = 0; i < t && staged < k; ++i) {  // the k survivors only
    if (!it.lens[i]) continue;
    ++staged;
    uint8_t* dst = i < k ? host_at(b, b->o_data + (slot * k + i) * P) : host_at(b, b->o_parity + (slot * m + (i - k)) * P);
    rs::stage_copy(dst, it.shards[i], it.S, co->nt_copy);
  }
  if (co->per_stripe) {
    reinterpret_cast<uint32_t*>(host_at(b, b->o_masks))[slot] = it.present;
    note_missing(b, static_cast<uint32_t>(t - __builtin_popcount(it.present)));
    stage_ptrs(co, b, slot, it.present);
  } else {
    set_plan(co, b, slot, it.present, data_only, false);
  }
}

void rec_drain(const rs_coalescer* co, Batch* b, size_t slot, const RecItem& it, bool data_only) {
  const int k = co->k, m = co->m, t = k + m;
  int r = 0;  // r-th missing shard (index order, data before parity) = out slot r
  for (int i = 0; i < t; ++i) {
    if (it.lens[i]) continue;
    if (!data_only || i < k) {
      if (!it.direct) rs::stage_copy(it.shards[i], host_at(b, b->o_out + (slot * m + r) * b->P), it.S, co->nt_copy);
      it.lens[i] = it.S;  // direct: the kernel wrote the caller's buffer
    }
    ++r;
  }
}

int co_reconstruct(rs_coalescer* co, uint8_t* const* shards, size_t* lens, bool data_only) {
  if (!co || !shards || !lens) return RS_ERR_INVALID_ARG;
  RecItem it;
  bool need = false;
  const int rc = rec_check(co, shards, lens, data_only, &it, &need);
  if (rc || !need) return rc;
  rec_direct(co, &it, data_only);
  return submit(
      co, Kind::kApply, it.S, it.parity_used, [&](Batch* b, size_t slot) { rec_fill(co, b, slot, it, data_only); },
      [&](Batch* b, size_t slot) { rec_drain(co, b, slot, it, data_only); });
}

}  // namespace

extern "C" {

int rs_coalescer_create(rs_ctx* ctx, const rs_coalescer_opts* opts, rs_coalescer** out) {
  if (!ctx || !out) return RS_ERR_INVALID_ARG;
  *out = nullptr;
  const int ne = rs::ctx_engine_count(ctx);
  rs_coalescer_opts o{4096, 0, std::max(16, 8 * ne), size_t(32) << 20, 2, 0, 0, 0};
  if (opts) {
    if (opts->max_batch) o.max_batch = opts->max_batch;
    o.max_wait_us = opts->max_wait_us;
    if (opts->inflight > 0) o.inflight = opts->inflight;
    if (opts->max_batch_bytes) o.max_batch_bytes = opts->max_batch_bytes;
    if (opts->max_exec > 0) o.max_exec = opts->max_exec;
    o.staged_dma = opts->staged_dma;
    o.spin_waiters = opts->spin_waiters;
    o.plain_copy = opts->plain_copy;
  }
  if (o.inflight > 256 || o.max_exec > o.inflight || o.inflight < ne || o.spin_waiters < 0) return RS_ERR_INVALID_ARG;
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
  co->nt_copy = o.plain_copy == 0;
  co->direct_ok = co->zero_copy && co->k + co->m <= 16 && rs::apply_ptrs_supported(co->k, co->m);
  co->spin_slots = std::min(o.spin_waiters, std::max(0, usable_cpus() - 2 - 2 * ne));
  co->engine_load.assign(static_cast<size_t>(ne), 0);
  // the most slots a batch can hold: max_batch, bounded by the bytes budget at
  // the smallest slot (16-B shards) and by 2^20
  const size_t max_cap = std::max<size_t>(
      1, std::min({o.max_batch, o.max_batch_bytes / (16 * static_cast<size_t>(co->k + 2 * co->m) + 8),
                   size_t(1) << 20}));
  for (int e = 0; e < ne; ++e) {
    co->disp.push_back(std::make_unique<Dispatcher>());
    co->disp.back()->engine = e;
  }
  for (int i = 0; i < o.inflight; ++i) {
    co->batches.push_back(std::make_unique<Batch>());
    Batch* b = co->batches.back().get();
    b->index = i;
    b->engine = i % ne;
    b->n_groups_alloc = static_cast<uint32_t>((max_cap + Batch::kGroup - 1) / Batch::kGroup);
    b->grp.reset(new std::atomic<uint32_t>[b->n_groups_alloc]);
    b->has_waiter.reset(new std::atomic<uint32_t>[b->n_groups_alloc]);
    for (uint32_t g = 0; g < b->n_groups_alloc; ++g) {
      b->grp[g].store(0, std::memory_order_relaxed);
      b->has_waiter[g].store(0, std::memory_order_relaxed);
    }
    const size_t slots = static_cast<size_t>(b->n_groups_alloc) * Batch::kGroup;
    b->slot_state.reset(new std::atomic<uint32_t>[slots]);
    b->slot_req.reset(new std::atomic<const FillReq*>[slots]);
    for (size_t i = 0; i < slots; ++i) {
      b->slot_state[i].store(kSlotReserved, std::memory_order_relaxed);
      b->slot_req[i].store(nullptr, std::memory_order_relaxed);
    }
    b->host.numa = rs::device_numa_node(rs::engine_device(rs::ctx_engine(ctx, b->engine)));
    co->free_list.push_back(b);
    co->disp[static_cast<size_t>(b->engine)]->mine.push_back(b);
  }
  for (auto& d : co->disp) {
    d->launcher = std::thread(launcher_loop, co.get(), d.get());
    d->completer = std::thread(completer_loop, co.get(), d.get());
  }
  *out = co.release();
  return RS_OK;
}

void rs_coalescer_destroy(rs_coalescer* co) { delete co; }

// Encode, and with value_len != kSha256Skip also the SHA-256 of the value's first
// value_len bytes (its data shards in order) into digest.
static int co_encode(rs_coalescer* co, uint8_t* const* shards, const size_t* lens, uint64_t value_len,
                     uint8_t* digest) {
  if (!co || !shards || !lens) return RS_ERR_INVALID_ARG;
  const int k = co->k, m = co->m;
  const bool hash = value_len != rs::kSha256Skip;
  if (hash && !digest) return RS_ERR_INVALID_ARG;
  size_t S = 0;
  int rc = rs::check_shards(k + m, lens, false, &S);
  if (rc) return rc;
  if (hash && value_len > static_cast<uint64_t>(k) * S) return RS_ERR_INVALID_ARG;
  if (m == 0) return hash ? RS_ERR_NOT_SUPPORTED : RS_OK;
  for (int i = 0; i < k + m; ++i)
    if (!shards[i]) return RS_ERR_INVALID_ARG;
  if (S > 0xFFFFFFF0u) return RS_ERR_INVALID_ARG;
  // every shard in rs_host_alloc'ed memory (a cold_hash's value contiguous in it): the
  // kernels read the data and write the parity in place
  uint64_t dev[32];
  const bool direct =
      direct_ptrs(co, shards, S, (1u << (k + m)) - 1u, dev) && (!hash || hash_in_place_ok(shards, S, value_len));
  auto fill = [&](Batch* b, size_t slot) { encode_fill(co, b, slot, shards, S, direct ? dev : nullptr, value_len); };
  auto drain = [&](Batch* b, size_t slot) {
    if (!direct)
      for (int r = 0; r < m; ++r) rs::stage_copy(shards[k + r], host_at(b, b->o_out + (slot * m + r) * b->P), S, co->nt_copy);
    if (hash) std::memcpy(digest, host_at(b, b->o_digest + slot * 32), 32);
  };
  return submit(co, Kind::kApply, S, false, fill, drain);
}

int rs_co_encode(rs_coalescer* co, uint8_t* const* shards, const size_t* lens) {
  return co_encode(co, shards, lens, rs::kSha256Skip, nullptr);
}

int rs_co_encode_hash(rs_coalescer* co, uint8_t* const* shards, const size_t* lens, size_t value_len,
                      uint8_t* digest) {
  return co_encode(co, shards, lens, value_len, digest);
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
    for (int c = 0; c < k; ++c) rs::stage_copy(host_at(b, b->o_data + (slot * k + c) * b->P), shards[c], S, co->nt_copy);
    for (int r = 0; r < m; ++r) rs::stage_copy(host_at(b, b->o_parity + (slot * m + r) * b->P), shards[k + r], S, co->nt_copy);
  };
  auto drain = [&](Batch* b, size_t slot) { *ok = reinterpret_cast<uint32_t*>(host_at(b, b->o_bad))[slot] == 0; };
  return submit(co, Kind::kVerify, S, true, fill, drain);
}

// ---- asynchronous calls ----------------------------------------------------------
int rs_co_submit_encode(rs_coalescer* co, uint8_t* const* shards, const size_t* lens, uint64_t tag) {
  if (!co || !shards || !lens) return RS_ERR_INVALID_ARG;
  const int k = co->k, m = co->m;
  size_t S = 0;
  int rc = rs::check_shards(k + m, lens, false, &S);
  if (rc) return rc;
  for (int i = 0; i < k + m; ++i)
    if (!shards[i]) return RS_ERR_INVALID_ARG;
  if (m == 0) return RS_ERR_NOT_SUPPORTED;  // nothing to compute, nothing would be reaped
  if (S > 0xFFFFFFF0u) return RS_ERR_INVALID_ARG;
  uint64_t dev[32];
  const bool direct = direct_ptrs(co, shards, S, (1u << (k + m)) - 1u, dev);  // in place: nothing to copy back
  AsyncRec rec;
  rec.tag = tag;
  rec.n_out = direct ? 0u : static_cast<uint32_t>(m);
  for (int r = 0; r < m; ++r) rec.out[r] = shards[k + r];
  auto fill = [&](Batch* b, size_t slot) {
    encode_fill(co, b, slot, shards, S, direct ? dev : nullptr, rs::kSha256Skip);
  };
  return submit_async(co, Kind::kApply, S, false, fill, rec);
}

int rs_co_submit_reconstruct(rs_coalescer* co, uint8_t* const* shards, const size_t* lens, uint64_t tag) {
  if (!co || !shards || !lens) return RS_ERR_INVALID_ARG;
  RecItem it;
  bool need = false;
  const int rc = rec_check(co, shards, const_cast<size_t*>(lens), false, &it, &need);
  if (rc) return rc;
  if (!need) return RS_ERR_NOT_SUPPORTED;  // nothing missing: nothing would be reaped
  rec_direct(co, &it, false);
  AsyncRec rec;
  rec.tag = tag;
  if (!it.direct)  // in place: the kernel writes the missing shards' buffers itself
    for (int i = 0; i < co->k + co->m; ++i)
      if (!lens[i]) rec.out[rec.n_out++] = shards[i];
  return submit_async(
      co, Kind::kApply, it.S, it.parity_used, [&](Batch* b, size_t slot) { rec_fill(co, b, slot, it, false); }, rec);
}

int rs_co_reap(rs_coalescer* co, uint64_t* tags, int* rcs, int max, int timeout_us) {
  if (!co || !tags || !rcs || max <= 0) return -RS_ERR_INVALID_ARG;
  const int m = co->m;
  int got = 0;
  std::unique_lock<std::mutex> lk(co->done_mu);
  for (;;) {
    while (got < max && !co->done.empty()) {
      Batch* b = co->done.front();
      const uint32_t na = b->n_async.load(std::memory_order_relaxed);
      const uint32_t c0 = b->async_cursor;
      const uint32_t take = std::min<uint32_t>(static_cast<uint32_t>(max - got), na - c0);
      b->async_cursor += take;
      if (b->async_cursor == na) co->done.pop_front();
      lk.unlock();
      const int brc = b->rc;
      for (uint32_t j = c0; j < c0 + take; ++j) {
        const AsyncRec& r = b->arec[j];
        if (brc == RS_OK) {
          for (uint32_t o = 0; o < r.n_out; ++o)
            rs::stage_copy(r.out[o], host_at(b, b->o_out + (static_cast<size_t>(r.slot) * m + o) * b->P), b->S, co->nt_copy);
        }
        tags[got] = r.tag;
        rcs[got] = brc;
        ++got;
      }
      release_slots(co, b, take);
      lk.lock();
    }
    if (got > 0 || timeout_us == 0 || co->stop.load(std::memory_order_acquire)) return got;
    if (timeout_us < 0) {
      co->done_cv.wait(lk);
    } else if (co->done_cv.wait_for(lk, std::chrono::microseconds(timeout_us)) == std::cv_status::timeout &&
               co->done.empty()) {
      return 0;
    }
  }
}

// Batched healer repair: the objects a scan found damaged
// (poller.go:227-309 audits one object per goroutine, 10 at a time) go through in
// as few device batches as their shard lengths allow.  Per object exactly
// rs_reconstruct's contract; its code lands in rcs[i].
int rs_co_reconstruct_many(rs_coalescer* co, size_t n_objects, uint8_t* const* shards, size_t* lens, int* rcs) {
  if (!co || (n_objects && (!shards || !lens || !rcs))) return RS_ERR_INVALID_ARG;
  const size_t t = static_cast<size_t>(co->k + co->m);
  co->calls.fetch_add(n_objects, std::memory_order_relaxed);
  std::vector<RecItem> items(n_objects);
  std::map<size_t, std::vector<size_t>> by_len;
  for (size_t i = 0; i < n_objects; ++i) {
    bool need = false;
    rcs[i] = rec_check(co, shards + i * t, lens + i * t, false, &items[i], &need);
    if (need) {
      rec_direct(co, &items[i], false);
      by_len[items[i].S].push_back(i);
    }
  }
  for (auto& g : by_len) {
    const std::vector<size_t>& idx = g.second;
    bool parity_in = false;
    for (size_t i : idx) parity_in |= items[i].parity_used;
    const int rc = submit_many(
        co, Kind::kApply, g.first, idx.size(), parity_in,
        [&](Batch* b, size_t slot, size_t j) { rec_fill(co, b, slot, items[idx[j]], false); },
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
// contract, results in rcs[i]; with value_lens / digests, also each object's
// cold_hash (rs_co_encode_hash's contract).
static int co_encode_many(rs_coalescer* co, size_t n_objects, uint8_t* const* shards, const size_t* lens,
                          const size_t* value_lens, uint8_t* digests, int* rcs) {
  if (!co || (n_objects && (!shards || !lens || !rcs))) return RS_ERR_INVALID_ARG;
  if (n_objects && (value_lens != nullptr) != (digests != nullptr)) return RS_ERR_INVALID_ARG;
  const int k = co->k, m = co->m;
  const size_t t = static_cast<size_t>(k + m);
  const bool hash = value_lens != nullptr;
  co->calls.fetch_add(n_objects, std::memory_order_relaxed);
  std::map<size_t, std::vector<size_t>> by_len;
  for (size_t i = 0; i < n_objects; ++i) {
    size_t S = 0;
    int rc = rs::check_shards(k + m, lens + i * t, false, &S);
    for (size_t j = 0; rc == RS_OK && j < t; ++j)
      if (!shards[i * t + j]) rc = RS_ERR_INVALID_ARG;
    if (rc == RS_OK && S > 0xFFFFFFF0u) rc = RS_ERR_INVALID_ARG;
    if (rc == RS_OK && hash && value_lens[i] > static_cast<uint64_t>(k) * S) rc = RS_ERR_INVALID_ARG;
    if (rc == RS_OK && hash && m == 0) rc = RS_ERR_NOT_SUPPORTED;
    rcs[i] = rc;
    if (rc == RS_OK && m > 0) by_len[S].push_back(i);
  }
  // objects whose shards are all rs_host_alloc'ed run in place (as rs_co_encode's)
  std::vector<uint64_t> devs(co->direct_ok ? n_objects * t : 0);
  std::vector<uint8_t> direct(n_objects, 0);
  for (auto& g : by_len)
    for (size_t i : g.second)
      direct[i] = co->direct_ok && direct_ptrs(co, shards + i * t, g.first, (1u << t) - 1u, &devs[i * t]) &&
                  (!hash || hash_in_place_ok(shards + i * t, g.first, value_lens[i]));
  for (auto& g : by_len) {
    const std::vector<size_t>& idx = g.second;
    const size_t S = g.first;
    const int rc = submit_many(
        co, Kind::kApply, S, idx.size(), false,
        [&](Batch* b, size_t slot, size_t j) {
          const size_t i = idx[j];
          encode_fill(co, b, slot, shards + i * t, S, direct[i] ? &devs[i * t] : nullptr,
                      hash ? value_lens[i] : rs::kSha256Skip);
        },
        [&](Batch* b, size_t slot, size_t j) {
          const size_t i = idx[j];
          uint8_t* const* sh = shards + i * t;
          if (!direct[i])
            for (int r = 0; r < m; ++r) rs::stage_copy(sh[k + r], host_at(b, b->o_out + (slot * m + r) * b->P), S, co->nt_copy);
          if (hash) std::memcpy(digests + i * 32, host_at(b, b->o_digest + slot * 32), 32);
        });
    if (rc) {
      for (size_t i : idx) rcs[i] = rc;
      return rc;
    }
  }
  return RS_OK;
}

int rs_co_encode_many(rs_coalescer* co, size_t n_objects, uint8_t* const* shards, const size_t* lens, int* rcs) {
  return co_encode_many(co, n_objects, shards, lens, nullptr, nullptr, rcs);
}

int rs_co_encode_hash_many(rs_coalescer* co, size_t n_objects, uint8_t* const* shards, const size_t* lens,
                           const size_t* value_lens, uint8_t* digests, int* rcs) {
  if (n_objects && (!value_lens || !digests)) return RS_ERR_INVALID_ARG;
  return co_encode_many(co, n_objects, shards, lens, value_lens, digests, rcs);
}

int rs_co_stats(rs_coalescer* co, uint64_t* calls, uint64_t* batches, uint64_t* stripes, uint64_t* max_batch) {
  if (!co) return RS_ERR_INVALID_ARG;
  if (calls) *calls = co->calls.load();
  if (batches) *batches = co->n_batches.load();
  if (stripes) *stripes = co->stripes.load();
  if (max_batch) *max_batch = co->max_seen.load();
  return RS_OK;
}

int rs_co_timing(rs_coalescer* co, uint64_t* straggle_ns, uint64_t* launch_ns, uint64_t* exec_ns,
                 uint64_t* free_waits) {
  if (!co) return RS_ERR_INVALID_ARG;
  if (straggle_ns) *straggle_ns = co->straggle_ns.load();
  if (launch_ns) *launch_ns = co->launch_ns.load();
  if (exec_ns) *exec_ns = co->exec_ns.load();
  if (free_waits) *free_waits = co->free_waits.load();
  return RS_OK;
}

}  // extern "C"
