// coalesce_bench.cpp -- per-object IEcDriver throughput with T concurrent callers
// (the gateway's goroutine-per-request model, cmd/api/main.go:227): direct
// (rs_encode / rs_reconstruct: one H2D->kernel->D2H per object), through the batch
// coalescer (rs_co_*), or the CPU codec on the caller's own thread ("cpu": the
// oracle/ C restatement of klauspost's AVX-512 GFNI / AVX2 kernels with tables
// prepared once, as klauspost keeps them in its Encoder -- the reported baseline,
// single goroutine per call as ec.go:26 configures it).  RS(4+2) objects of
// obj_bytes (4 KiB default; the reference's payloads: 10 / 100 / 800 KiB,
// benchmark/k6/benchmark.js:14-19, and 1500 KiB, go-ycsb hybridstore db.go:56), host
// memory.  Workload per call: "enc" = Encode; "mix" = 50/50 Encode and 1-erasure
// Reconstruct (SURVEY.md §8d config 5's mix); "hash" = the write path's Encode +
// cold_hash of the whole value (writeservice.go:222,267: rs_co_encode_hash; the CPU
// codec plus SHA-256 of the k data shards in "cpu" mode).  Prints one JSON line per run.
//
// Build: g++ -std=c++17 -O2 -pthread tools/coalesce_bench.cpp -o tools/coalesce_bench \
//          -Lreplication_erasurecoding_object_store_amd -lrsgpu \
//          -Wl,-rpath,$PWD/replication_erasurecoding_object_store_amd -Loracle -lrs_oracle \
//          -Wl,-rpath,$PWD/oracle -L/opt/rocm/lib -Wl,-rpath,/opt/rocm/lib
// "async": the coalescer's asynchronous calls (rs_co_submit_* / rs_co_reap), each
// thread an event loop with `depth` calls in flight (the Go shim's model: request
// goroutines park on a channel while one poller reaps).
// REGISTER=1: the objects live in one rs_host_register'ed arena: coalesced calls on
// them run in place (pointer-table kernel, no staging copies).
// ROTATE_MB=<n>: each blocking thread cycles through its share of n MiB of objects
// (DRAM-resident calls, as objects fresh off the network or a disk are) instead of
// re-using one cache-resident object.
// Usage: coalesce_bench <threads> <seconds> <enc|mix> <direct|co|cpu|async|hybrid> [max_batch] [max_wait_us] [obj_bytes] [max_exec] [staged_dma] [inflight] [depth]
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "../include/rsgpu.h"
#include "../oracle/rs_oracle.h"

int main(int argc, char** argv) {
  if (argc < 5) {
    std::fprintf(stderr, "usage: %s threads seconds enc|mix direct|co [max_batch] [max_wait_us] [obj_bytes]\n",
                 argv[0]);
    return 2;
  }
  const int T = std::atoi(argv[1]);
  const double secs = std::atof(argv[2]);
  const bool mix = std::strcmp(argv[3], "mix") == 0;
  const bool hash_wl = std::strcmp(argv[3], "hash") == 0;
  const bool co_mode = std::strcmp(argv[4], "co") == 0;
  const bool cpu_mode = std::strcmp(argv[4], "cpu") == 0;
  // "hybrid": the asynchronous loop, but an object goes to the GPU only while fewer
  // than GPU_LIMIT calls (all threads) are in flight there and the object is at least
  // MIN_OBJ bytes; every other object runs on the CPU codec on the loop's own thread
  // (the Go shim's hybrid dispatch: a call never waits for a full GPU pipeline or a
  // busy staging batch, and objects too small to pay for their staging stay on the
  // CPU -- VERDICT round 5 item 4)
  const bool hybrid_mode = std::strcmp(argv[4], "hybrid") == 0;
  const bool async_mode = hybrid_mode || std::strcmp(argv[4], "async") == 0;  // rs_co_submit_* + rs_co_reap
  const long gpu_limit = std::getenv("GPU_LIMIT") ? std::atol(std::getenv("GPU_LIMIT")) : 256;
  const size_t min_obj = std::getenv("MIN_OBJ") ? std::strtoull(std::getenv("MIN_OBJ"), nullptr, 10) : 0;
  rs_coalescer_opts opts{0, 0, 0, 0, 0, 0, 0};
  if (const char* sw = std::getenv("SPIN")) opts.spin_waiters = std::atoi(sw);  // callers spin-waiting at once
  if (const char* mb = std::getenv("BATCH_MB")) opts.max_batch_bytes = std::strtoull(mb, nullptr, 10) << 20;
  if (const char* pc = std::getenv("PLAIN_COPY")) opts.plain_copy = std::atoi(pc);  // A/B: memcpy staging copies
  if (argc > 5) opts.max_batch = std::strtoull(argv[5], nullptr, 10);
  if (argc > 6) opts.max_wait_us = static_cast<uint32_t>(std::atoi(argv[6]));
  const size_t obj = argc > 7 ? std::strtoull(argv[7], nullptr, 10) : 4096;
  if (argc > 8) opts.max_exec = std::atoi(argv[8]);
  if (argc > 9) opts.staged_dma = std::atoi(argv[9]);
  if (argc > 10) opts.inflight = std::atoi(argv[10]);
  const int k = 4, m = 2;
  rs_ctx* ctx = nullptr;
  if (int rc = rs_create(k, m, 0, 0, &ctx)) {
    std::fprintf(stderr, "rs_create: %s\n", rs_strerror(rc));
    return 1;
  }
  rs_coalescer* co = nullptr;
  if ((co_mode || async_mode) && rs_coalescer_create(ctx, &opts, &co)) return 1;
  const size_t S = rs_shard_size(ctx, obj);
  // CPU codec plans: encode rows, and per lost shard the composed decode row over
  // the first k survivors (klauspost caches decode matrices per erasure pattern)
  void* enc_plan = nullptr;
  std::vector<void*> rec_plan(k + m, nullptr);
  std::vector<std::vector<int>> rec_in(k + m, std::vector<int>(k));
  if (cpu_mode || hybrid_mode) {
    std::vector<uint8_t> mat((k + m) * k);
    rso_build_matrix(k, m, mat.data());
    enc_plan = rso_baseline_plan_new(k, m, mat.data() + k * k);
    for (int lost = 0; lost < k + m; ++lost) {
      std::vector<uint8_t> present(k + m, 1), rows(m * k);
      present[lost] = 0;
      int miss[32], nmiss = 0;
      rso_decode_rows(k, m, present.data(), rec_in[lost].data(), miss, &nmiss, rows.data());
      rec_plan[lost] = rso_baseline_plan_new(k, nmiss, rows.data());
    }
  }
  const int depth = argc > 11 ? std::atoi(argv[11]) : 64;  // async: calls in flight per thread
  const size_t rotate_bytes = std::getenv("ROTATE_MB") ? std::strtoull(std::getenv("ROTATE_MB"), nullptr, 10) << 20 : 0;
  std::atomic<bool> stop{false}, start{false};
  std::atomic<int> ready{0};  // threads done building their objects: the clock starts after all
  std::atomic<uint64_t> ops{0}, bad{0}, busy{0}, cpu_ops{0};
  std::atomic<long> gpu_inflight{0};  // hybrid: calls submitted and not yet reaped (all threads)
  std::vector<std::thread> ts;
  // One object's k+m shards; the reference parity comes from a direct call, and
  // before every call the shards it must write are scribbled, so a call that writes
  // nothing cannot pass.
  struct Obj {
    std::vector<std::vector<uint8_t>> sh, keep;
    uint8_t digest[32];  // SHA-256 of the value (the k data shards in order)
    std::vector<uint8_t*> p;
    std::vector<size_t> n;
    uint64_t j = 0;
  };
  // REGISTER=1: every object's shards live in one rs_host_register'ed arena (the
  // gateway's request bodies / the healer's shard buffers in a pinned arena), so
  // coalesced calls run in place (no staging copies); else per-shard heap vectors.
  // REGISTER=2: the arena comes from rs_host_alloc (context-owned page-locked memory).
  const int reg_mode = std::getenv("REGISTER") ? std::atoi(std::getenv("REGISTER")) : 0;
  const bool reg = reg_mode != 0;
  const size_t SP = (S + 63) / 64 * 64;
  // objects per thread: blocking and hybrid threads cycle through their share of
  // ROTATE_MB (DRAM-resident calls); an asynchronous GPU loop holds `depth` in flight
  const size_t rot_share = std::max<size_t>(1, rotate_bytes / (static_cast<size_t>(T) * (k + m) * S));
  const size_t per_thread = hybrid_mode  ? std::max<size_t>(static_cast<size_t>(depth), rot_share)
                            : async_mode ? static_cast<size_t>(depth)
                                         : rot_share;
  std::unique_ptr<std::atomic<int>[]> done_word(new std::atomic<int>[static_cast<size_t>(T) * per_thread]);
  for (size_t i = 0; i < static_cast<size_t>(T) * per_thread; ++i) done_word[i].store(0);
  uint8_t* arena = nullptr;
  size_t arena_bytes = 0;
  if (reg) {
    arena_bytes = static_cast<size_t>(T) * per_thread * (k + m) * SP;
    void* p = nullptr;
    if (reg_mode == 2) {
      if (rs_host_alloc(ctx, arena_bytes, &p) != RS_OK) p = nullptr;
      arena = static_cast<uint8_t*>(p);
    } else {
      arena = static_cast<uint8_t*>(std::aligned_alloc(4096, (arena_bytes + 4095) / 4096 * 4096));
      if (arena && rs_host_register(ctx, arena, arena_bytes) != RS_OK) arena = nullptr;  // (leaks: exits)
    }
    if (!arena) {
      std::fprintf(stderr, "REGISTER: arena of %zu bytes failed\n", arena_bytes);
      return 1;
    }
  }
  auto make_obj = [&](uint64_t seed, size_t place) {
    Obj o;
    o.sh.assign(k + m, std::vector<uint8_t>(S));
    uint64_t x = 0x9E3779B97F4A7C15ull * (seed + 1);
    for (int i = 0; i < k; ++i)
      for (auto& b : o.sh[i]) {
        x ^= x << 13;
        x ^= x >> 7;
        x ^= x << 17;
        b = static_cast<uint8_t>(x);
      }
    o.p.resize(k + m);
    o.n.assign(k + m, S);
    for (int i = 0; i < k + m; ++i) {
      if (arena) {
        o.p[i] = arena + (place * (k + m) + i) * SP;
        std::memcpy(o.p[i], o.sh[i].data(), S);
      } else {
        o.p[i] = o.sh[i].data();
      }
    }
    if (rs_encode(ctx, o.p.data(), o.n.data()) != RS_OK) ++bad;
    {
      std::vector<uint8_t> value;
      for (int i = 0; i < k; ++i) value.insert(value.end(), o.p[i], o.p[i] + S);
      rso_sha256(value.data(), value.size(), o.digest);
    }
    o.keep.assign(k + m, std::vector<uint8_t>(S));
    for (int i = 0; i < k + m; ++i) std::memcpy(o.keep[i].data(), o.p[i], S);
    if (arena) o.sh.clear();  // the arena holds the shards
    return o;
  };
  // Call j of an object: every 7th pair (an encode and a reconstruct
  // each) scribbles the shards it must write and is checked byte-for-byte after;
  // the others rewrite identical bytes unchecked (a full compare of every call
  // would cost as much CPU as the codec itself at large objects).
  auto verified = [&](const Obj& o) { return (o.j >> 1) % 7 == 0; };  // 7: every lost index in turn
  // prepares call j: returns the lost shard (-1: encode), lens set
  auto prep = [&](Obj& o) -> int {
    o.n.assign(k + m, S);
    const bool v = verified(o);
    if (mix && (o.j & 1)) {
      const int lost = static_cast<int>((o.j >> 1) % (k + m));
      o.n[lost] = 0;
      if (v) std::memset(o.p[lost], 0x5a, S);
      return lost;
    }
    if (v)
      for (int r = 0; r < m; ++r) std::memset(o.p[k + r], 0x5a, S);
    return -1;
  };
  auto check = [&](Obj& o) -> uint64_t {
    uint64_t e = 0;
    if (verified(o))
      for (int i = 0; i < k + m; ++i)
        if (std::memcmp(o.p[i], o.keep[i].data(), S) != 0) {
          ++e;
          std::memcpy(o.p[i], o.keep[i].data(), S);
        }
    ++o.j;
    return e;
  };
  // the CPU codec on this thread for the call prep() set up (lost < 0: encode)
  auto cpu_call = [&](Obj& o, int lost) -> int {
    if (lost >= 0) {
      const uint8_t* in[32];
      for (int c = 0; c < k; ++c) in[c] = o.p[rec_in[lost][c]];
      uint8_t* out[1] = {o.p[lost]};
      return rso_baseline_plan_apply(rec_plan[lost], in, out, S) >= 0 ? RS_OK : RS_ERR_DEVICE;
    }
    return rso_baseline_plan_apply(enc_plan, o.p.data(), o.p.data() + k, S) >= 0 ? RS_OK : RS_ERR_DEVICE;
  };
  const bool gpu_size_ok = static_cast<size_t>(k) * S >= min_obj;
  for (int t = 0; t < T; ++t)
    ts.emplace_back([&, t] {
      if (async_mode) {
        // An event loop with `depth` calls in flight.  Reaping is global (any thread
        // may reap any call, as the Go shim's single reaper goroutine does), so a
        // reaped tag = (thread << 32 | object) is routed to its owner through a
        // completion word; each loop then handles its own completed objects.
        const int npool = static_cast<int>(per_thread);
        std::vector<Obj> objs;
        for (int d = 0; d < npool; ++d)
          objs.push_back(make_obj(static_cast<uint64_t>(t) * npool + d, static_cast<size_t>(t) * per_thread + d));
        std::deque<int> idle;  // in rotation order: the least recently used object first
        for (int d = 0; d < npool; ++d) idle.push_back(d);
        std::vector<int> flying;  // submitted, not yet completed
        auto last_reap = std::chrono::steady_clock::now();
        std::vector<uint64_t> tags(256);
        std::vector<int> rcs(256);
        std::atomic<int>* mine_done = &done_word[static_cast<size_t>(t) * per_thread];
        ++ready;
        while (!start.load()) std::this_thread::yield();
        uint64_t mine = 0, nb = 0, e = 0, inflight = 0, on_cpu = 0;
        while (!stop.load(std::memory_order_relaxed) || inflight) {
          bool cpu_ran = false;
          while (!idle.empty() && !stop.load(std::memory_order_relaxed)) {
            const int d = idle.front();
            Obj& o = objs[d];
            const int lost = prep(o);
            bool to_gpu = true;
            if (hybrid_mode) {
              to_gpu = gpu_size_ok && gpu_inflight.fetch_add(1, std::memory_order_relaxed) < gpu_limit;
              if (gpu_size_ok && !to_gpu) gpu_inflight.fetch_sub(1, std::memory_order_relaxed);
            }
            int rc = RS_ERR_BUSY;
            if (to_gpu) {
              const uint64_t tag = (static_cast<uint64_t>(t) << 32) | static_cast<uint64_t>(d);
              rc = lost < 0 ? rs_co_submit_encode(co, o.p.data(), o.n.data(), tag)
                            : rs_co_submit_reconstruct(co, o.p.data(), o.n.data(), tag);
              if (rc != RS_OK && hybrid_mode) gpu_inflight.fetch_sub(1, std::memory_order_relaxed);
            }
            if (rc == RS_ERR_BUSY && hybrid_mode) {
              // GPU pipeline full or no free staging batch: this thread does the call
              if (to_gpu) ++nb;
              if (cpu_call(o, lost) != RS_OK) ++e;
              e += check(o);
              ++mine;
              ++on_cpu;
              cpu_ran = true;
              idle.pop_front();
              idle.push_back(d);  // to the back of the rotation
              break;  // one CPU call, then reap what the GPU finished meanwhile
            }
            if (rc == RS_ERR_BUSY) {
              ++nb;
              break;
            }
            if (rc != RS_OK) {
              ++e;
              break;
            }
            idle.pop_front();
            flying.push_back(d);
            ++inflight;
          }
          if (!inflight) continue;
          if (cpu_ran) {
            // between CPU calls, poll the GPU's completions at most every 20 us: a reap
            // costs about as much as a 4 KiB CPU call
            const auto now = std::chrono::steady_clock::now();
            if (now - last_reap < std::chrono::microseconds(20)) continue;
            last_reap = now;
          }
          const int got = rs_co_reap(co, tags.data(), rcs.data(), 256, cpu_ran ? 0 : 50);
          if (hybrid_mode && got > 0) gpu_inflight.fetch_sub(got, std::memory_order_relaxed);
          for (int g = 0; g < got; ++g)
            done_word[(tags[g] >> 32) * static_cast<uint64_t>(per_thread) + (tags[g] & 0xFFFFFFFFu)].store(
                rcs[g] + 1, std::memory_order_release);
          for (size_t q = 0; q < flying.size();) {  // this loop's calls in flight
            const int d = flying[q];
            const int v = mine_done[d].load(std::memory_order_acquire);
            if (!v) {
              ++q;
              continue;
            }
            flying[q] = flying.back();
            flying.pop_back();
            mine_done[d].store(0, std::memory_order_relaxed);
            if (v - 1 != RS_OK) ++e;
            e += check(objs[d]);
            idle.push_back(d);
            --inflight;
            ++mine;
          }
        }
        ops += mine;
        bad += e;
        busy += nb;
        cpu_ops += on_cpu;
        return;
      }
      // ROTATE_MB: the thread cycles through its share of that many MiB of objects,
      // so calls find their object in DRAM instead of the cache (1 GiB >> the host's
      // 256 MiB of L3); default one object, cache-resident after the first call
      const size_t npool = per_thread;
      std::vector<Obj> pool;
      for (size_t i = 0; i < npool; ++i)
        pool.push_back(make_obj(static_cast<uint64_t>(t) * npool + i, static_cast<size_t>(t) * npool + i));
      size_t cur = 0;
      ++ready;
      while (!start.load()) std::this_thread::yield();
      uint64_t mine = 0;
      while (!stop.load(std::memory_order_relaxed)) {
        Obj& o = pool[cur];
        cur = cur + 1 == npool ? 0 : cur + 1;
        int rc;
        const int lost = prep(o);
        if (lost >= 0) {
          if (cpu_mode) {
            rc = cpu_call(o, lost);
          } else {
            rc = co ? rs_co_reconstruct(co, o.p.data(), o.n.data()) : rs_reconstruct(ctx, o.p.data(), o.n.data());
          }
        } else if (hash_wl) {
          uint8_t dg[32];
          if (cpu_mode) {
            rc = rso_baseline_plan_apply(enc_plan, o.p.data(), o.p.data() + k, S) >= 0 ? RS_OK : RS_ERR_DEVICE;
            // SHA-NI on this thread (Go's crypto/sha256 class of code), the same bytes
            // hashed shard by shard
            for (int c = 0; c < k; ++c) rso_baseline_sha256_batch(o.p[c], 0, S, 1, dg, 1);
          } else {
            rc = co ? rs_co_encode_hash(co, o.p.data(), o.n.data(), static_cast<size_t>(k) * S, dg) : RS_ERR_INVALID_ARG;
            if (rc == RS_OK && verified(o) && std::memcmp(dg, o.digest, 32) != 0) ++bad;
          }
        } else {
          if (cpu_mode)
            rc = cpu_call(o, -1);
          else
            rc = co ? rs_co_encode(co, o.p.data(), o.n.data()) : rs_encode(ctx, o.p.data(), o.n.data());
        }
        if (rc != RS_OK) ++bad;
        bad += check(o);
        ++mine;
      }
      ops += mine;
    });
  while (ready.load() < T) std::this_thread::sleep_for(std::chrono::milliseconds(1));
  start = true;
  const auto t0 = std::chrono::steady_clock::now();
  std::this_thread::sleep_for(std::chrono::duration<double>(secs));
  stop = true;
  for (auto& th : ts) th.join();
  const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  uint64_t calls = 0, batches = 0, stripes = 0, maxb = 0;
  if (co) rs_co_stats(co, &calls, &batches, &stripes, &maxb);
  const double n_ops = static_cast<double>(ops.load());
  std::printf(
      "{\"mode\": \"%s\", \"workload\": \"%s\", \"threads\": %d, \"obj_bytes\": %zu, \"seconds\": %.2f, "
      "\"calls_per_s\": %.0f, \"user_GiBps\": %.3f, \"errors\": %llu, \"batches\": %llu, \"avg_batch\": %.1f, "
      "\"max_batch\": %llu, \"max_exec\": %d, \"max_wait_us\": %u, \"staged_dma\": %d, \"inflight\": %d, "
      "\"depth\": %d, \"busy\": %llu, \"rotate_mb\": %zu, \"registered\": %d, \"gpu_limit\": %ld, "
      "\"min_obj\": %zu, \"cpu_share\": %.3f}\n",
      hybrid_mode ? "hybrid" : async_mode ? "async" : (co ? "coalesced" : (cpu_mode ? "cpu" : "direct")), mix ? "mix" : (hash_wl ? "hash" : "enc"), T, obj, dt,
      n_ops / dt, n_ops * static_cast<double>(k * S) / dt / (1 << 30), static_cast<unsigned long long>(bad.load()),
      static_cast<unsigned long long>(batches), batches ? static_cast<double>(stripes) / batches : 0.0,
      static_cast<unsigned long long>(maxb), opts.max_exec, opts.max_wait_us, opts.staged_dma, opts.inflight,
      async_mode ? depth : 0, static_cast<unsigned long long>(busy.load()), rotate_bytes >> 20, reg_mode,
      hybrid_mode ? gpu_limit : 0L, hybrid_mode ? min_obj : size_t(0),
      n_ops > 0 ? static_cast<double>(cpu_ops.load()) / n_ops : 0.0);
  if (co && std::getenv("CO_TIMING")) {  // launcher diagnostics (rs_co_timing)
    uint64_t st = 0, la = 0, ex = 0, fw = 0, nb = 0;
    rs_co_timing(co, &st, &la, &ex, &fw);
    rs_co_stats(co, nullptr, &nb, nullptr, nullptr);
    std::fprintf(stderr, "[rs_coalescer] batches %llu straggle_ms %.1f launch_ms %.1f exec_ms %.1f free_waits %llu\n",
                 (unsigned long long)nb, st / 1e6, la / 1e6, ex / 1e6, (unsigned long long)fw);
  }
  if (co) rs_coalescer_destroy(co);
  if (arena) {
    if (reg_mode == 2) {
      rs_host_free(ctx, arena);
    } else {
      rs_host_unregister(ctx, arena);
      std::free(arena);
    }
  }
  if (enc_plan) rso_baseline_plan_free(enc_plan);
  for (void* pl : rec_plan)
    if (pl) rso_baseline_plan_free(pl);
  rs_destroy(ctx);
  return bad.load() ? 1 : 0;
}
