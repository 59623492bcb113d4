// coalesce_bench.cpp -- per-object IEcDriver throughput with T concurrent callers
// (the gateway's goroutine-per-request model, cmd/api/main.go:227), direct
// (rs_encode / rs_reconstruct: one H2D->kernel->D2H per object) vs through the
// batch coalescer (rs_co_*).  Objects: 4 KiB RS(4+2) (S = 1024), host memory.
// Workload per call: "enc" = Encode; "mix" = 50/50 Encode and 1-erasure
// Reconstruct (SURVEY.md §8d config 5's mix).  Prints one JSON line per run.
//
// Build: g++ -std=c++17 -O2 -pthread tools/coalesce_bench.cpp -o tools/coalesce_bench \
//          -Ireplication_erasurecoding_object_store_amd -Lreplication_erasurecoding_object_store_amd \
//          -lrsgpu -Wl,-rpath,$PWD/replication_erasurecoding_object_store_amd \
//          -L/opt/rocm/lib -Wl,-rpath,/opt/rocm/lib
// Usage: coalesce_bench <threads> <seconds> <enc|mix> <direct|co> [max_batch] [max_wait_us] [obj_bytes] [max_exec] [staged_dma] [inflight]
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../include/rsgpu.h"

int main(int argc, char** argv) {
  if (argc < 5) {
    std::fprintf(stderr, "usage: %s threads seconds enc|mix direct|co [max_batch] [max_wait_us] [obj_bytes]\n",
                 argv[0]);
    return 2;
  }
  const int T = std::atoi(argv[1]);
  const double secs = std::atof(argv[2]);
  const bool mix = std::strcmp(argv[3], "mix") == 0;
  const bool co_mode = std::strcmp(argv[4], "co") == 0;
  rs_coalescer_opts opts{0, 0, 0, 0, 0, 0};
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
  if (co_mode && rs_coalescer_create(ctx, &opts, &co)) return 1;
  const size_t S = rs_shard_size(ctx, obj);
  std::atomic<bool> stop{false}, start{false};
  std::atomic<uint64_t> ops{0}, bad{0};
  std::vector<std::thread> ts;
  for (int t = 0; t < T; ++t)
    ts.emplace_back([&, t] {
      std::vector<std::vector<uint8_t>> sh(k + m, std::vector<uint8_t>(S));
      uint64_t x = 0x9E3779B97F4A7C15ull * (t + 1);
      for (int i = 0; i < k; ++i)
        for (auto& b : sh[i]) {
          x ^= x << 13;
          x ^= x >> 7;
          x ^= x << 17;
          b = static_cast<uint8_t>(x);
        }
      std::vector<uint8_t*> p(k + m);
      std::vector<size_t> n(k + m, S);
      for (int i = 0; i < k + m; ++i) p[i] = sh[i].data();
      // reference parity from a direct call; every later call must reproduce all
      // k+m shards byte for byte (data is never changed, so parity is constant)
      if (rs_encode(ctx, p.data(), n.data()) != RS_OK) ++bad;
      const std::vector<std::vector<uint8_t>> keep = sh;
      while (!start.load()) std::this_thread::yield();
      uint64_t j = 0, mine = 0;
      while (!stop.load(std::memory_order_relaxed)) {
        int rc;
        if (mix && (j & 1)) {
          const int lost = static_cast<int>((j >> 1) % (k + m));
          n.assign(k + m, S);
          n[lost] = 0;
          rc = co ? rs_co_reconstruct(co, p.data(), n.data()) : rs_reconstruct(ctx, p.data(), n.data());
        } else {
          n.assign(k + m, S);
          rc = co ? rs_co_encode(co, p.data(), n.data()) : rs_encode(ctx, p.data(), n.data());
        }
        if (rc != RS_OK) ++bad;
        for (int i = 0; i < k + m; ++i)
          if (std::memcmp(sh[i].data(), keep[i].data(), S) != 0) {
            ++bad;
            std::memcpy(sh[i].data(), keep[i].data(), S);
          }
        ++j;
        ++mine;
      }
      ops += mine;
    });
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
      "\"max_batch\": %llu, \"max_exec\": %d, \"max_wait_us\": %u, \"staged_dma\": %d, \"inflight\": %d}\n",
      co ? "coalesced" : "direct", mix ? "mix" : "enc", T, obj, dt, n_ops / dt,
      n_ops * static_cast<double>(k * S) / dt / (1 << 30), static_cast<unsigned long long>(bad.load()),
      static_cast<unsigned long long>(batches), batches ? static_cast<double>(stripes) / batches : 0.0,
      static_cast<unsigned long long>(maxb), opts.max_exec, opts.max_wait_us, opts.staged_dma, opts.inflight);
  if (co) rs_coalescer_destroy(co);
  rs_destroy(ctx);
  return bad.load() ? 1 : 0;
}
