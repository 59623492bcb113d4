// rs_host_util.hpp -- host-side helpers shared by rs_engine.cpp and
// rs_coalescer.cpp (internal to librsgpu.so; not part of the C-ABI).
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>

#include "../../include/rsgpu.h"

namespace rs {

#define RS_HIP(expr)                                \
  do {                                              \
    if ((expr) != hipSuccess) return RS_ERR_DEVICE; \
  } while (0)

inline size_t round_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

// [upstream reedsolomon.go checkShards]: the first non-empty length is S; every
// other shard must match it (empty allowed only where nilok).
inline int check_shards(int n, const size_t* lens, bool nilok, size_t* S) {
  size_t s = 0;
  for (int i = 0; i < n; ++i)
    if (lens[i]) {
      s = lens[i];
      break;
    }
  if (s == 0) return RS_ERR_SHARD_NO_DATA;
  for (int i = 0; i < n; ++i)
    if (lens[i] != s && (lens[i] != 0 || !nilok)) return RS_ERR_SHARD_SIZE;
  *S = s;
  return RS_OK;
}

// Pinned host allocation usable by every GPU of the process (portable), placed on
// `numa_node` when >= 0 (the GPU's own node, so its DMA and zero-copy traffic stays
// off the inter-socket link).  Returns nullptr on failure.  (rs_engine.cpp)
void* pinned_alloc(size_t bytes, int numa_node);
void pinned_free(void* p);
// NUMA node of a GPU from sysfs (-1 if unknown).
int device_numa_node(int device);
// Copy into / out of pinned staging: streaming stores for shard-sized copies unless
// `streaming` is false (the coalescer's opts.plain_copy A/B setting; rs_host_copy.cpp).
void stage_copy(void* dst, const void* src, size_t n, bool streaming = true);

// Device memory on the calling thread's current device (callers hold a
// DeviceScope).  ensure() only grows; hipFree synchronises the device first, so
// growing under in-flight work is safe, just slow.
struct DevBuf {
  void* p = nullptr;
  size_t n = 0;
  int ensure(size_t bytes) {
    if (bytes <= n) return RS_OK;
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
    if (hipMalloc(&p, bytes) != hipSuccess) return RS_ERR_DEVICE;
    n = bytes;
    return RS_OK;
  }
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
};

struct PinnedBuf {
  void* p = nullptr;
  size_t n = 0;
  int numa = -1;  // NUMA node to place the pages on (-1: the allocating thread's)
  int ensure(size_t bytes) {
    if (bytes <= n) return RS_OK;
    if (p) pinned_free(p);
    n = 0;
    p = pinned_alloc(bytes, numa);
    if (!p) return RS_ERR_DEVICE;
    n = bytes;
    return RS_OK;
  }
  PinnedBuf() = default;
  PinnedBuf(const PinnedBuf&) = delete;
  PinnedBuf& operator=(const PinnedBuf&) = delete;
  ~PinnedBuf() {
    if (p) pinned_free(p);
  }
};

}  // namespace rs
