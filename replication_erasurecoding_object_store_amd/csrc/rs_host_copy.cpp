// rs_host_copy.cpp -- host-only helpers of librsgpu.so built by the host compiler
// (x86 intrinsics and CPU-feature builtins have no meaning in a HIP translation
// unit's device pass).
#include <immintrin.h>

#include <algorithm>
#include <cstdint>
#include <cstring>

namespace rs {

void stage_copy(void* dst, const void* src, size_t n, bool streaming);  // rs_host_util.hpp

namespace {

// Copies into and out of the pinned staging (the callers' share of a per-object
// call).  Shard-sized copies use streaming (non-temporal) stores: the CPU never
// reads the destination back soon -- the GPU reads the staging over PCIe, an output
// buffer goes to the network -- and a streaming store skips the read-for-ownership
// of every destination line, a third of a cached copy's DRAM traffic.  Small copies
// stay with memcpy.  The coalescer's opts.plain_copy turns streaming off (A/B).
constexpr size_t kStreamMin = 16 << 10;

__attribute__((target("avx2"))) void copy_streaming(uint8_t* dst, const uint8_t* src, size_t n) {
  const size_t head = std::min(n, (32 - (reinterpret_cast<uintptr_t>(dst) & 31)) & 31);
  std::memcpy(dst, src, head);
  dst += head;
  src += head;
  n -= head;
  size_t i = 0;
  for (; i + 128 <= n; i += 128) {
    const __m256i a = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + i));
    const __m256i b = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + i + 32));
    const __m256i c = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + i + 64));
    const __m256i d = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + i + 96));
    _mm256_stream_si256(reinterpret_cast<__m256i*>(dst + i), a);
    _mm256_stream_si256(reinterpret_cast<__m256i*>(dst + i + 32), b);
    _mm256_stream_si256(reinterpret_cast<__m256i*>(dst + i + 64), c);
    _mm256_stream_si256(reinterpret_cast<__m256i*>(dst + i + 96), d);
  }
  for (; i + 32 <= n; i += 32)
    _mm256_stream_si256(reinterpret_cast<__m256i*>(dst + i),
                        _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + i)));
  std::memcpy(dst + i, src + i, n - i);
  _mm_sfence();  // the streamed lines are globally visible before the slot is published
}

bool have_avx2() {
  __builtin_cpu_init();
  return __builtin_cpu_supports("avx2");
}

}  // namespace

void stage_copy(void* dst, const void* src, size_t n, bool streaming) {
  static const bool avx2 = have_avx2();
  if (streaming && avx2 && n >= kStreamMin)
    copy_streaming(static_cast<uint8_t*>(dst), static_cast<const uint8_t*>(src), n);
  else
    std::memcpy(dst, src, n);
}

}  // namespace rs
