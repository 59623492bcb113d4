// test_host_copy.cpp -- the coalescer's staging copy (csrc/rs_host_copy.cpp):
// streaming stores for large copies, memcpy for small ones.  Every length and
// source / destination alignment gives memcpy's bytes and writes nothing outside
// [dst, dst + n).  CPU only; prints "ALL OK".
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <initializer_list>
#include <vector>

namespace rs {
void stage_copy(void* dst, const void* src, size_t n, bool streaming);
}

int main() {
  std::vector<uint8_t> src((4u << 20) + 64);
  uint64_t x = 0x9E3779B97F4A7C15ull;
  for (auto& b : src) {
    x ^= x << 13;
    x ^= x >> 7;
    x ^= x << 17;
    b = static_cast<uint8_t>(x);
  }
  const size_t lens[] = {0, 1, 31, 32, 33, 127, 128, 129, 16383, 16384, 16385, 25600, 100000, 384000, 1u << 20,
                         (1u << 20) + 77, 4u << 20};
  int bad = 0;
  for (bool streaming : {true, false})  // streaming stores and the plain-memcpy A/B setting
  for (size_t n : lens)
    for (size_t so = 0; so < 64; so += 7)
      for (size_t dofs = 0; dofs < 64; dofs += 5) {
        std::vector<uint8_t> d(n + 192, 0xA5);
        rs::stage_copy(d.data() + 64 + dofs, src.data() + so, n, streaming);
        if (std::memcmp(d.data() + 64 + dofs, src.data() + so, n) != 0) ++bad;
        for (size_t i = 0; i < 64 + dofs; ++i)
          if (d[i] != 0xA5) {
            ++bad;
            break;
          }
        for (size_t i = 64 + dofs + n; i < d.size(); ++i)
          if (d[i] != 0xA5) {
            ++bad;
            break;
          }
      }
  if (bad) {
    std::printf("%d bad copies\n", bad);
    return 1;
  }
  std::printf("ALL OK\n");
  return 0;
}
