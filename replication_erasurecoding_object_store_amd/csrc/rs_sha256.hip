// rs_sha256.hip -- batched SHA-256 on gfx950: the reference's per-write
// "cold_hash" (writeservice.go:51-54 computeSHA256Hex = hex(crypto/sha256.Sum256),
// stored at :267 and compared at :326-327 to skip re-encoding unchanged cold
// fields), computed for a whole batch of objects next to the encode (SURVEY.md
// §8f rank 4).  FIPS 180-4; checked against oracle/sha256_oracle.c and hashlib.
//
// One lane per message: SHA-256 is a serial chain of 64-byte blocks, so the
// parallelism is across objects (65 536 objects = 1 024 waves).  64-thread blocks
// spread the waves over every CU.  All 64 rounds and the message schedule are
// unrolled: round constants become literals, the 16-word schedule window lives in
// VGPRs, rotations are v_alignbit_b32, Ch / Maj single v_bitop3_b32, the five-way
// sums v_add3_u32.  Messages are read as big-endian dwords (4-B loads + byte
// swap) when they start 4-B aligned, bytewise otherwise; the partial last word,
// the 0x80 terminator and the bit length are assembled in registers, so nothing
// past a message's last byte is ever read.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rs_sha256.hpp"

namespace rs {

namespace {

__device__ __forceinline__ uint32_t rotr(uint32_t x, int n) { return __builtin_amdgcn_alignbit(x, x, n); }
// 3-input XOR in one v_bitop3_b32 (truth table 0x96); the compiler does not form it
// from a ^ b ^ c on its own here.
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

struct State {
  uint32_t h[8];
};

__device__ __forceinline__ void compress(State& s, uint32_t (&w)[16]) {
  constexpr uint32_t kK[64] = {
      0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
      0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
      0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
      0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
      0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
      0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
      0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
      0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};
  uint32_t a = s.h[0], b = s.h[1], c = s.h[2], d = s.h[3], e = s.h[4], f = s.h[5], g = s.h[6], h = s.h[7];
#pragma unroll
  for (int t = 0; t < 64; ++t) {
    if (t >= 16) {
      const uint32_t w15 = w[(t - 15) & 15], w2 = w[(t - 2) & 15];
      const uint32_t s0 = xor3(rotr(w15, 7), rotr(w15, 18), w15 >> 3);
      const uint32_t s1 = xor3(rotr(w2, 17), rotr(w2, 19), w2 >> 10);
      w[t & 15] = w[t & 15] + s0 + w[(t - 7) & 15] + s1;
    }
    const uint32_t S1 = xor3(rotr(e, 6), rotr(e, 11), rotr(e, 25));
    const uint32_t ch = (e & f) ^ (~e & g);
    const uint32_t t1 = h + S1 + ch + kK[t] + w[t & 15];
    const uint32_t S0 = xor3(rotr(a, 2), rotr(a, 13), rotr(a, 22));
    const uint32_t maj = (a & b) ^ (a & c) ^ (b & c);
    h = g;
    g = f;
    f = e;
    e = d + t1;
    d = c;
    c = b;
    b = a;
    a = t1 + S0 + maj;
  }
  s.h[0] += a;
  s.h[1] += b;
  s.h[2] += c;
  s.h[3] += d;
  s.h[4] += e;
  s.h[5] += f;
  s.h[6] += g;
  s.h[7] += h;
}

// Big-endian word at message byte offset `off` (< len), message bytes only.
__device__ __forceinline__ uint32_t load_word(const uint8_t* p, uint64_t off, uint64_t len, bool aligned) {
  if (off + 4 <= len) {
    if (aligned) return __builtin_bswap32(*reinterpret_cast<const uint32_t*>(p + off));
    return static_cast<uint32_t>(p[off]) << 24 | static_cast<uint32_t>(p[off + 1]) << 16 |
           static_cast<uint32_t>(p[off + 2]) << 8 | p[off + 3];
  }
  uint32_t v = 0;
  for (uint32_t q = 0; q < 4; ++q) {
    const uint64_t o = off + q;
    const uint32_t byte = o < len ? p[o] : (o == len ? 0x80u : 0u);  // FIPS 180-4 §5.1.1 terminator
    v |= byte << (24 - 8 * q);
  }
  return v;
}

// Message byte `off` of a chunked message (see Sha256Args).
__device__ __forceinline__ const uint8_t* chunk_addr(const uint8_t* p, uint64_t off, uint64_t chunk, uint64_t pitch) {
  const uint64_t c = off / chunk;
  return p + c * pitch + (off - c * chunk);
}

// Big-endian word at message byte offset `off` of a chunked message (bytes past len:
// the 0x80 terminator, then zeros).
__device__ __forceinline__ uint32_t load_word_chunked(const uint8_t* p, uint64_t off, uint64_t len, uint64_t chunk,
                                                      uint64_t pitch) {
  uint32_t v = 0;
  for (uint32_t q = 0; q < 4; ++q) {
    const uint64_t o = off + q;
    const uint32_t byte = o < len ? *chunk_addr(p, o, chunk, pitch) : (o == len ? 0x80u : 0u);
    v |= byte << (24 - 8 * q);
  }
  return v;
}

__global__ __launch_bounds__(64) void sha256_kernel(Sha256Args a) {
  const uint32_t i = blockIdx.x * 64u + threadIdx.x;
  if (i >= a.n) return;
  const uint64_t len = a.lens ? a.lens[i] : a.len;
  if (len == kSha256Skip) return;
  const uint8_t* p = a.base + (a.offsets ? a.offsets[i] : static_cast<uint64_t>(i) * a.stride);
  const bool chunked = a.chunk != 0 && len > a.chunk;  // a message inside its first chunk is contiguous
  const bool aligned = (reinterpret_cast<uintptr_t>(p) & 3u) == 0;
  const uint64_t nblocks = (len + 8u) / 64u + 1u;  // message + 0x80 + 64-bit length, padded
  State s = {{0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au, 0x510e527fu, 0x9b05688cu, 0x1f83d9abu,
              0x5be0cd19u}};
  const uint64_t full = len / 64u;  // blocks made of message bytes only
  for (uint64_t blk = 0; blk < full; ++blk) {
    uint32_t w[16];
    const uint64_t o0 = blk * 64u;
    const uint8_t* q = p + o0;
    bool fast = aligned;
    if (chunked) {  // contiguous only if the block lies in one chunk
      const uint64_t c0 = o0 / a.chunk;
      q = p + c0 * a.chunk_pitch + (o0 - c0 * a.chunk);
      fast = (o0 + 63u) / a.chunk == c0 && (reinterpret_cast<uintptr_t>(q) & 3u) == 0;
    }
    if (fast) {
#pragma unroll
      for (int t = 0; t < 16; ++t) w[t] = __builtin_bswap32(reinterpret_cast<const uint32_t*>(q)[t]);
    } else if (!chunked) {
#pragma unroll
      for (int t = 0; t < 16; ++t)
        w[t] = static_cast<uint32_t>(q[4 * t]) << 24 | static_cast<uint32_t>(q[4 * t + 1]) << 16 |
               static_cast<uint32_t>(q[4 * t + 2]) << 8 | q[4 * t + 3];
    } else {
      for (int t = 0; t < 16; ++t) w[t] = load_word_chunked(p, o0 + 4u * t, len, a.chunk, a.chunk_pitch);
    }
    compress(s, w);
  }
  for (uint64_t blk = full; blk < nblocks; ++blk) {  // 1 or 2 padded blocks
    uint32_t w[16];
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      const uint64_t off = blk * 64u + 4u * t;
      w[t] = off > len ? 0u
             : chunked ? load_word_chunked(p, off, len, a.chunk, a.chunk_pitch)
                       : load_word(p, off, len, aligned);
    }
    if (blk + 1 == nblocks) {
      const uint64_t bits = len * 8u;
      w[14] = static_cast<uint32_t>(bits >> 32);
      w[15] = static_cast<uint32_t>(bits);
    }
    compress(s, w);
  }
  uint32_t* o = reinterpret_cast<uint32_t*>(a.out + static_cast<uint64_t>(i) * 32u);
#pragma unroll
  for (int q = 0; q < 8; ++q) o[q] = __builtin_bswap32(s.h[q]);
}

}  // namespace

int launch_sha256(const Sha256Args& a, hipStream_t s) {
  if (a.n == 0) return 0;
  const uint32_t grid = (a.n + 63u) / 64u;
  hipLaunchKernelGGL(sha256_kernel, dim3(grid), dim3(64), 0, s, a);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace rs
