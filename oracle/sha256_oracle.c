/* sha256_oracle.c -- TEST INFRASTRUCTURE ONLY (checker for the GPU batched
 * SHA-256, never linked into the product).
 *
 * Scalar restatement of FIPS 180-4 SHA-256, the function the reference applies to
 * every EC-written value: writeservice.go:51-54 computeSHA256Hex(data) =
 * hex(crypto/sha256.Sum256(data)), stored as metadata "cold_hash"
 * (writeservice.go:267, :326-327, :433-436).  Pinned by the FIPS 180-2 appendix
 * vectors ("abc", the empty string, the 448-bit message) in tests/test_oracle.py,
 * and cross-checked against Python's hashlib there.
 */
#include <stddef.h>
#include <stdint.h>
#include <string.h>

#include "rs_oracle.h"

static const uint32_t K256[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

static uint32_t rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

/* FIPS 180-4 §6.2.2: one 512-bit block */
static void compress(uint32_t h[8], const uint8_t blk[64]) {
  uint32_t w[64];
  for (int t = 0; t < 16; ++t)
    w[t] = (uint32_t)blk[4 * t] << 24 | (uint32_t)blk[4 * t + 1] << 16 | (uint32_t)blk[4 * t + 2] << 8 | blk[4 * t + 3];
  for (int t = 16; t < 64; ++t) {
    const uint32_t s0 = rotr(w[t - 15], 7) ^ rotr(w[t - 15], 18) ^ (w[t - 15] >> 3);
    const uint32_t s1 = rotr(w[t - 2], 17) ^ rotr(w[t - 2], 19) ^ (w[t - 2] >> 10);
    w[t] = w[t - 16] + s0 + w[t - 7] + s1;
  }
  uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
  for (int t = 0; t < 64; ++t) {
    const uint32_t S1 = rotr(e, 6) ^ rotr(e, 11) ^ rotr(e, 25);
    const uint32_t ch = (e & f) ^ (~e & g);
    const uint32_t t1 = hh + S1 + ch + K256[t] + w[t];
    const uint32_t S0 = rotr(a, 2) ^ rotr(a, 13) ^ rotr(a, 22);
    const uint32_t maj = (a & b) ^ (a & c) ^ (b & c);
    const uint32_t t2 = S0 + maj;
    hh = g;
    g = f;
    f = e;
    e = d + t1;
    d = c;
    c = b;
    b = a;
    a = t1 + t2;
  }
  h[0] += a;
  h[1] += b;
  h[2] += c;
  h[3] += d;
  h[4] += e;
  h[5] += f;
  h[6] += g;
  h[7] += hh;
}

/* FIPS 180-4 §5.1.1 padding + §6.2: digest of msg[0..len) into out[32]. */
void rso_sha256(const uint8_t *msg, size_t len, uint8_t out[32]) {
  uint32_t h[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  size_t i = 0;
  for (; i + 64 <= len; i += 64) compress(h, msg + i);
  uint8_t tail[128];
  memset(tail, 0, sizeof(tail));
  const size_t rem = len - i;
  memcpy(tail, msg + i, rem);
  tail[rem] = 0x80;
  const size_t tlen = rem + 9 <= 64 ? 64 : 128;
  const uint64_t bits = (uint64_t)len * 8u;
  for (int q = 0; q < 8; ++q) tail[tlen - 1 - q] = (uint8_t)(bits >> (8 * q));
  compress(h, tail);
  if (tlen == 128) compress(h, tail + 64);
  for (int q = 0; q < 8; ++q) {
    out[4 * q] = (uint8_t)(h[q] >> 24);
    out[4 * q + 1] = (uint8_t)(h[q] >> 16);
    out[4 * q + 2] = (uint8_t)(h[q] >> 8);
    out[4 * q + 3] = (uint8_t)h[q];
  }
}

/* n messages at base + i*stride, lens[i] bytes each (lens == NULL: all `len`). */
void rso_sha256_batch(const uint8_t *base, size_t stride, const uint64_t *lens, size_t len, size_t n,
                      uint8_t *out) {
  for (size_t i = 0; i < n; ++i) rso_sha256(base + i * stride, lens ? (size_t)lens[i] : len, out + 32 * i);
}
