/* sha256_cpu_baseline.c -- TEST / BENCH INFRASTRUCTURE ONLY: the CPU baseline for
 * the GPU batched SHA-256 (bench.py's sha256 extra).  The reference hashes each
 * value with Go's crypto/sha256 (writeservice.go:51-54), whose amd64 code uses the
 * SHA extensions when present; this restates that class of code: x86 SHA-NI
 * (sha256rnds2 / sha256msg1 / sha256msg2) on one message per task, all host
 * threads, scalar FIPS 180-4 (sha256_oracle.c) when the CPU lacks SHA-NI.
 */
#include <immintrin.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdlib.h>
#include <string.h>

#include "rs_oracle.h"

static const uint32_t K[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

/* SHA-NI keeps the state as two vectors: abef = {a,b,e,f}, cdgh = {c,d,g,h}
 * (highest lane first).  Four rounds per step: two sha256rnds2, each consuming
 * two words of W+K. */
__attribute__((target("sha,sse4.1"))) static void compress_ni(__m128i *abef, __m128i *cdgh, const uint8_t *blk) {
  const __m128i bswap = _mm_set_epi64x(0x0c0d0e0f08090a0bULL, 0x0405060700010203ULL);
  __m128i w[4];
  for (int q = 0; q < 4; ++q) w[q] = _mm_shuffle_epi8(_mm_loadu_si128((const __m128i *)(blk + 16 * q)), bswap);
  const __m128i s0 = *abef, s1 = *cdgh;
  __m128i a = *abef, c = *cdgh;
  for (int r = 0; r < 16; ++r) {  /* rounds 4r .. 4r+3 */
    __m128i *cur = &w[r & 3];
    if (r >= 4) {
      /* W[4r..4r+3] from the previous 16 words: msg1 folds in sigma0, the
       * alignr adds W[t-7], msg2 adds sigma1 */
      __m128i t = _mm_sha256msg1_epu32(*cur, w[(r + 1) & 3]);
      t = _mm_add_epi32(t, _mm_alignr_epi8(w[(r + 3) & 3], w[(r + 2) & 3], 4));
      *cur = _mm_sha256msg2_epu32(t, w[(r + 3) & 3]);
    }
    __m128i wk = _mm_add_epi32(*cur, _mm_loadu_si128((const __m128i *)(K + 4 * r)));
    c = _mm_sha256rnds2_epu32(c, a, wk);
    wk = _mm_shuffle_epi32(wk, 0x0E);
    a = _mm_sha256rnds2_epu32(a, c, wk);
  }
  *abef = _mm_add_epi32(a, s0);
  *cdgh = _mm_add_epi32(c, s1);
}

__attribute__((target("sha,sse4.1"))) static void sha256_ni(const uint8_t *msg, size_t len, uint8_t out[32]) {
  /* initial state H0..H7 packed as abef / cdgh */
  __m128i abef = _mm_set_epi32(0x6a09e667, 0xbb67ae85, 0x510e527f, 0x9b05688c);
  __m128i cdgh = _mm_set_epi32(0x3c6ef372, 0xa54ff53a, 0x1f83d9ab, 0x5be0cd19);
  size_t i = 0;
  for (; i + 64 <= len; i += 64) compress_ni(&abef, &cdgh, msg + i);
  uint8_t tail[128];
  memset(tail, 0, sizeof(tail));
  const size_t rem = len - i;
  memcpy(tail, msg + i, rem);
  tail[rem] = 0x80;
  const size_t tlen = rem + 9 <= 64 ? 64 : 128;
  const uint64_t bits = (uint64_t)len * 8u;
  for (int q = 0; q < 8; ++q) tail[tlen - 1 - q] = (uint8_t)(bits >> (8 * q));
  compress_ni(&abef, &cdgh, tail);
  if (tlen == 128) compress_ni(&abef, &cdgh, tail + 64);
  uint32_t h[8], v[4];
  _mm_storeu_si128((__m128i *)v, abef); /* v = {f, e, b, a} */
  h[0] = v[3]; h[1] = v[2]; h[4] = v[1]; h[5] = v[0];
  _mm_storeu_si128((__m128i *)v, cdgh); /* v = {h, g, d, c} */
  h[2] = v[3]; h[3] = v[2]; h[6] = v[1]; h[7] = v[0];
  for (int q = 0; q < 8; ++q) {
    out[4 * q] = (uint8_t)(h[q] >> 24);
    out[4 * q + 1] = (uint8_t)(h[q] >> 16);
    out[4 * q + 2] = (uint8_t)(h[q] >> 8);
    out[4 * q + 3] = (uint8_t)h[q];
  }
}

typedef struct {
  const uint8_t *base;
  size_t stride, len, n;
  uint8_t *out;
  int ni;
  atomic_size_t next;
} job_t;

static void *worker(void *p) {
  job_t *j = (job_t *)p;
  for (;;) {
    const size_t i0 = atomic_fetch_add(&j->next, 64);
    if (i0 >= j->n) break;
    const size_t i1 = i0 + 64 < j->n ? i0 + 64 : j->n;
    for (size_t i = i0; i < i1; ++i) {
      if (j->ni)
        sha256_ni(j->base + i * j->stride, j->len, j->out + 32 * i);
      else
        rso_sha256(j->base + i * j->stride, j->len, j->out + 32 * i);
    }
  }
  return NULL;
}

/* n messages of len bytes at base + i*stride on `threads` threads; returns 1 if
 * SHA-NI ran, 0 for the scalar path.  RSO_BASELINE_LEVEL=0 forces scalar. */
int rso_baseline_sha256_batch(const uint8_t *base, size_t stride, size_t len, size_t n, uint8_t *out,
                              int threads) {
  __builtin_cpu_init();
  int ni = __builtin_cpu_supports("sha") && __builtin_cpu_supports("sse4.1");
  const char *lvl = getenv("RSO_BASELINE_LEVEL");
  if (lvl && atoi(lvl) == 0) ni = 0;
  job_t j = {base, stride, len, n, out, ni, 0};
  if (threads < 1) threads = 1;
  pthread_t *tid = (pthread_t *)malloc(sizeof(pthread_t) * (size_t)threads);
  for (int t = 1; t < threads; t++) pthread_create(&tid[t], NULL, worker, &j);
  worker(&j);
  for (int t = 1; t < threads; t++) pthread_join(tid[t], NULL);
  free(tid);
  return ni;
}
