/*
 * rs_cpu_baseline.c -- the CPU baseline leg of bench.py (a "port": a C restatement
 * of the reference's CPU codec, NOT klauspost itself, which is Go and absent here).
 *
 * TEST/BENCH INFRASTRUCTURE ONLY (see rs_oracle.h): loaded by bench.py's
 * cpu_baseline leg and by tests/ which check it against the scalar oracle.
 *
 * Algorithm class follows the reference's native kernels [upstream
 * klauspost/reedsolomon v1.12.1 galois_amd64.go / galois_gen_amd64.s]:
 *   - AVX-512 + GFNI: one VGF2P8AFFINEQB per (input, output) coefficient with an
 *     8x8 bit-matrix per coefficient (the library's mulGFNI_KxM_64 family);
 *   - AVX2: split-nibble VPSHUFB with 16-entry low/high product tables
 *     (mulAvxTwo_KxM family);
 *   - scalar table lookup otherwise.
 * Loop order as upstream codeSomeShards: per 64-byte column load the K inputs once
 * and produce every output.  Concurrency as the reference deploys it: one stripe
 * (object) per call, single goroutine per call (ec.go:26 WithAutoGoroutines(NumCPU)
 * yields maxGoroutines=1), many concurrent callers -> here a pool of
 * `threads` workers pulling stripes from a shared counter.
 */
#include "rs_oracle.h"

#include <immintrin.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdlib.h>
#include <string.h>

#define MAXK 32
#define MAXE 32

typedef struct {
    int k, e;
    const int *in_idx, *out_idx;
    uint8_t *base;
    size_t stripe_pitch, shard_pitch, S, N;
    uint8_t mul[MAXE * MAXK][256];             /* scalar tables */
    uint8_t lo[MAXE * MAXK][16], hi[MAXE * MAXK][16]; /* split-nibble tables */
    uint64_t gfni[MAXE * MAXK];                /* affine bit-matrices */
    int level;
    atomic_size_t next;
} job_t;

/* One stripe: in[c] / out[r] are its k input and e output shards, S bytes each. */
static void stripe_scalar(const job_t *j, const uint8_t *const *in, uint8_t *const *out, size_t S) {
    for (int r = 0; r < j->e; r++) {
        uint8_t *o = out[r];
        for (size_t b = 0; b < S; b++) {
            uint8_t acc = 0;
            for (int c = 0; c < j->k; c++) acc ^= j->mul[r * j->k + c][in[c][b]];
            o[b] = acc;
        }
    }
}

__attribute__((target("avx2"))) static void stripe_avx2(const job_t *j, const uint8_t *const *in,
                                                       uint8_t *const *out, size_t S) {
    const size_t full = S & ~(size_t)31;
    const __m256i mask = _mm256_set1_epi8(0x0f);
    __m256i acc[MAXE];
    for (size_t b = 0; b < full; b += 32) {
        for (int r = 0; r < j->e; r++) acc[r] = _mm256_setzero_si256();
        for (int c = 0; c < j->k; c++) {
            __m256i x = _mm256_loadu_si256((const __m256i *)(in[c] + b));
            __m256i xl = _mm256_and_si256(x, mask);
            __m256i xh = _mm256_and_si256(_mm256_srli_epi64(x, 4), mask);
            for (int r = 0; r < j->e; r++) {
                const int q = r * j->k + c;
                __m256i tl = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i *)j->lo[q]));
                __m256i th = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i *)j->hi[q]));
                acc[r] = _mm256_xor_si256(acc[r], _mm256_xor_si256(_mm256_shuffle_epi8(tl, xl),
                                                                    _mm256_shuffle_epi8(th, xh)));
            }
        }
        for (int r = 0; r < j->e; r++)
            _mm256_storeu_si256((__m256i *)(out[r] + b), acc[r]);
    }
    for (size_t b = full; b < S; b++)
        for (int r = 0; r < j->e; r++) {
            uint8_t a = 0;
            for (int c = 0; c < j->k; c++)
                a ^= j->mul[r * j->k + c][in[c][b]];
            out[r][b] = a;
        }
}

__attribute__((target("avx512f,avx512bw,gfni"))) static void stripe_gfni(const job_t *j, const uint8_t *const *in,
                                                                       uint8_t *const *out, size_t S) {
    const size_t full = S & ~(size_t)63;
    __m512i acc[MAXE];
    for (size_t b = 0; b < full; b += 64) {
        for (int r = 0; r < j->e; r++) acc[r] = _mm512_setzero_si512();
        for (int c = 0; c < j->k; c++) {
            __m512i x = _mm512_loadu_si512((const void *)(in[c] + b));
            for (int r = 0; r < j->e; r++) {
                __m512i a = _mm512_set1_epi64((long long)j->gfni[r * j->k + c]);
                acc[r] = _mm512_xor_si512(acc[r], _mm512_gf2p8affine_epi64_epi8(x, a, 0));
            }
        }
        for (int r = 0; r < j->e; r++)
            _mm512_storeu_si512((void *)(out[r] + b), acc[r]);
    }
    for (size_t b = full; b < S; b++)
        for (int r = 0; r < j->e; r++) {
            uint8_t a = 0;
            for (int c = 0; c < j->k; c++)
                a ^= j->mul[r * j->k + c][in[c][b]];
            out[r][b] = a;
        }
}

static void stripe_apply(const job_t *j, const uint8_t *const *in, uint8_t *const *out, size_t S) {
    if (j->level == 3) stripe_gfni(j, in, out, S);
    else if (j->level == 2) stripe_avx2(j, in, out, S);
    else stripe_scalar(j, in, out, S);
}

static void *worker(void *arg) {
    job_t *j = (job_t *)arg;
    for (;;) {
        size_t i = atomic_fetch_add(&j->next, 16);
        if (i >= j->N) break;
        size_t end = i + 16 < j->N ? i + 16 : j->N;
        for (; i < end; i++) {
            uint8_t *st = j->base + i * j->stripe_pitch;
            const uint8_t *in[MAXK];
            uint8_t *out[MAXE];
            for (int c = 0; c < j->k; c++) in[c] = st + (size_t)j->in_idx[c] * j->shard_pitch;
            for (int r = 0; r < j->e; r++) out[r] = st + (size_t)j->out_idx[r] * j->shard_pitch;
            stripe_apply(j, in, out, j->S);
        }
    }
    return NULL;
}

/* Tables for an e x k coefficient matrix (scalar, split-nibble, GFNI affine). */
static job_t *job_new(int k, int e, const uint8_t *rows) {
    if (k > MAXK || e > MAXE || k <= 0 || e < 0) return NULL;
    job_t *j = (job_t *)aligned_alloc(64, (sizeof(job_t) + 63) & ~(size_t)63);
    memset(j, 0, sizeof(*j));
    j->k = k; j->e = e;
    for (int q = 0; q < e * k; q++) {
        uint8_t f = rows[q];
        for (int v = 0; v < 256; v++) j->mul[q][v] = rso_gf_mul(f, (uint8_t)v);
        for (int v = 0; v < 16; v++) {
            j->lo[q][v] = rso_gf_mul(f, (uint8_t)v);
            j->hi[q][v] = rso_gf_mul(f, (uint8_t)(v << 4));
        }
        /* affine matrix: result bit i = parity(A.byte[7-i] & x); bit j of that
         * byte = bit i of f*2^j */
        uint64_t a = 0;
        for (int bi = 0; bi < 8; bi++) {
            uint8_t row = 0;
            for (int bj = 0; bj < 8; bj++)
                row |= (uint8_t)(((rso_gf_mul(f, (uint8_t)(1u << bj)) >> bi) & 1u) << bj);
            a |= (uint64_t)row << (8 * (7 - bi));
        }
        j->gfni[q] = a;
    }
    __builtin_cpu_init();
    if (__builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512bw") &&
        __builtin_cpu_supports("gfni"))
        j->level = 3;
    else if (__builtin_cpu_supports("avx2"))
        j->level = 2;
    else
        j->level = 0;
    {
        const char *force = getenv("RSO_BASELINE_LEVEL");
        if (force) {
            int f = atoi(force);
            if (f < j->level) j->level = f == 1 ? 0 : f;
        }
    }
    return j;
}

int rso_baseline_apply_batch(int k, int e, const uint8_t *rows, const int *in_idx,
                             const int *out_idx, uint8_t *base, size_t stripe_pitch,
                             size_t shard_pitch, size_t S, size_t N, int threads) {
    job_t *j = job_new(k, e, rows);
    if (!j) return -1;
    j->in_idx = in_idx; j->out_idx = out_idx; j->base = base;
    j->stripe_pitch = stripe_pitch; j->shard_pitch = shard_pitch; j->S = S; j->N = N;
    atomic_init(&j->next, 0);
    if (threads < 1) threads = 1;
    pthread_t *tid = (pthread_t *)malloc(sizeof(pthread_t) * (size_t)threads);
    for (int t = 1; t < threads; t++) pthread_create(&tid[t], NULL, worker, j);
    worker(j);
    for (int t = 1; t < threads; t++) pthread_join(tid[t], NULL);
    free(tid);
    int level = j->level;
    free(j);
    return level;
}

void *rso_baseline_plan_new(int k, int e, const uint8_t *rows) { return job_new(k, e, rows); }

void rso_baseline_plan_free(void *plan) { free(plan); }

int rso_baseline_plan_apply(const void *plan, const uint8_t *const *in, uint8_t *const *out, size_t S) {
    const job_t *j = (const job_t *)plan;
    if (!j) return -1;
    stripe_apply(j, in, out, S);
    return j->level;
}
