/*
 * rsgpu.h -- C-ABI of the MI355X Reed-Solomon engine (librsgpu.so).
 *
 * Drop-in boundary for the reference's codec package internal/ec
 * (internal/ec/ec.go:15-61) behind interfaces.IEcDriver
 * (internal/interfaces/interfaces.go:41-52).  A cgo shim keeps the
 * Go surface NewService / Split / Encode / Reconstruct and calls these entry points;
 * the codec arithmetic that klauspost/reedsolomon v1.12.1 did on the CPU
 * (go.mod:16) runs in hand-written gfx950 HIP kernels.
 *
 * Conventions
 *  - Plain C types only: pointers, sizes, ints.  No torch / HIP types in signatures
 *    (streams are passed as void* = hipStream_t, NULL = the HIP null stream).
 *  - Return value: RS_OK (0) or an RS_ERR_* code; rs_strerror() gives the message.
 *    Codes 1..7 carry klauspost's sentinel messages (errors.go) so that a Go shim
 *    can return errors whose %v text matches the reference's.
 *  - Thread safety: every function may be called concurrently on one context
 *    (the reference shares one IEcDriver across all request goroutines and the
 *    healer's workers: cmd/api/main.go:206, cmd/healer/main.go:42, poller.go:49).
 *  - Devices: a context spans one GPU (rs_create) or several (rs_create_multi,
 *    rs_create_devices).  Calls never change the calling thread's current HIP
 *    device.  Per-object calls and host-memory batches are spread over the
 *    context's GPUs by the library; a device-memory batch runs on the GPU its
 *    `stream` belongs to (the calling thread's current device for the NULL
 *    stream), which the context must span.
 *  - No CPU fallback in the library: creation fails with RS_ERR_NO_DEVICE when no
 *    gfx950 GPU is visible and the library never computes parity on the host.  The
 *    Go shim then falls back to klauspost itself.
 */
#ifndef RSGPU_H
#define RSGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- error codes ------------------------------------------------------- */
#define RS_OK 0
#define RS_ERR_INV_SHARD_NUM 1  /* klauspost ErrInvShardNum  */
#define RS_ERR_MAX_SHARD_NUM 2  /* klauspost ErrMaxShardNum  */
#define RS_ERR_TOO_FEW_SHARDS 3 /* klauspost ErrTooFewShards "too few shards given" */
#define RS_ERR_SHARD_NO_DATA 4  /* klauspost ErrShardNoData "no shard data" */
#define RS_ERR_SHARD_SIZE 5     /* klauspost ErrShardSize "shard sizes do not match" */
#define RS_ERR_SHORT_DATA 6     /* klauspost ErrShortData */
#define RS_ERR_SINGULAR 7       /* klauspost errSingular "matrix is singular" */
#define RS_ERR_INVALID_ARG 16   /* pointer / layout contract violated */
#define RS_ERR_NO_DEVICE 17     /* no usable GPU */
#define RS_ERR_DEVICE 18        /* HIP runtime failure */
#define RS_ERR_NOT_SUPPORTED 19 /* klauspost ErrNotSupported "operation not supported" */
#define RS_ERR_BUSY 20          /* coalescer: no staging batch free (all executing or awaiting rs_co_reap) */

/* memory kinds for the batched entry points */
#define RS_MEM_DEVICE 0 /* pointers are device memory; call is asynchronous on `stream` */
#define RS_MEM_HOST 1   /* pointers are host memory (pinned or pageable); synchronous */

typedef struct rs_ctx rs_ctx;

/* ---- lifecycle ---------------------------------------------------------
 * Replaces reedsolomon.New(config.K, config.M, WithAutoGoroutines(NumCPU))
 * at internal/ec/ec.go:26.  k >= 1, m >= 0, k+m <= 256 (klauspost limits, checked
 * first, same order and sentinels); the GPU engine additionally needs k <= 32,
 * m <= 16, k+m <= 32 (RS_ERR_NOT_SUPPORTED).
 *   rs_create:         one GPU, HIP ordinal `device`.
 *   rs_create_multi:   the GPUs whose bit is set in device_mask (bit d = ordinal
 *                      d); 0 = every visible gfx950 GPU.  SURVEY.md §8b's
 *                      rs_create(k, m, device_mask, flags): what the Go shim's
 *                      NewService calls, so one IEcDriver drives the whole node.
 *   rs_create_devices: an explicit list of n_devices ordinals; an ordinal may
 *                      repeat (several engines, each with its own streams and
 *                      staging, on one GPU).
 * RS_ERR_NO_DEVICE: no GPU visible, or a named ordinal missing / not gfx950.
 */
int rs_create(int k, int m, int device, int flags, rs_ctx **out);
int rs_create_multi(int k, int m, uint64_t device_mask, int flags, rs_ctx **out);
int rs_create_devices(int k, int m, const int *devices, int n_devices, int flags, rs_ctx **out);
void rs_destroy(rs_ctx *ctx);
int rs_data_shards(const rs_ctx *ctx);
int rs_parity_shards(const rs_ctx *ctx);
int rs_device(const rs_ctx *ctx);               /* the first engine's ordinal */
int rs_device_count(const rs_ctx *ctx);         /* engines in the context */
int rs_device_at(const rs_ctx *ctx, int i);     /* ordinal of engine i (-1 if none) */
/* Codec kernels (encode / reconstruct / verify) this context has launched on engine
 * i since creation: which GPUs of a multi-GPU context a host batch or a coalesced
 * burst actually used (bench.py's multi_ctx leg). */
int rs_device_launches(const rs_ctx *ctx, int i, uint64_t *launches);
/* Description of the backend for NewService's log line (ec.go:32-41). */
const char *rs_backend(const rs_ctx *ctx);
const char *rs_strerror(int code);
/* Copy the (k+m) x k encode matrix (row-major) into out. */
int rs_encode_matrix(const rs_ctx *ctx, uint8_t *out);

/* ---- per-object API, host memory (IEcDriver drop-in) --------------------
 * Split  (ec.go:48-50): host-only, no arithmetic -> the shim keeps it in Go; this
 *         gives perShard = ceil(len/k) (0 if len == 0 -> ErrShortData).
 * Encode (ec.go:54-56): shards[k+m], lens[k+m]; all lens equal and nonzero, else
 *         RS_ERR_SHARD_SIZE / RS_ERR_SHARD_NO_DATA.  Parity written in place.
 * Reconstruct (ec.go:59-61): lens[i] == 0 marks a missing shard (Go: len==0); the
 *         caller supplies writable storage of >= S bytes for each missing shard in
 *         shards[i].  Every missing shard (data AND parity) is filled and its
 *         lens[i] set to S.  Fewer than k present -> RS_ERR_TOO_FEW_SHARDS.
 * Verify: *ok = 1 iff the parity shards match the data shards.
 */
size_t rs_shard_size(const rs_ctx *ctx, size_t data_len);
int rs_encode(rs_ctx *ctx, uint8_t *const *shards, const size_t *lens);
int rs_reconstruct(rs_ctx *ctx, uint8_t *const *shards, size_t *lens);
int rs_reconstruct_data(rs_ctx *ctx, uint8_t *const *shards, size_t *lens);
int rs_verify(rs_ctx *ctx, uint8_t *const *shards, const size_t *lens, int *ok);

/* ---- batched API: the throughput path -----------------------------------
 * A batch holds n_stripes independent stripes (objects) in a SPLIT layout (the
 * reference's shard order: shards[0..k) data, shards[k..k+m) parity):
 *   data shard s  (s < k)  of stripe i:  data   + i*data_stripe_pitch   + s*shard_pitch
 *   parity shard p (p < m) of stripe i:  parity + i*parity_stripe_pitch + p*shard_pitch
 * each shard_len (S) bytes.  A unified K+M-slot layout is the special case
 * parity = data + k*shard_pitch with equal stripe pitches.
 *
 * RS_MEM_DEVICE: pitches must be multiples of 16 and shard_pitch >= round_up(S, 16),
 *   bases 16-B aligned (the kernels read whole 16-B columns; bytes of a slot past S
 *   may be read, never written).  The call enqueues on `stream` and returns;
 *   synchronise with hipStreamSynchronize or rs_sync.  S up to 0xFFFFFFF0.
 * RS_MEM_HOST: any pitches; shards in memory the context allocated (rs_host_alloc)
 *   are read and written in place by the kernels (zero-copy), all others --
 *   pageable, rs_host_register'ed, or pinned by another allocator -- are staged
 *   through device slabs with H2D / kernel / D2H overlapped on several streams.
 *   Returns when the outputs are in host memory.  A multi-GPU context splits the
 *   batch into contiguous stripe ranges, one per GPU, run in parallel.
 *
 * rs_encode_batch: reads data shards, writes every parity shard.
 * rs_reconstruct_batch: in place.  present_masks: host array of n_masks uint32
 *   (bit s set = shard s present); n_masks == 1 applies one pattern to every
 *   stripe, n_masks == n_stripes gives a pattern per stripe (k+m <= 16).  Every
 *   missing shard (data and parity) is written.  Any mask with < k present ->
 *   RS_ERR_TOO_FEW_SHARDS and nothing is modified.
 */
int rs_encode_batch(rs_ctx *ctx, const uint8_t *data, size_t data_stripe_pitch, uint8_t *parity,
                    size_t parity_stripe_pitch, size_t shard_pitch, size_t shard_len,
                    size_t n_stripes, int mem, void *stream);
int rs_reconstruct_batch(rs_ctx *ctx, uint8_t *data, size_t data_stripe_pitch, uint8_t *parity,
                         size_t parity_stripe_pitch, size_t shard_pitch, size_t shard_len,
                         size_t n_stripes, const uint32_t *present_masks, size_t n_masks, int mem,
                         void *stream);
/* Device-resident masks (RS_MEM_DEVICE only, k+m <= 16): present_masks_dev is a
 * device array of n_stripes uint32.  Stripes with < k present are left untouched
 * and reported by the next rs_sync on THAT stream as RS_ERR_TOO_FEW_SHARDS (each
 * stream has its own deferred-error word, however many streams there are; rs_sync
 * on another stream neither sees nor clears it). */
int rs_reconstruct_batch_devmask(rs_ctx *ctx, uint8_t *data, size_t data_stripe_pitch,
                                 uint8_t *parity, size_t parity_stripe_pitch, size_t shard_pitch,
                                 size_t shard_len, size_t n_stripes,
                                 const uint32_t *present_masks_dev, void *stream);
/* Out-of-place reconstruct (RS_MEM_DEVICE only): the shard buffers are read-only;
 * the r-th missing shard of stripe i (missing shards in index order, data before
 * parity) is written to  out + i*out_stripe_pitch + r*shard_pitch.  This is the
 * reference's own semantics (Reconstruct gives missing entries NEW slices) and the
 * healer's (it writes back only the missing shards), and it streams faster: writes
 * that land in the region being read cost ~20 % of HBM throughput on MI355X
 * (profiles/r01_hbm_probe3.log).  present_masks is a host array of n_masks (1 or
 * n_stripes) uint32, or with masks_on_device != 0 a device array of n_stripes
 * (k+m <= 16; errors deferred to rs_sync).  out_stripe_pitch >= (#missing,
 * at most m) * shard_pitch, multiple of 16. */
int rs_reconstruct_batch_out(rs_ctx *ctx, const uint8_t *data, size_t data_stripe_pitch,
                             const uint8_t *parity, size_t parity_stripe_pitch, size_t shard_pitch,
                             size_t shard_len, size_t n_stripes, const uint32_t *present_masks,
                             size_t n_masks, int masks_on_device, uint8_t *out,
                             size_t out_stripe_pitch, void *stream);
/* The same with device masks and a caller-known bound on the erasures per stripe:
 * 1 <= max_missing <= m (0 = m).  Host masks give the engine their maximum; device
 * masks cannot, and a kernel sized for m outputs per stripe carries registers and
 * work a batch of 1-2 erasure repairs never uses (the healer's case, poller.go:282;
 * a degraded read, readservice.go:285).  out_stripe_pitch >= max_missing *
 * shard_pitch.  A stripe missing more than max_missing shards is left untouched
 * and reported by rs_sync on the stream as RS_ERR_INVALID_ARG (one with < k present
 * as RS_ERR_TOO_FEW_SHARDS, which takes precedence). */
int rs_reconstruct_batch_out_devmask(rs_ctx *ctx, const uint8_t *data, size_t data_stripe_pitch,
                                     const uint8_t *parity, size_t parity_stripe_pitch,
                                     size_t shard_pitch, size_t shard_len, size_t n_stripes,
                                     const uint32_t *present_masks_dev, int max_missing, uint8_t *out,
                                     size_t out_stripe_pitch, void *stream);
/* Packed out-of-place reconstruct (RS_MEM_DEVICE only, k+m <= 16), for scans whose
 * stripes miss 0..m shards each (the healer's audit of a batch of objects,
 * poller.go:227-309): the missing shards of the whole batch are written back to
 * back, stripe i's r-th missing shard (index order, data before parity) at
 *   out + (row_offsets[i] + r) * shard_pitch,
 * where row_offsets (a device array of n_stripes + 1 uint32 the call fills) is the
 * exclusive prefix sum of the stripes' erasure counts and row_offsets[n_stripes] the
 * batch's total -- so out needs total * shard_pitch bytes, not n_stripes * m rows
 * (intact stripes take none, a stripe with < k present none either: at most
 * n_stripes * m rows).  present_masks: host (n_stripes) or, with masks_on_device != 0,
 * device (errors deferred to rs_sync: a stripe with < k present is reported and
 * skipped).  Whole-line rows follow rs_set_out_pad_writes (each row
 * owns one shard_pitch).  Streams faster than the m-row slots of
 * rs_reconstruct_batch_out on scans. */
int rs_reconstruct_batch_out_packed(rs_ctx *ctx, const uint8_t *data, size_t data_stripe_pitch,
                                    const uint8_t *parity, size_t parity_stripe_pitch, size_t shard_pitch,
                                    size_t shard_len, size_t n_stripes, const uint32_t *present_masks,
                                    int masks_on_device, uint8_t *out, uint32_t *row_offsets, void *stream);
/* Batched parity verify / bit-rot scrub ([upstream reedsolomon.go Verify], per
 * object: rs_verify).  Recomputes every parity shard from the data shards and
 * compares it with the stored one: bad[i] = bitmask of stripe i's parity shards
 * that differ (bit r = parity shard r; 0 = stripe intact).  bad has n_stripes
 * uint32 in the memory kind `mem` (device: written asynchronously on `stream`;
 * host: synchronous).  Nothing else is written.  Reads K+M shards per stripe. */
int rs_verify_batch(rs_ctx *ctx, const uint8_t *data, size_t data_stripe_pitch,
                    const uint8_t *parity, size_t parity_stripe_pitch, size_t shard_pitch,
                    size_t shard_len, size_t n_stripes, uint32_t *bad, int mem, void *stream);
/* Wait for `stream` and return (and clear) its deferred device-side errors. */
int rs_sync(rs_ctx *ctx, void *stream);
/* rs_sync, then forget the stream: its deferred-error word goes back to the engine.
 * Call it before destroying a stream that ran device-mask batches, so a later stream
 * that gets the same handle starts with no errors and no word is kept for it. */
int rs_stream_release(rs_ctx *ctx, void *stream);

/* ---- batch coalescer (per-object calls -> device batches) ------------------
 * Drop-in for the per-object entry points when many threads call them at once
 * (one goroutine per request: writeservice.go:218-222, readservice.go:144,285,
 * poller.go:282).  rs_co_* take exactly the arguments, perform the same checks
 * and return the same codes as rs_encode / rs_reconstruct / rs_reconstruct_data /
 * rs_verify, and are synchronous: on return the outputs are in the caller's
 * buffers and nothing of the caller's is retained.  Concurrent calls with the
 * same shard length are staged into one batch and run as one device launch (a
 * batch closes when max_batch slots are taken or max_wait_us after its first
 * call).  Every call kind coalesces: with k+m <= 16 a staged object carries its
 * present mask (resolved by the kernel through the all-pattern LUT), with k+m > 16
 * the address of its plan from the engine's plan cache.  Thread-safe; the context
 * must outlive the coalescer.
 * Batching is group commit: a batch starts as soon as fewer than max_exec batches
 * are on the device (after an optional max_wait_us linger); calls arriving
 * meanwhile join the open batch, so batch size follows the load and a lone caller
 * waits for no timer. */
typedef struct rs_coalescer rs_coalescer;
typedef struct {
  size_t max_batch;       /* stripes per batch (0 = 4096) */
  uint32_t max_wait_us;   /* linger before a batch may start (0 = none) */
  int inflight;           /* staging batches (0 = 16); each: stream + pinned + device slab */
  size_t max_batch_bytes; /* staging bytes per batch (0 = 32 MiB) */
  int max_exec;           /* batches executing at once (0 = 2; <= inflight) */
  int staged_dma;         /* 0: kernels read/write the pinned staging in place (zero-copy);
                             1: H2D / D2H copies around the kernel */
  int spin_waiters;       /* callers that may spin-wait for their batch at once instead of
                             sleeping on a futex: 0 = none (default), > 0 = that many, capped
                             at the CPUs this process may use minus the coalescer's threads */
  int plain_copy;         /* 0 (default): shard-sized staging copies use streaming stores;
                             1: plain memcpy (A/B measurements) */
} rs_coalescer_opts;
int rs_coalescer_create(rs_ctx *ctx, const rs_coalescer_opts *opts /* NULL = defaults */,
                        rs_coalescer **out);
void rs_coalescer_destroy(rs_coalescer *co);
int rs_co_encode(rs_coalescer *co, uint8_t *const *shards, const size_t *lens);
int rs_co_reconstruct(rs_coalescer *co, uint8_t *const *shards, size_t *lens);
int rs_co_reconstruct_data(rs_coalescer *co, uint8_t *const *shards, size_t *lens);
int rs_co_verify(rs_coalescer *co, uint8_t *const *shards, const size_t *lens, int *ok);
/* Many objects in one call (batched healer repair; bulk
 * writes): object i's K+M shard pointers / lengths are shards[i*(k+m) ...] /
 * lens[i*(k+m) ...]; each object gets exactly rs_reconstruct's (rs_encode's)
 * contract and its return code in rcs[i].  Objects are grouped by shard length
 * and staged into as few device batches as possible.  Returns RS_OK unless the
 * call itself fails (bad arguments, device error). */
int rs_co_reconstruct_many(rs_coalescer *co, size_t n_objects, uint8_t *const *shards, size_t *lens,
                           int *rcs);
int rs_co_encode_many(rs_coalescer *co, size_t n_objects, uint8_t *const *shards,
                      const size_t *lens, int *rcs);
/* Encode + cold_hash in one coalesced batch: the write path
 * hashes the very value it splits and encodes -- Split writeservice.go:218, Encode
 * :222, cold_hash = computeSHA256Hex(value) :267 (:51-54); hybrid writes :326,
 * :382-386.  rs_co_encode's contract, and digest (32 bytes, FIPS 180-4 order) =
 * SHA-256 of the first value_len bytes of data shards 0..k-1 taken in order -- the
 * Split input, since Split's data shards are the value followed by zero padding.
 * 0 <= value_len <= k * S (RS_ERR_INVALID_ARG otherwise).  The hash runs on the GPU
 * in the same batch, one lane per object: SHA-256 is a serial chain, and one lane
 * hashes ~30-40 MB/s where a SHA-NI CPU core does ~2 GB/s, so this pays only with
 * thousands of values per launch (rs_co_encode_hash_many on a bulk load,
 * rs_sha256_batch).  Per-object writers should hash on the CPU while rs_co_encode
 * runs, as the Go shim's EncodeHash does: measured per object, this call moves
 * 0.5 GiB/s against 4-40 GiB/s for rs_co_encode (`HISTORY.md` §A.4). */
int rs_co_encode_hash(rs_coalescer *co, uint8_t *const *shards, const size_t *lens, size_t value_len,
                      uint8_t *digest);
int rs_co_encode_hash_many(rs_coalescer *co, size_t n_objects, uint8_t *const *shards, const size_t *lens,
                           const size_t *value_lens, uint8_t *digests, int *rcs);
/* Asynchronous per-object calls, for callers that multiplex many requests on few
 * threads (the Go runtime's goroutines on GOMAXPROCS threads, an event loop): a
 * blocking call costs its thread a futex sleep and wake-up per object, several
 * microseconds of CPU against ~1 us of codec work for a 4 KiB object on one core.
 * rs_co_submit_* validate and stage the object exactly as rs_co_encode /
 * rs_co_reconstruct do and return at once; the call completes when rs_co_reap
 * returns its tag, with its code: encode -> every parity shard written;
 * reconstruct -> every missing (len 0) shard filled with S bytes (lens is not
 * written).  Until then the caller keeps every shard buffer valid and untouched
 * (the arrays of pointers and lengths may be reused at once).  A call rejected at
 * submit returns its code and is never reaped; RS_ERR_BUSY: no staging batch is
 * free -- each is executing on a GPU or holds finished calls not reaped yet; wait
 * until some reap has returned calls (a reaper can signal that), then submit again
 * (submit never blocks).  An object
 * with nothing to compute (a reconstruct with nothing missing, m == 0) is rejected
 * with RS_ERR_NOT_SUPPORTED.
 * rs_co_reap: up to max completed calls -> tags[i], rcs[i]; copies their outputs
 * into the callers' buffers on the reaping thread.  Waits up to timeout_us for at
 * least one (0: poll, < 0: until one completes); returns how many (a negative
 * code on bad arguments).  It returns 0 at once, or as soon as it wakes, once
 * rs_coalescer_destroy has begun; still, no thread may be inside rs_co_reap when
 * that call frees the coalescer, so stop reapers first (a finite timeout_us lets
 * them notice).  Any number of threads may submit and reap; each reaper copies the
 * outputs of the calls it returns, so several reapers share that work.  Reap every
 * submitted call before rs_coalescer_destroy. */
int rs_co_submit_encode(rs_coalescer *co, uint8_t *const *shards, const size_t *lens, uint64_t tag);
int rs_co_submit_reconstruct(rs_coalescer *co, uint8_t *const *shards, const size_t *lens, uint64_t tag);
int rs_co_reap(rs_coalescer *co, uint64_t *tags, int *rcs, int max, int timeout_us);
/* Counters since creation: calls, device batches, stripes batched, largest batch. */
int rs_co_stats(rs_coalescer *co, uint64_t *calls, uint64_t *batches, uint64_t *stripes,
                uint64_t *max_batch);
/* Launcher diagnostics since creation (any pointer may be NULL): time spent waiting
 * for callers still staging a closed batch, time in launch calls, time batches
 * executed, and how often a caller waited for a free batch. */
int rs_co_timing(rs_coalescer *co, uint64_t *straggle_ns, uint64_t *launch_ns, uint64_t *exec_ns,
                 uint64_t *free_waits);

/* ---- batched SHA-256 (cold_hash next to encode) -----
 * The reference hashes every EC-written value (writeservice.go:51-54
 * computeSHA256Hex, stored as "cold_hash" :267, compared :326-327).  Digest i
 * (32 bytes, FIPS 180-4 byte order) of message i goes to digests + 32*i.  Device
 * memory (or pinned host memory the GPU can address), asynchronous on `stream`;
 * digests 4-B aligned.
 *   rs_sha256_batch:     message i = base + i*stride, `len` bytes each
 *   rs_sha256_batch_var: message i = base + offsets[i], lens[i] bytes (device
 *                        arrays of n uint64) */
int rs_sha256_batch(rs_ctx *ctx, const uint8_t *base, size_t stride, size_t len, size_t n,
                    uint8_t *digests, void *stream);
int rs_sha256_batch_var(rs_ctx *ctx, const uint8_t *base, const uint64_t *offsets,
                        const uint64_t *lens, size_t n, uint8_t *digests, void *stream);

/* ---- host memory helpers ------------------------------------------------ */
/* In-place host memory: page-locked memory the context allocates itself
 * (hipHostMalloc, portable, on the first GPU's NUMA node when the runtime allows),
 * GPU-mapped, page aligned.  A coalesced call (rs_co_encode / rs_co_reconstruct,
 * their _submit_ and _many forms, and the _hash forms when the data shards holding
 * the value are contiguous -- shard c at shard 0 + c*S, as Split carves them; not
 * the _data form) whose shards -- the ones it reads and the ones it fills -- all lie
 * inside one rs_host_alloc'ed range, 16-B aligned, runs in place: the kernel reads
 * the caller's shards and writes the parity / missing shards straight into them
 * over PCIe, with no staging copy either way (the request
 * body and the HTTP send buffers, or a healer's shard buffers, in an arena).  Such a
 * call writes nothing outside [0, S) of any shard.  RS_MEM_HOST batches in such
 * memory run zero-copy.  rs_host_free only pointers rs_host_alloc returned, when no
 * call is using them; rs_destroy frees any left (after every queued kernel). */
int rs_host_alloc(rs_ctx *ctx, size_t bytes, void **out);
int rs_host_free(rs_ctx *ctx, void *ptr);
/* DEPRECATED -- a range recorder that never pins (the name is historical; do not
 * call it expecting faster transfers: registered and unregistered caller memory
 * take exactly the same staged path).
 * Records [ptr, ptr + bytes) as caller memory and nothing more: the library never
 * pins, maps or addresses caller memory in place (round 4).  amdgpu maps
 * hipHostRegister'ed pageable memory as a user-pointer range whose pages may still
 * be migrated, compacted or collapsed into huge pages while a kernel runs, which is
 * how in-place writes into it were lost (`HISTORY.md` §A.1).  Calls on registered
 * buffers are staged like any pageable buffer; use rs_host_alloc for in-place
 * work.  Kept for ABI compatibility: RS_ERR_INVALID_ARG for a range overlapping a
 * known one; rs_host_unregister(ptr) forgets the range starting at ptr
 * (RS_ERR_INVALID_ARG if there is none, or it is rs_host_free's).  A recorded range
 * that rs_host_alloc later gets memory inside (the caller freed it without
 * unregistering) is dropped, never an allocation failure. */
int rs_host_register(rs_ctx *ctx, void *ptr, size_t bytes);
int rs_host_unregister(rs_ctx *ctx, void *ptr);

/* ---- measurement helpers (bench.py) ------------------------------------- */
/* Name of the kernel the last batched call on this context launched (any thread). */
const char *rs_last_kernel(const rs_ctx *ctx);
/* Name of the last kernel this context launched on `stream` ("none" if none): the
 * launch that preceded a device error reported on that stream, whatever other
 * threads launched meanwhile. */
const char *rs_last_kernel_on(rs_ctx *ctx, void *stream);
/* Streaming device copy, the measured HBM ceiling beside the RS kernels. */
int rs_device_copy(rs_ctx *ctx, void *dst, const void *src, size_t bytes, void *stream);
/* Tuning knob: workgroups (256 threads) per CU for the batched kernels
 * (0 = the default, 2). */
int rs_set_blocks_per_cu(rs_ctx *ctx, int blocks_per_cu);
/* Tuning knob: at most waves_per_simd waves of a batched encode / reconstruct
 * launch per SIMD (a dynamic-LDS reservation admits that many 4-wave workgroups
 * per CU); -1 (default) = each kernel's measured default, 0 = uncapped.  For
 * measurement (tools/ab_bench.py, tools/ceiling_probe.sh); bytes never change. */
int rs_set_occupancy_cap(rs_ctx *ctx, int waves_per_simd);
/* Batched encode may write each parity slot's padding up to the next 128-B line
 * (bytes [S, min(pitch, round_up(S, 128))) of every parity slot; never past the
 * pitch) and reads the data slots' padding over the same range: every parity shard
 * write then ends on a whole 128-B line.  A partial last line costs HBM a
 * read-modify-write, and with the line-aligned shard length the flat-task
 * bitsliced encode covers the batch without partial columns (RS(10+4) at 64 KiB
 * objects: S = 6554 -> 6656, profiles/r02c_flat_encode.log).  The parity bytes
 * [0, S) are unchanged; the padding then holds the code of the data padding.
 * 0 (the default): no byte past S of any slot is ever written. */
int rs_set_parity_pad_writes(rs_ctx *ctx, int enable);
/* The same for the out-of-place reconstructs (rs_reconstruct_batch_out and its
 * _devmask form), opt-in: each output row written gets its padding up to the next
 * 128-B line, bytes [S, min(pitch, round_up(S, 128))) of the row at
 * out + i*out_sp + r*pitch -- never past the row's own slot: only when that line end
 * also fits the out stripe pitch (plane-major outputs with out_sp below it are
 * written exactly) -- and the inputs' padding is read over the same range.  Enable
 * it only when every output row owns its whole pitch (the last row of the buffer
 * included): a partial last line costs HBM a read-modify-write (RS(10+4) 64 KiB
 * 2-erasure 0.728 -> 0.756 of 8 TB/s, profiles/r04zj_sweep_trace.md).  Bytes [0, S)
 * are unchanged, rows a stripe does not miss are untouched.  0 (the default): no
 * byte past S of an output row is written, so an output buffer may end exactly at
 * the last row's byte S.  (Round 5 shipped this ON by default; round 6 restored the
 * exact-row default for C and Go callers.  The Python BatchEngine, whose outputs are
 * whole-pitch tensors, and the engine's own staging slabs turn it on.) */
int rs_set_out_pad_writes(rs_ctx *ctx, int enable);
/* RS_MEM_HOST batches whose shards all lie in rs_host_alloc'ed memory, 16-B
 * aligned, run zero-copy by default: the kernel reads the survivors and writes the
 * missing shards across PCIe in place.  0 forces the staged H2D -> kernel -> D2H
 * pipeline (A/B and tests). */
int rs_set_host_zero_copy(rs_ctx *ctx, int enable);
/* "zero-copy" or "staged": how the last RS_MEM_HOST batch ran. */
const char *rs_last_host_path(const rs_ctx *ctx);

#ifdef __cplusplus
}
#endif
#endif /* RSGPU_H */
