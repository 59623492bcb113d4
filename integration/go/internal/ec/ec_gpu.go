//go:build rsgpu

// Package ec, GPU build: a drop-in for internal/ec/ec.go that keeps the package
// surface (NewService, Split, Encode, Reconstruct; interfaces.IEcDriver) and runs
// the GF(2^8) arithmetic in librsgpu.so (MI355X / gfx950 HIP kernels) through the
// C-ABI in include/rsgpu.h.  Build with:  CGO_ENABLED=1 go build -tags rsgpu ./...
// (NOT compiled in this repo's image: there is no Go toolchain; see INTEGRATION.md.)
package ec

/*
#cgo CFLAGS: -I${SRCDIR}/../../third_party/rsgpu/include
#cgo LDFLAGS: -L${SRCDIR}/../../third_party/rsgpu/lib -lrsgpu -Wl,-rpath,/opt/rsgpu/lib
#include <stdlib.h>
#include "rsgpu.h"
*/
import "C"

import (
	"crypto/sha256"
	"errors"
	"log"
	"runtime"
	"sync"
	"sync/atomic"
	"time"
	"unsafe"

	"github.com/klauspost/reedsolomon"

	"hybrid_distributed_store/internal/config"
	"hybrid_distributed_store/internal/interfaces"
)

// Service implements interfaces.IEcDriver on the GPU engine (ec.go:15-17).
// Calls go through the engine's batch coalescer: concurrent request goroutines
// with the same shard length share one device launch (group commit), while each
// call keeps rs_encode / rs_reconstruct's exact contract.  One Service drives
// every MI355X of the node (rs_create_multi): the coalescer spreads its batches
// over the GPUs.  enc is the reference's own codec (klauspost, configured exactly
// as ec.go:26) on every host: Split (no arithmetic) always runs there, and on a
// host with no usable GPU (gpu == false) so does every other call.
//
// Encode and Reconstruct use the coalescer's asynchronous calls: the request
// goroutine stages its object (rs_co_submit_*, no blocking in C), then parks on a
// channel; reaper goroutines collect finished calls (rs_co_reap, which also copies
// the staged outputs into the callers' slices -- so several reapers share that copy
// work) and wake their goroutines.  A blocking cgo call would instead hold an OS
// thread per in-flight request and pay a futex sleep and wake-up per object.
//
// Hybrid dispatch (round 6): a call runs on klauspost on its own goroutine instead
// of the GPU unless its shards all lie in one of the Service's Arenas (in place: the
// kernel reads and writes them over PCIe with no staging copy) and the object is at
// least gpuMinObject bytes, and fewer than gpuMaxInflight calls are on the GPU; a call
// that finds no free staging batch (RS_ERR_BUSY) runs on the CPU as well -- a call
// never waits for the GPU.  Measured per object on a 16-CPU quota
// (profiles/r06*_hybrid.log, DESIGN.md §6): a staged call (Go heap shards) costs the
// CPU more in staging copies than klauspost's GFNI kernels spend encoding it, so
// routing those to the GPU lowers throughput at every size, while arena calls of
// >= 100 KiB add the GPU's PCIe-bound rate to the CPU's (800 KiB: 72 -> 91 GiB/s).
type Service struct {
	ctx *C.rs_ctx
	co  *C.rs_coalescer
	enc reedsolomon.Encoder
	gpu bool

	mu      sync.Mutex
	nextTag uint64
	waiting map[uint64]chan int // result codes (Go ints: the tests cannot name cgo types)

	inflight   atomic.Int64 // calls submitted to the GPU and not yet completed
	maxInfl    int64        // gpuMaxInflight (tests may lower it)
	minGPUData int          // gpuMinObject (tests may change it)
	stagedGPU  bool         // tests: staged (non-arena) calls may use the GPU too
	reaping    atomic.Int32 // reaper goroutines still in their loop

	arenaMu sync.RWMutex
	arenas  []*Arena // live arenas: calls on their memory run in place

	// broken: a reaper failed; the calls it left waiting got its error and every
	// later call runs on klauspost (enc).  Set before waiting is flushed (mu).
	broken  atomic.Bool
	closing atomic.Bool
	reapers sync.WaitGroup
}

// Hybrid dispatch thresholds, measured on MI355X with a 16-CPU quota
// (profiles/r06*_hybrid.log, tools/run_hybrid.sh): objects of at least gpuMinObject
// bytes go to the GPU while fewer than gpuMaxInflight calls are in flight there.
const (
	gpuMinObject   = 64 << 10
	gpuMaxInflight = 64
)

// errGPUUnavailable: the call was not submitted (the engine is broken, or busy:
// RS_ERR_BUSY); the caller runs it on the CPU codec instead.
var errGPUUnavailable = errors.New("EC Driver: GPU engine unavailable")

// reapTimeoutUs bounds one rs_co_reap wait so a reaper notices Close.
const reapTimeoutUs = 100000

// useGPU reserves a GPU slot for a call on an object of dataBytes user bytes whose
// shards are `shards`, or says the call runs on the CPU (hybrid dispatch).  A
// reserved slot is released by call() when the call completes or is not submitted.
func (s *Service) useGPU(dataBytes int, shards [][]byte) bool {
	if !s.gpu || s.broken.Load() || dataBytes < s.minGPUData || (!s.stagedGPU && !s.inArena(shards)) {
		return false
	}
	if s.inflight.Add(1) > s.maxInfl {
		s.inflight.Add(-1)
		return false
	}
	return true
}

// call runs one asynchronous coalescer call in the GPU slot useGPU reserved:
// submit(tag) stages it; the result arrives from a reaper.  The caller keeps its
// shard buffers pinned until then.  errGPUUnavailable means nothing was submitted
// (engine broken, or no free staging batch): run the call on the CPU.
func (s *Service) call(submit func(tag C.uint64_t) C.int) error {
	defer s.inflight.Add(-1)
	ch := make(chan int, 1) // buffered: a reaper never blocks on a send
	s.mu.Lock()
	if s.broken.Load() {
		s.mu.Unlock()
		return errGPUUnavailable
	}
	s.nextTag++
	tag := s.nextTag
	s.waiting[tag] = ch
	s.mu.Unlock()
	rc := submit(C.uint64_t(tag))
	if rc == C.RS_OK {
		return toErr(C.int(<-ch)) // a reaper's result, or the error of a reaper that failed
	}
	s.mu.Lock()
	delete(s.waiting, tag) // rejected or busy: never reaped
	s.mu.Unlock()
	if rc == C.RS_ERR_BUSY && !s.closing.Load() {
		return errGPUUnavailable // every staging batch executing or unreaped: the CPU takes it
	}
	return toErr(rc)
}

// reap delivers finished calls to their goroutines; several run per Service.
// rs_co_reap returns 0 on its timeout (or when the coalescer stops) and a negative
// code on bad arguments: then this reaper fails every waiting call with that code
// and switches the Service to the CPU codec (fail, never hang a caller).
func (s *Service) reap() {
	defer s.reapers.Done()
	defer s.reaping.Add(-1)
	const max = 256
	tags := (*[max]C.uint64_t)(C.malloc(max * C.size_t(unsafe.Sizeof(C.uint64_t(0)))))
	rcs := (*[max]C.int)(C.malloc(max * C.size_t(unsafe.Sizeof(C.int(0)))))
	defer C.free(unsafe.Pointer(tags))
	defer C.free(unsafe.Pointer(rcs))
	for !s.closing.Load() && !s.broken.Load() {
		n := int(C.rs_co_reap(s.co, &tags[0], &rcs[0], max, reapTimeoutUs))
		if n < 0 {
			s.fail(-n)
			return
		}
		for i := 0; i < n; i++ {
			s.mu.Lock()
			ch, ok := s.waiting[uint64(tags[i])]
			delete(s.waiting, uint64(tags[i]))
			s.mu.Unlock()
			if ok { // a tag already failed by fail() has no waiter left
				ch <- int(rcs[i])
			}
		}
	}
}

// fail completes every waiting call with rc and sends later calls to the CPU codec.
// The other reapers stop first (they leave their loop once broken is set, within
// one reapTimeoutUs), so no reap copies outputs into a failed caller's buffers after
// it has returned and unpinned them (ADVICE round 5).  Calls whose shards lie in an
// Arena may still be written by a kernel already queued: their buffers must not be
// reused before Close, which drains the coalescer.
func (s *Service) fail(rc int) {
	log.Printf("EC Driver: rs_co_reap failed: %v; failing %d waiting calls, using klauspost/reedsolomon on the CPU from now on",
		toErr(C.int(rc)), s.pending())
	s.broken.Store(true) // before the flush: no call registers after it
	for s.reaping.Load() > 1 { // the other reapers leave their loop within reapTimeoutUs
		time.Sleep(time.Millisecond)
	}
	s.mu.Lock()
	for tag, ch := range s.waiting {
		ch <- rc
		delete(s.waiting, tag)
	}
	s.mu.Unlock()
}

func (s *Service) pending() int {
	s.mu.Lock()
	defer s.mu.Unlock()
	return len(s.waiting)
}

// Close stops the reapers and frees the engine.  No call may be in flight (an
// IEcDriver lives for the process in the reference; this is for tests and a
// graceful shutdown).
func (s *Service) Close() {
	if !s.gpu || s.closing.Swap(true) {
		return
	}
	s.reapers.Wait()
	C.rs_coalescer_destroy(s.co)
	C.rs_destroy(s.ctx)
}

// inArena: every shard's storage (len or, for a missing shard, cap) lies inside one
// live Arena of this Service -- the calls the engine runs in place.
func (s *Service) inArena(shards [][]byte) bool {
	s.arenaMu.RLock()
	defer s.arenaMu.RUnlock()
	for _, a := range s.arenas {
		lo := uintptr(a.base)
		hi := lo + uintptr(a.size)
		all := true
		for _, sh := range shards {
			if cap(sh) == 0 {
				all = false
				break
			}
			p := uintptr(unsafe.Pointer(&sh[:cap(sh)][0]))
			if p < lo || p+uintptr(cap(sh)) > hi {
				all = false
				break
			}
		}
		if all {
			return true
		}
	}
	return false
}

// gpuLaunches: codec kernels the engine has launched on all its GPUs so far
// (rs_device_launches; the routing tests read it).
func (s *Service) gpuLaunches() uint64 {
	if !s.gpu {
		return 0
	}
	var total uint64
	for i := 0; i < int(C.rs_device_count(s.ctx)); i++ {
		var n C.uint64_t
		if C.rs_device_launches(s.ctx, C.int(i), &n) == C.RS_OK {
			total += uint64(n)
		}
	}
	return total
}

// Keep klauspost's exported sentinels so errors.Is and %v output match ec.go.
func toErr(rc C.int) error {
	switch rc {
	case C.RS_OK:
		return nil
	case C.RS_ERR_TOO_FEW_SHARDS:
		return reedsolomon.ErrTooFewShards
	case C.RS_ERR_SHARD_NO_DATA:
		return reedsolomon.ErrShardNoData
	case C.RS_ERR_SHARD_SIZE:
		return reedsolomon.ErrShardSize
	case C.RS_ERR_SHORT_DATA:
		return reedsolomon.ErrShortData
	case C.RS_ERR_INV_SHARD_NUM:
		return reedsolomon.ErrInvShardNum
	case C.RS_ERR_MAX_SHARD_NUM:
		return reedsolomon.ErrMaxShardNum
	case C.RS_ERR_NOT_SUPPORTED:
		return reedsolomon.ErrNotSupported
	default:
		return errors.New(C.GoString(C.rs_strerror(rc)))
	}
}

// NewService replaces reedsolomon.New(config.K, config.M, ...) at ec.go:26.
// Construction fails (log.Fatalf, as ec.go:27-29) only on invalid K/M or a GPU
// runtime error; a GPU-less host gets the CPU codec instead.
func NewService() interfaces.IEcDriver {
	log.Println("--- Initializing EC Driver (Reed-Solomon, MI355X) ---")
	// the reference's codec, exactly ec.go:26: Split on every host, everything on a
	// GPU-less one
	enc, err := reedsolomon.New(config.K, config.M, reedsolomon.WithAutoGoroutines(runtime.NumCPU()))
	if err != nil {
		log.Fatalf("Failed to create Reed-Solomon encoder: %v", err)
	}
	var ctx *C.rs_ctx
	rc := C.rs_create_multi(C.int(config.K), C.int(config.M), 0 /* every visible gfx950 GPU */, 0, &ctx)
	if rc == C.RS_ERR_NO_DEVICE {
		log.Printf("EC Driver loaded (k=%d, m=%d): no MI355X visible (%v), using klauspost/reedsolomon on the CPU\n",
			config.K, config.M, toErr(rc))
		return &Service{enc: enc}
	}
	if rc != C.RS_OK {
		log.Fatalf("Failed to create Reed-Solomon encoder: %v", toErr(rc))
	}
	var co *C.rs_coalescer
	if rc := C.rs_coalescer_create(ctx, nil, &co); rc != C.RS_OK { // defaults: group commit, zero-copy staging
		log.Fatalf("Failed to create Reed-Solomon batch coalescer: %v", toErr(rc))
	}
	log.Printf("EC Driver loaded (k=%d, m=%d) on %s\n", config.K, config.M, C.GoString(C.rs_backend(ctx)))
	s := &Service{ctx: ctx, co: co, enc: enc, gpu: true, waiting: make(map[uint64]chan int),
		maxInfl: gpuMaxInflight, minGPUData: gpuMinObject}
	// reapers share rs_co_reap's output copies: one per 4 Ps, 1..8
	n := min(max(runtime.GOMAXPROCS(0)/4, 1), 8)
	s.reapers.Add(n)
	s.reaping.Store(int32(n))
	for i := 0; i < n; i++ {
		go s.reap()
	}
	return s
}

// Split is klauspost's own Split (ec.go:48-50, writeservice.go:218,382): it does no
// arithmetic, so the GPU build delegates to the reference codec on every host --
// the same shards, aliasing and use of data's spare capacity as before.
func (s *Service) Split(data []byte) ([][]byte, error) {
	return s.enc.Split(data)
}

// shardArgs builds C arrays of shard pointers and lengths.  Every Go pointer
// handed to C is pinned for the duration of the call and never retained.
func shardArgs(shards [][]byte, pin *runtime.Pinner) (**C.uint8_t, *C.size_t, func()) {
	n := len(shards)
	ptrs := (*[1 << 28]*C.uint8_t)(C.malloc(C.size_t(n) * C.size_t(unsafe.Sizeof(uintptr(0)))))[:n:n]
	lens := (*[1 << 28]C.size_t)(C.malloc(C.size_t(n) * C.size_t(unsafe.Sizeof(C.size_t(0)))))[:n:n]
	for i, sh := range shards {
		ptrs[i], lens[i] = nil, C.size_t(len(sh))
		if cap(sh) > 0 {
			p := &sh[:cap(sh)][0]
			pin.Pin(p)
			ptrs[i] = (*C.uint8_t)(unsafe.Pointer(p))
		}
	}
	return &ptrs[0], &lens[0], func() { C.free(unsafe.Pointer(&ptrs[0])); C.free(unsafe.Pointer(&lens[0])) }
}

// Encode fills shards[K:] in place (ec.go:54-56).
func (s *Service) Encode(shards [][]byte) error {
	if len(shards) != config.K+config.M || !s.useGPU(config.K*len(shards[0]), shards) {
		return s.enc.Encode(shards) // klauspost's own checks and sentinels on the CPU path
	}
	var pin runtime.Pinner
	defer pin.Unpin() // after the call completed: the engine writes parity until then
	p, l, free := shardArgs(shards, &pin)
	defer free()
	err := s.call(func(tag C.uint64_t) C.int { return C.rs_co_submit_encode(s.co, p, l, tag) })
	if err == errGPUUnavailable {
		return s.enc.Encode(shards)
	}
	return err
}

// Reconstruct fills every empty entry, data and parity (ec.go:59-61;
// readservice.go:285 and poller.go:282 rely on all nil entries being filled).
func (s *Service) Reconstruct(shards [][]byte) error {
	if !s.gpu || s.broken.Load() || len(shards) != config.K+config.M {
		return s.enc.Reconstruct(shards)
	}
	size := 0
	for _, sh := range shards {
		if len(sh) > 0 {
			size = len(sh)
			break
		}
	}
	if size == 0 || config.K*size < s.minGPUData {
		return s.enc.Reconstruct(shards) // ErrShardNoData, or an object the CPU takes
	}
	missing := 0
	for i := range shards {
		if len(shards[i]) == 0 {
			missing++
			if cap(shards[i]) < size {
				shards[i] = make([]byte, 0, size) // storage for the engine; len 0 = missing
			}
		}
	}
	if missing == 0 { // klauspost: nothing to do (shard sizes are still checked by it)
		for _, sh := range shards {
			if len(sh) != size {
				return reedsolomon.ErrShardSize
			}
		}
		return nil
	}
	if !s.useGPU(config.K*size, shards) {
		return s.enc.Reconstruct(shards) // the GPU has enough in flight: this goroutine computes it
	}
	var pin runtime.Pinner
	defer pin.Unpin()
	p, l, free := shardArgs(shards, &pin)
	defer free()
	err := s.call(func(tag C.uint64_t) C.int { return C.rs_co_submit_reconstruct(s.co, p, l, tag) })
	if err == errGPUUnavailable {
		// nothing was submitted; the entries made above have len 0, so klauspost
		// sees the same missing set and reuses their capacity
		return s.enc.Reconstruct(shards)
	}
	if err != nil {
		return err
	}
	for i := range shards { // every missing entry was filled
		if len(shards[i]) == 0 {
			shards[i] = shards[i][:size]
		}
	}
	return nil
}

// EncodeHash is Encode plus the write path's cold_hash: WriteEC splits and encodes
// `value` (writeservice.go:218-222) and later stores computeSHA256Hex(value) (:267;
// hybrid writes :326, :382-386).  The data shards of Split(value) are the value
// followed by zero padding, so the SHA-256 of their first valueLen = len(value)
// bytes is that hash.  It is computed here with Go's crypto/sha256 (SHA-NI on amd64,
// the reference's own code) while the GPU encodes.  SHA-256 is sequential within a
// message: one GPU lane hashes ~30-40 MB/s against ~2 GB/s for a SHA-NI core, so
// the engine's digest (rs_co_encode_hash) pays only with thousands of values per
// launch (rs_co_encode_hash_many, rs_sha256_batch); per object it cut this path
// from 4-40 GiB/s to 0.5 GiB/s (DESIGN.md §6).  Not part of IEcDriver: a caller
// type-asserts for
//   interface{ EncodeHash([][]byte, int) ([32]byte, error) }
// and keeps Encode + computeSHA256Hex otherwise.
func (s *Service) EncodeHash(shards [][]byte, valueLen int) (sum [32]byte, err error) {
	if len(shards) < config.K {
		return sum, reedsolomon.ErrTooFewShards
	}
	rem := valueLen
	for i := 0; i < config.K && rem > 0; i++ {
		rem -= min(rem, len(shards[i]))
	}
	if rem > 0 {
		return sum, errors.New(C.GoString(C.rs_strerror(C.RS_ERR_INVALID_ARG)))
	}
	done := make(chan struct{})
	go func() { // reads the data shards only, as the encode does
		h := sha256.New()
		left := valueLen
		for i := 0; i < config.K && left > 0; i++ {
			n := min(left, len(shards[i]))
			h.Write(shards[i][:n])
			left -= n
		}
		copy(sum[:], h.Sum(nil))
		close(done)
	}()
	err = s.Encode(shards) // the GPU (klauspost on a GPU-less host)
	<-done
	if err != nil {
		return [32]byte{}, err
	}
	return sum, nil
}

// ReconstructMany repairs many objects in one call (batched healer repair,
// SURVEY.md §8f rank 2): the healer's scan gathers the audited shard sets of the
// damaged objects (poller.go:227-262) and submits them together instead of one
// Reconstruct per worker goroutine (poller.go:282).  errs[i] is exactly what
// Reconstruct(objects[i]) would have returned.  Not part of IEcDriver: the healer
// type-asserts for it and falls back to Reconstruct.
func (s *Service) ReconstructMany(objects [][][]byte) (errs []error) {
	t := config.K + config.M
	errs = make([]error, len(objects))
	if !s.gpu || s.broken.Load() {
		for i, shards := range objects {
			errs[i] = s.enc.Reconstruct(shards)
		}
		return errs
	}
	var pin runtime.Pinner
	defer pin.Unpin()
	flat := make([][]byte, 0, len(objects)*t)
	idx := make([]int, 0, len(objects))
	sizes := make([]int, 0, len(objects))
	for i, shards := range objects {
		if len(shards) != t {
			errs[i] = reedsolomon.ErrTooFewShards
			continue
		}
		size := 0
		for _, sh := range shards {
			if len(sh) > 0 {
				size = len(sh)
				break
			}
		}
		for j := range shards {
			if len(shards[j]) == 0 && cap(shards[j]) < size {
				shards[j] = make([]byte, 0, size)
			}
		}
		flat = append(flat, shards...)
		idx = append(idx, i)
		sizes = append(sizes, size)
	}
	if len(idx) == 0 {
		return errs
	}
	p, l, free := shardArgs(flat, &pin)
	defer free()
	rcs := (*[1 << 24]C.int)(C.malloc(C.size_t(len(idx)) * C.size_t(unsafe.Sizeof(C.int(0)))))[:len(idx):len(idx)]
	defer C.free(unsafe.Pointer(&rcs[0]))
	if rc := C.rs_co_reconstruct_many(s.co, C.size_t(len(idx)), p, l, &rcs[0]); rc != C.RS_OK {
		for _, i := range idx {
			errs[i] = toErr(rc)
		}
		return errs
	}
	lens := unsafe.Slice(l, len(flat))
	for n, i := range idx {
		if errs[i] = toErr(rcs[n]); errs[i] != nil {
			continue
		}
		for j := 0; j < t; j++ {
			if len(objects[i][j]) == 0 && int(lens[n*t+j]) == sizes[n] {
				objects[i][j] = objects[i][j][:sizes[n]]
			}
		}
	}
	return errs
}

// Arena hands out []byte backed by page-locked C memory the engine owns
// (rs_host_alloc: pinned by the driver for life, so no page can move under a call;
// the only host memory the engine's kernels address in place -- Go heap slices and
// rs_host_register'ed memory are staged): a call whose shards -- those it reads and
// those it fills -- all come from an arena runs in place on the GPU, with no staging
// copy of the request body and the parity written straight into the caller's slices
// (DESIGN.md §6, "In place in an arena").  Meant for buffers the service
// owns end to end: the gateway reading a request body into Alloc'd memory before
// Split, parity slices for the storage-node uploads, the healer's shard fetches.
// A bump allocator: Alloc until full, Reset when none of its slices is in use.
// Nil on a GPU-less host (the CPU codec needs no arena).
type Arena struct {
	svc  *Service
	ctx  *C.rs_ctx
	base unsafe.Pointer
	size int
	mu   sync.Mutex
	off  int
}

// NewArena allocates `size` bytes of page-locked memory for in-place calls.
func (s *Service) NewArena(size int) (*Arena, error) {
	if !s.gpu || size <= 0 {
		return nil, nil
	}
	n := (size + 4095) &^ 4095
	var p unsafe.Pointer
	if rc := C.rs_host_alloc(s.ctx, C.size_t(n), &p); rc != C.RS_OK {
		return nil, toErr(rc)
	}
	a := &Arena{svc: s, ctx: s.ctx, base: p, size: n}
	s.arenaMu.Lock()
	s.arenas = append(s.arenas, a)
	s.arenaMu.Unlock()
	return a, nil
}

// Alloc returns n bytes (16-B aligned, len = cap = n) or nil when the arena is full.
func (a *Arena) Alloc(n int) []byte {
	if a == nil || n <= 0 {
		return nil
	}
	a.mu.Lock()
	defer a.mu.Unlock()
	off := (a.off + 15) &^ 15
	if off+n > a.size {
		return nil
	}
	a.off = off + n
	return unsafe.Slice((*byte)(unsafe.Add(a.base, off)), n)
}

// Reset makes the whole arena available again (no slice of it may be in use).
func (a *Arena) Reset() {
	if a != nil {
		a.mu.Lock()
		a.off = 0
		a.mu.Unlock()
	}
}

// Close frees the arena (no call may be using it).
func (a *Arena) Close() {
	if a != nil && a.base != nil {
		a.svc.arenaMu.Lock()
		for i, x := range a.svc.arenas {
			if x == a {
				a.svc.arenas = append(a.svc.arenas[:i], a.svc.arenas[i+1:]...)
				break
			}
		}
		a.svc.arenaMu.Unlock()
		C.rs_host_free(a.ctx, a.base)
		a.base = nil
	}
}
