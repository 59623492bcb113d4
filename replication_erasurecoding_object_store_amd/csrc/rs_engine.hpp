// rs_engine.hpp -- internal interface between the context / dispatch layer
// (rs_engine.cpp) and the batch coalescer (rs_coalescer.cpp).  Not part of the
// C-ABI.
//
// An rs_ctx owns one Engine per device it spans (rs_create: one; rs_create_multi /
// rs_create_devices: several, one process driving several GPUs the way the
// reference's single IEcDriver serves every request goroutine,
// cmd/api/main.go:206).  An Engine is everything one GPU needs: plans and LUT in
// its HBM, streams, staging, status words.  The coalescer stages batches in
// portable pinned memory and hands each one to the least-loaded Engine.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

#include "../../include/rsgpu.h"

namespace rs {

struct Engine;

int ctx_engine_count(const rs_ctx* c);
Engine* ctx_engine(rs_ctx* c, int i);
int engine_device(const Engine* e);

// Makes `device` current for the scope and restores the caller's device after, so
// library calls never change the calling thread's HIP device (a Go thread or a
// torch program may be using another GPU).
class DeviceScope {
 public:
  explicit DeviceScope(int device) {
    if (hipGetDevice(&prev_) != hipSuccess) prev_ = -1;
    if (prev_ != device) ok_ = hipSetDevice(device) == hipSuccess;
    else prev_ = -1;  // nothing to restore
  }
  ~DeviceScope() {
    if (prev_ >= 0) (void)hipSetDevice(prev_);
  }
  bool ok() const { return ok_; }
  DeviceScope(const DeviceScope&) = delete;
  DeviceScope& operator=(const DeviceScope&) = delete;

 private:
  int prev_ = -1;
  bool ok_ = true;
};

// Device-resident batch entry points on one Engine (asynchronous on s, which must
// belong to the engine's device; the caller holds a DeviceScope for it).
// Contracts as rs_encode_batch / rs_reconstruct_batch_out(_devmask) / rs_verify_batch
// with RS_MEM_DEVICE; the pointers may also be GPU-mapped pinned host memory.
// max_missing bounds device masks (0 = m; see rs_reconstruct_batch_out_devmask).
int engine_encode_batch(Engine* e, const uint8_t* data, size_t data_sp, uint8_t* parity, size_t parity_sp,
                        size_t pitch, size_t S, size_t N, hipStream_t s);
int engine_reconstruct_batch_out(Engine* e, const uint8_t* data, size_t data_sp, const uint8_t* parity,
                                 size_t parity_sp, size_t pitch, size_t S, size_t N, const uint32_t* masks,
                                 size_t n_masks, int masks_on_device, int max_missing, uint8_t* out, size_t out_sp,
                                 hipStream_t s);
int engine_reconstruct_batch_packed(Engine* e, const uint8_t* data, size_t data_sp, const uint8_t* parity,
                                    size_t parity_sp, size_t pitch, size_t S, size_t N, const uint32_t* masks,
                                    int masks_on_device, uint8_t* out, uint32_t* row_offsets, hipStream_t s);
int engine_verify_batch(Engine* e, const uint8_t* data, size_t data_sp, const uint8_t* parity, size_t parity_sp,
                        size_t pitch, size_t S, size_t N, uint32_t* bad_dev, hipStream_t s);
// Device address of the plan for one pattern on this engine (cached; thread-safe):
// reconstruct (data_only: ReconstructData) of `present`, or the encode plan.
int engine_plan_for(Engine* e, uint64_t present, bool data_only, const uint8_t** plan);
const uint8_t* engine_encode_plan(Engine* e);
// Out-of-place batch with a plan per stripe (any k+m; the coalescer's k+m > 16
// batches): the r-th output of stripe i at out + i*out_sp + r*pitch, the plan's
// inputs read from the split layout.  plans_dev: n device-visible plan addresses.
int engine_apply_batch_plans(Engine* e, const uint8_t* data, size_t data_sp, const uint8_t* parity,
                             size_t parity_sp, size_t pitch, size_t S, size_t N, const uint64_t* plans_dev,
                             uint8_t* out, size_t out_sp, hipStream_t s);
// Per-stripe masks (k+m <= 16) over a table of shard addresses: stripe i's shard s
// at shard_ptrs_dev[i*(k+m) + s], every shard S bytes and 16-B aligned, inputs the
// first k present, outputs the missing shards' buffers; nothing outside [0, S) of
// any shard is written (apply_ptr_kernel).  RS_ERR_NOT_SUPPORTED for (k, m) without
// a specialised kernel (the caller then stages).  The status word of s collects
// deferred errors as for device masks.
int engine_apply_batch_ptrs(Engine* e, const uint64_t* shard_ptrs_dev, const uint32_t* masks_dev, size_t S,
                            size_t N, int max_missing, hipStream_t s);
// GPU address of [p, p + bytes) when it lies inside one range of page-locked memory
// the context allocated itself (rs_host_alloc), else nullptr.  Only such memory is
// ever read or written in place by a kernel: its pages are the driver's and never
// move.  Caller memory -- rs_host_register'ed ranges included -- is staged
// (DESIGN.md §2).  Cheap when the context owns no host memory.
uint8_t* ctx_owned(rs_ctx* c, const void* p, size_t bytes);
bool apply_ptrs_supported(int k, int m);  // engine_apply_batch_ptrs has a kernel for (k, m)

}  // namespace rs
