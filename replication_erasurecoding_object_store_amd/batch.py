"""Batched API over librsgpu.so (the throughput path).

torch provides device memory and the stream (plumbing only): tensors are passed to
the C-ABI as raw pointers and kernels run on torch's *current* stream, so
``torch.cuda.Event`` brackets them exactly.

Layouts (include/rsgpu.h):
  split   data [N, K, P] + parity [N, M, P]  -- the fast device layout (two
          sequential streams; object i's K data shards contiguous = its Split view)
  unified one buffer [N, K+M, P]             -- parity = data + K*P
P (shard pitch) >= S rounded up to 16; :func:`shard_pitch_for` picks 256-B multiples.
"""
from __future__ import annotations

import ctypes
from typing import Optional

import numpy as np

from . import _lib
from .ec import ECError, Service


def _check(rc: int) -> None:
    if rc != _lib.RS_OK:
        raise ECError(rc)


def shard_pitch_for(shard_len: int) -> int:
    """Device shard slot: 256-B multiple (16 B is the contract).  Slots that start
    mid-128-B-line make every 1 KiB wave access touch 9 lines instead of 8: a
    compute-free RS(10+4) stream at S = 6 554 ran 5.65 TB/s with a 6 592-B pitch
    and 6.30 TB/s with 6 656 (profiles/r01_hbm_probe4.log)."""
    return (shard_len + 255) // 256 * 256


def _stream_handle(stream=None) -> ctypes.c_void_p:
    import torch
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


def _masks(present_masks) -> np.ndarray:
    return np.ascontiguousarray(np.atleast_1d(np.asarray(present_masks, dtype=np.uint32)))


def _u32p(a: np.ndarray):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))


class BatchEngine(Service):
    """Service plus the batched entry points (rs_*_batch).

    Out-of-place outputs are whole-pitch tensors ([N, rows, P] with P the shard
    pitch; reconstruct_out derives the stripe pitch from the tensor), so every
    output row owns its padding up to the next 128-B line: the engine turns
    rs_set_out_pad_writes on (the C-ABI default is exact rows)."""

    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.set_out_pad_writes(True)

    # ---- device-resident, split layout --------------------------------------------
    def encode(self, data, parity, shard_len: int, n_stripes: int, shard_pitch: Optional[int] = None,
               data_stripe_pitch: Optional[int] = None, parity_stripe_pitch: Optional[int] = None,
               stream=None) -> None:
        """data [N, K, P] / parity [N, M, P] uint8 device tensors.  Asynchronous."""
        P = shard_pitch or data.shape[-1]
        dsp = data_stripe_pitch or self.k * P
        psp = parity_stripe_pitch or self.m * P
        _check(_lib.lib().rs_encode_batch(self.ctx, data.data_ptr(), dsp, parity.data_ptr(), psp, P, shard_len,
                                          n_stripes, _lib.RS_MEM_DEVICE, _stream_handle(stream)))

    def reconstruct(self, data, parity, shard_len: int, n_stripes: int, present_masks,
                    shard_pitch: Optional[int] = None, stream=None) -> None:
        """present_masks: int (one pattern) or host uint32 array (one per stripe)."""
        P = shard_pitch or data.shape[-1]
        m = _masks(present_masks)
        _check(_lib.lib().rs_reconstruct_batch(self.ctx, data.data_ptr(), self.k * P, parity.data_ptr(), self.m * P,
                                               P, shard_len, n_stripes, _u32p(m), m.size, _lib.RS_MEM_DEVICE,
                                               _stream_handle(stream)))

    def reconstruct_devmask(self, data, parity, shard_len: int, n_stripes: int, masks_dev,
                            shard_pitch: Optional[int] = None, stream=None) -> None:
        P = shard_pitch or data.shape[-1]
        _check(_lib.lib().rs_reconstruct_batch_devmask(self.ctx, data.data_ptr(), self.k * P, parity.data_ptr(),
                                                       self.m * P, P, shard_len, n_stripes, masks_dev.data_ptr(),
                                                       _stream_handle(stream)))

    def reconstruct_out(self, data, parity, out, shard_len: int, n_stripes: int, present_masks=None,
                        masks_dev=None, shard_pitch: Optional[int] = None, stream=None,
                        max_missing: int = 0) -> None:
        """Out-of-place: the r-th missing shard of stripe i goes to out[i, r].
        `present_masks` (host: int or uint32 array) or `masks_dev` (device tensor);
        with device masks, `max_missing` > 0 is the caller's bound on erasures per
        stripe (rs_reconstruct_batch_out_devmask)."""
        P = shard_pitch or data.shape[-1]
        osp = out.shape[-2] * out.shape[-1] if out.dim() == 3 else self.m * P
        if masks_dev is not None and max_missing:
            _check(_lib.lib().rs_reconstruct_batch_out_devmask(
                self.ctx, data.data_ptr(), self.k * P, parity.data_ptr(), self.m * P, P, shard_len, n_stripes,
                masks_dev.data_ptr(), max_missing, out.data_ptr(), osp, _stream_handle(stream)))
            return
        if masks_dev is not None:
            mptr, n, on_dev = ctypes.c_void_p(masks_dev.data_ptr()), n_stripes, 1
            keep = None
        else:
            keep = _masks(present_masks)
            mptr, n, on_dev = ctypes.c_void_p(keep.ctypes.data), keep.size, 0
        _check(_lib.lib().rs_reconstruct_batch_out(self.ctx, data.data_ptr(), self.k * P, parity.data_ptr(),
                                                   self.m * P, P, shard_len, n_stripes, mptr, n, on_dev,
                                                   out.data_ptr(), osp, _stream_handle(stream)))
        del keep

    def reconstruct_packed(self, data, parity, out, row_offsets, shard_len: int, n_stripes: int,
                           present_masks=None, masks_dev=None, shard_pitch: Optional[int] = None,
                           stream=None) -> None:
        """Packed out-of-place reconstruct (rs_reconstruct_batch_out_packed): the missing
        shards of the batch back to back, stripe i's r-th at row row_offsets[i] + r of
        `out` (rows of shard_pitch bytes); row_offsets: int32/uint32 device tensor of
        n_stripes + 1, filled by the call.  Masks: host array or device tensor."""
        P = shard_pitch or data.shape[-1]
        if masks_dev is not None:
            mptr, on_dev, keep = ctypes.c_void_p(masks_dev.data_ptr()), 1, None
        else:
            keep = _masks(present_masks)
            if keep.size != n_stripes:
                raise ValueError("present_masks: one per stripe")
            mptr, on_dev = ctypes.c_void_p(keep.ctypes.data), 0
        _check(_lib.lib().rs_reconstruct_batch_out_packed(
            self.ctx, data.data_ptr(), self.k * P, parity.data_ptr(), self.m * P, P, shard_len, n_stripes, mptr,
            on_dev, out.data_ptr(), row_offsets.data_ptr(), _stream_handle(stream)))
        del keep

    def verify(self, data, parity, bad, shard_len: int, n_stripes: int, shard_pitch: Optional[int] = None,
               stream=None) -> None:
        """Scrub: bad [N] int32/uint32 device tensor <- bitmask of mismatching parity
        shards per stripe (0 = intact).  Asynchronous; nothing else is written."""
        P = shard_pitch or data.shape[-1]
        _check(_lib.lib().rs_verify_batch(self.ctx, data.data_ptr(), self.k * P, parity.data_ptr(), self.m * P, P,
                                          shard_len, n_stripes, bad.data_ptr(), _lib.RS_MEM_DEVICE,
                                          _stream_handle(stream)))

    def sha256(self, data, length: int, n: int, stride: Optional[int] = None, digests=None, stream=None):
        """SHA-256 of n device messages at data + i*stride (`length` bytes each) ->
        uint8 [n, 32] device tensor (the reference's cold_hash).  Asynchronous."""
        import torch

        if digests is None:
            digests = torch.empty((n, 32), dtype=torch.uint8, device=data.device)
        st = stride if stride is not None else length
        _check(_lib.lib().rs_sha256_batch(self.ctx, data.data_ptr(), st, length, n, digests.data_ptr(),
                                          _stream_handle(stream)))
        return digests

    def sha256_var(self, base, offsets, lens, digests=None, stream=None):
        """Variable-length messages: base (uint8 device tensor), offsets / lens
        (int64 device tensors of n) -> uint8 [n, 32]."""
        import torch

        n = offsets.numel()
        if digests is None:
            digests = torch.empty((n, 32), dtype=torch.uint8, device=base.device)
        _check(_lib.lib().rs_sha256_batch_var(self.ctx, base.data_ptr(), offsets.data_ptr(), lens.data_ptr(), n,
                                              digests.data_ptr(), _stream_handle(stream)))
        return digests

    # ---- device-resident, unified layout ------------------------------------------
    def encode_unified(self, buf, shard_len: int, shard_pitch: int, n_stripes: int, stream=None) -> None:
        """buf: [n_stripes, k+m, shard_pitch] uint8 device tensor; fills parity slots."""
        sp = (self.k + self.m) * shard_pitch
        base = buf.data_ptr()
        _check(_lib.lib().rs_encode_batch(self.ctx, base, sp, base + self.k * shard_pitch, sp, shard_pitch,
                                          shard_len, n_stripes, _lib.RS_MEM_DEVICE, _stream_handle(stream)))

    def reconstruct_unified(self, buf, shard_len: int, shard_pitch: int, n_stripes: int, present_masks,
                            stream=None) -> None:
        m = _masks(present_masks)
        sp = (self.k + self.m) * shard_pitch
        base = buf.data_ptr()
        _check(_lib.lib().rs_reconstruct_batch(self.ctx, base, sp, base + self.k * shard_pitch, sp, shard_pitch,
                                               shard_len, n_stripes, _u32p(m), m.size, _lib.RS_MEM_DEVICE,
                                               _stream_handle(stream)))

    def reconstruct_unified_devmask(self, buf, shard_len: int, shard_pitch: int, n_stripes: int, masks_dev,
                                    stream=None) -> None:
        sp = (self.k + self.m) * shard_pitch
        base = buf.data_ptr()
        _check(_lib.lib().rs_reconstruct_batch_devmask(self.ctx, base, sp, base + self.k * shard_pitch, sp,
                                                       shard_pitch, shard_len, n_stripes, masks_dev.data_ptr(),
                                                       _stream_handle(stream)))

    def sync(self, stream=None) -> None:
        _check(_lib.lib().rs_sync(self.ctx, _stream_handle(stream)))

    def stream_release(self, stream=None) -> None:
        """rs_sync, then the engine forgets the stream (before destroying it)."""
        _check(_lib.lib().rs_stream_release(self.ctx, _stream_handle(stream)))

    # ---- host-resident (synchronous, pipelined H2D / kernel / D2H) -------------------
    def encode_host(self, data: np.ndarray, parity: np.ndarray, shard_len: int, n_stripes: int,
                    shard_pitch: Optional[int] = None) -> None:
        """data [N, K, P] / parity [N, M, P] host uint8 arrays."""
        P = shard_pitch or data.shape[-1]
        _check(_lib.lib().rs_encode_batch(self.ctx, data.ctypes.data, self.k * P, parity.ctypes.data, self.m * P, P,
                                          shard_len, n_stripes, _lib.RS_MEM_HOST, None))

    def reconstruct_host(self, data: np.ndarray, parity: np.ndarray, shard_len: int, n_stripes: int,
                         present_masks, shard_pitch: Optional[int] = None) -> None:
        P = shard_pitch or data.shape[-1]
        m = _masks(present_masks)
        _check(_lib.lib().rs_reconstruct_batch(self.ctx, data.ctypes.data, self.k * P, parity.ctypes.data,
                                               self.m * P, P, shard_len, n_stripes, _u32p(m), m.size,
                                               _lib.RS_MEM_HOST, None))

    def encode_host_unified(self, buf: np.ndarray, shard_len: int, shard_pitch: int, n_stripes: int) -> None:
        sp = (self.k + self.m) * shard_pitch
        base = buf.ctypes.data
        _check(_lib.lib().rs_encode_batch(self.ctx, base, sp, base + self.k * shard_pitch, sp, shard_pitch,
                                          shard_len, n_stripes, _lib.RS_MEM_HOST, None))

    def reconstruct_host_unified(self, buf: np.ndarray, shard_len: int, shard_pitch: int, n_stripes: int,
                                 present_masks) -> None:
        m = _masks(present_masks)
        sp = (self.k + self.m) * shard_pitch
        base = buf.ctypes.data
        _check(_lib.lib().rs_reconstruct_batch(self.ctx, base, sp, base + self.k * shard_pitch, sp, shard_pitch,
                                               shard_len, n_stripes, _u32p(m), m.size, _lib.RS_MEM_HOST, None))

    def verify_host(self, data: np.ndarray, parity: np.ndarray, shard_len: int, n_stripes: int,
                    shard_pitch: Optional[int] = None) -> np.ndarray:
        """Host-resident scrub: returns uint32 [N] mismatch bitmasks."""
        P = shard_pitch or data.shape[-1]
        bad = np.empty(n_stripes, np.uint32)
        _check(_lib.lib().rs_verify_batch(self.ctx, data.ctypes.data, self.k * P, parity.ctypes.data, self.m * P, P,
                                          shard_len, n_stripes, bad.ctypes.data, _lib.RS_MEM_HOST, None))
        return bad

    def host_register(self, arr: np.ndarray) -> None:
        """Records arr as caller memory (rs_host_register): never mapped into the GPU,
        calls on it are staged; host_alloc gives memory the kernels use in place."""
        _check(_lib.lib().rs_host_register(self.ctx, arr.ctypes.data, arr.nbytes))

    def host_unregister(self, arr: np.ndarray) -> None:
        _check(_lib.lib().rs_host_unregister(self.ctx, arr.ctypes.data))

    def host_alloc(self, nbytes: int) -> np.ndarray:
        """Page-locked host memory owned by the context (rs_host_alloc) as a uint8
        array; free with host_free before the engine closes (or let close free it)."""
        p = ctypes.c_void_p()
        _check(_lib.lib().rs_host_alloc(self.ctx, nbytes, ctypes.byref(p)))
        return np.ctypeslib.as_array((ctypes.c_uint8 * nbytes).from_address(p.value))

    def host_free(self, arr: np.ndarray) -> None:
        _check(_lib.lib().rs_host_free(self.ctx, arr.ctypes.data))

    # ---- measurement helpers ----------------------------------------------------------
    def device_copy(self, dst, src, nbytes: Optional[int] = None, stream=None) -> None:
        n = nbytes if nbytes is not None else src.numel() * src.element_size()
        _check(_lib.lib().rs_device_copy(self.ctx, dst.data_ptr(), src.data_ptr(), n, _stream_handle(stream)))

    def last_kernel(self) -> str:
        return _lib.lib().rs_last_kernel(self.ctx).decode()

    def last_kernel_on(self, stream=None) -> str:
        """The last kernel this context launched on `stream` (torch's current stream by
        default): names the launch before a device error on that stream."""
        return _lib.lib().rs_last_kernel_on(self.ctx, _stream_handle(stream)).decode()

    def set_host_zero_copy(self, enable: bool) -> None:
        _check(_lib.lib().rs_set_host_zero_copy(self.ctx, 1 if enable else 0))

    def last_host_path(self) -> str:
        return _lib.lib().rs_last_host_path(self.ctx).decode()

    def set_blocks_per_cu(self, n: int) -> None:
        _check(_lib.lib().rs_set_blocks_per_cu(self.ctx, n))

    def set_occupancy_cap(self, waves_per_simd: int) -> None:
        """-1: each kernel's tuned default; 0: uncapped; c: at most c waves per SIMD."""
        _check(_lib.lib().rs_set_occupancy_cap(self.ctx, waves_per_simd))

    def set_out_pad_writes(self, enable: bool) -> None:
        """Out-of-place reconstructs may write each output row's padding up to the
        next 128-B line (rsgpu.h)."""
        _check(_lib.lib().rs_set_out_pad_writes(self.ctx, 1 if enable else 0))

    def set_parity_pad_writes(self, enable: bool) -> None:
        """Encode may write parity slot padding up to the next 128-B line (rsgpu.h)."""
        _check(_lib.lib().rs_set_parity_pad_writes(self.ctx, 1 if enable else 0))
