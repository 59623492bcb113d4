"""Batched device-resident API over librsgpu.so (the throughput path).

torch provides device memory and the stream (plumbing only): tensors are passed to
the C-ABI as raw pointers, kernels run on torch's *current* stream so that
``torch.cuda.Event`` brackets them exactly.

Layout (unified, SURVEY.md 8d "shard-major per stripe"): a uint8 tensor viewed as
[n_stripes, k+m, shard_pitch]; shard s of stripe i is row (i, s); the first
shard_len bytes of each row are the shard, the rest is padding.
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
    """Device shard slot: 64-B multiple (16 B is the contract; 64 keeps every
    wave's 1 KiB column block on whole 64-B lines)."""
    return (shard_len + 63) // 64 * 64


def _stream_handle(stream=None) -> ctypes.c_void_p:
    import torch
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


class BatchEngine(Service):
    """Service plus the batched entry points (rs_*_batch)."""

    def encode_batch(self, data, parity, shard_len: int, shard_pitch: int, n_stripes: int,
                     data_stripe_pitch: int, parity_stripe_pitch: int, stream=None) -> None:
        """data/parity: device tensors (uint8).  Asynchronous on `stream`."""
        _check(_lib.lib().rs_encode_batch(self.ctx, data.data_ptr(), data_stripe_pitch, parity.data_ptr(),
                                          parity_stripe_pitch, shard_pitch, shard_len, n_stripes,
                                          _lib.RS_MEM_DEVICE, _stream_handle(stream)))

    def encode_unified(self, buf, shard_len: int, shard_pitch: int, n_stripes: int, stream=None) -> None:
        """buf: [n_stripes, k+m, shard_pitch] uint8 device tensor; fills parity slots."""
        sp = (self.k + self.m) * shard_pitch
        base = buf.data_ptr()
        _check(_lib.lib().rs_encode_batch(self.ctx, base, sp, base + self.k * shard_pitch, sp, shard_pitch,
                                          shard_len, n_stripes, _lib.RS_MEM_DEVICE, _stream_handle(stream)))

    def reconstruct_unified(self, buf, shard_len: int, shard_pitch: int, n_stripes: int, present_masks,
                            stream=None) -> None:
        """present_masks: int or host array of uint32 (one per stripe)."""
        masks = np.ascontiguousarray(np.atleast_1d(np.asarray(present_masks, dtype=np.uint32)))
        sp = (self.k + self.m) * shard_pitch
        _check(_lib.lib().rs_reconstruct_batch(
            self.ctx, buf.data_ptr(), sp, shard_pitch, shard_len, n_stripes,
            masks.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), masks.size, _lib.RS_MEM_DEVICE,
            _stream_handle(stream)))

    def reconstruct_unified_devmask(self, buf, shard_len: int, shard_pitch: int, n_stripes: int, masks_dev,
                                    stream=None) -> None:
        sp = (self.k + self.m) * shard_pitch
        _check(_lib.lib().rs_reconstruct_batch_devmask(self.ctx, buf.data_ptr(), sp, shard_pitch, shard_len,
                                                       n_stripes, masks_dev.data_ptr(), _stream_handle(stream)))

    def sync(self, stream=None) -> None:
        _check(_lib.lib().rs_sync(self.ctx, _stream_handle(stream)))

    # ---- host-resident batches (synchronous, pipelined H2D/kernel/D2H) ---------
    def encode_host(self, buf: np.ndarray, shard_len: int, shard_pitch: int, n_stripes: int) -> None:
        sp = (self.k + self.m) * shard_pitch
        base = buf.ctypes.data
        _check(_lib.lib().rs_encode_batch(self.ctx, base, sp, base + self.k * shard_pitch, sp, shard_pitch,
                                          shard_len, n_stripes, _lib.RS_MEM_HOST, None))

    def reconstruct_host(self, buf: np.ndarray, shard_len: int, shard_pitch: int, n_stripes: int,
                         present_masks) -> None:
        masks = np.ascontiguousarray(np.atleast_1d(np.asarray(present_masks, dtype=np.uint32)))
        sp = (self.k + self.m) * shard_pitch
        _check(_lib.lib().rs_reconstruct_batch(
            self.ctx, buf.ctypes.data, sp, shard_pitch, shard_len, n_stripes,
            masks.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), masks.size, _lib.RS_MEM_HOST, None))

    def host_register(self, arr: np.ndarray) -> None:
        _check(_lib.lib().rs_host_register(self.ctx, arr.ctypes.data, arr.nbytes))

    def host_unregister(self, arr: np.ndarray) -> None:
        _check(_lib.lib().rs_host_unregister(self.ctx, arr.ctypes.data))

    def device_copy(self, dst, src, nbytes: Optional[int] = None, stream=None) -> None:
        n = nbytes if nbytes is not None else src.numel() * src.element_size()
        _check(_lib.lib().rs_device_copy(self.ctx, dst.data_ptr(), src.data_ptr(), n, _stream_handle(stream)))

    def last_kernel(self) -> str:
        return _lib.lib().rs_last_kernel(self.ctx).decode()

    def set_blocks_per_cu(self, n: int) -> None:
        _check(_lib.lib().rs_set_blocks_per_cu(self.ctx, n))
