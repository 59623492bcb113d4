"""IEcDriver over the batch coalescer (include/rsgpu.h rs_coalescer_*, rs_co_*).

Same surface and error behaviour as :class:`ec.Service` -- Split / Encode /
Reconstruct / ReconstructData / Verify, internal/ec/ec.go:48-61 -- but concurrent
callers with the same shard length share one device launch (SURVEY.md §8f rank
1: callers stay unchanged while the GPU sees batches).  ctypes releases the GIL
for the duration of a foreign call, so Python threads really do call in
concurrently, as the reference's request goroutines do.
"""
from __future__ import annotations

import ctypes

from typing import List, Optional, Sequence, Union

from . import _lib
from .ec import ECError, ErrTooFewShards, M, K, Service, _check, _shard_array


class CoalescerOpts(ctypes.Structure):
    _fields_ = [("max_batch", ctypes.c_size_t), ("max_wait_us", ctypes.c_uint32), ("inflight", ctypes.c_int),
                ("max_batch_bytes", ctypes.c_size_t), ("max_exec", ctypes.c_int),
                ("staged_dma", ctypes.c_int), ("spin_waiters", ctypes.c_int), ("plain_copy", ctypes.c_int)]


class CoalescingService(Service):
    def __init__(self, k: int = K, m: int = M, device: Union[int, str, Sequence[int]] = 0, max_batch: int = 0,
                 max_wait_us: int = 0,
                 inflight: int = 0, max_batch_bytes: int = 0, max_exec: int = 0, staged_dma: bool = False):
        super().__init__(k, m, device)
        opts = CoalescerOpts(max_batch, max_wait_us, inflight, max_batch_bytes, max_exec, int(staged_dma))
        co = ctypes.c_void_p()
        _check(_lib.lib().rs_coalescer_create(self._ctx, ctypes.byref(opts), ctypes.byref(co)))
        self._co = co

    def _call(self, op: str, *args) -> int:
        return getattr(_lib.lib(), "rs_co_" + op)(self._co, *args)

    def _many(self, op: str, objects: Sequence[List[Optional[bytearray]]], fill_missing: bool) -> List[Optional[ECError]]:
        t = self.k + self.m
        n = len(objects)
        errs: List[Optional[ECError]] = [None] * n
        ok_idx = [i for i, sh in enumerate(objects) if len(sh) == t]
        for i in range(n):
            if len(objects[i]) != t:
                errs[i] = ECError(ErrTooFewShards)
        ptrs = (_lib._u8p * (len(ok_idx) * t))()
        lens = (ctypes.c_size_t * (len(ok_idx) * t))()
        keep = []
        for j, i in enumerate(ok_idx):
            sh = objects[i]
            S = next((len(s) for s in sh if s is not None and len(s) > 0), 0)
            p, ln, kp = _shard_array(sh, S, fill_missing=fill_missing)
            keep.append(kp)
            for q in range(t):
                ptrs[j * t + q] = p[q]
                lens[j * t + q] = ln[q]
        rcs = (ctypes.c_int * max(1, len(ok_idx)))()
        _check(getattr(_lib.lib(), "rs_co_" + op + "_many")(self._co, len(ok_idx), ptrs, lens, rcs))
        for j, i in enumerate(ok_idx):
            if rcs[j] != _lib.RS_OK:
                errs[i] = ECError(rcs[j])
            elif fill_missing:
                sh = objects[i]
                for q in range(t):
                    if (sh[q] is None or len(sh[q]) == 0) and lens[j * t + q] > 0:
                        sh[q] = bytearray(ctypes.string_at(ptrs[j * t + q], lens[j * t + q]))
        del keep
        return errs

    def ReconstructMany(self, objects: Sequence[List[Optional[bytearray]]]) -> List[Optional[ECError]]:
        """Reconstruct for many objects in one call (rs_co_reconstruct_many): each
        list is filled in place exactly as Reconstruct would; returns per-object
        errors (None = ok)."""
        return self._many("reconstruct", objects, True)

    def EncodeMany(self, objects: Sequence[List[bytearray]]) -> List[Optional[ECError]]:
        return self._many("encode", objects, False)

    def EncodeHash(self, shards: List[bytearray], value_len: int) -> bytes:
        """Encode (parity in place) plus the write path's cold_hash in the same
        coalesced batch (rs_co_encode_hash): returns SHA-256 of the first value_len
        bytes of the data shards -- the value Split was given (writeservice.go:218-222,
        :267)."""
        if len(shards) != self.k + self.m:
            raise ECError(ErrTooFewShards)
        ptrs, lens, keep = _shard_array(shards, 0, fill_missing=False)
        digest = (ctypes.c_uint8 * 32)()
        _check(_lib.lib().rs_co_encode_hash(self._co, ptrs, lens, value_len, ctypes.cast(digest, _lib._u8p)))
        del keep
        return bytes(digest)

    def EncodeHashMany(self, objects: Sequence[List[bytearray]], value_lens: Sequence[int]):
        """rs_co_encode_hash_many: per object (error or None, digest or None)."""
        t = self.k + self.m
        n = len(objects)
        ptrs = (_lib._u8p * (n * t))()
        lens = (ctypes.c_size_t * (n * t))()
        keep = []
        for i, sh in enumerate(objects):
            if len(sh) != t:
                raise ECError(ErrTooFewShards)
            p, ln, kp = _shard_array(sh, 0, fill_missing=False)
            keep.append(kp)
            for q in range(t):
                ptrs[i * t + q] = p[q]
                lens[i * t + q] = ln[q]
        vl = (ctypes.c_size_t * max(1, n))(*value_lens)
        digests = (ctypes.c_uint8 * (32 * max(1, n)))()
        rcs = (ctypes.c_int * max(1, n))()
        _check(_lib.lib().rs_co_encode_hash_many(self._co, n, ptrs, lens, vl, ctypes.cast(digests, _lib._u8p), rcs))
        del keep
        raw = bytes(digests)
        return [(ECError(rcs[i]) if rcs[i] else None, None if rcs[i] else raw[32 * i:32 * i + 32]) for i in range(n)]

    def stats(self) -> dict:
        v = [ctypes.c_uint64() for _ in range(4)]
        _check(_lib.lib().rs_co_stats(self._co, *[ctypes.byref(x) for x in v]))
        return dict(zip(("calls", "batches", "stripes", "max_batch"), (x.value for x in v)))

    def close(self) -> None:
        if getattr(self, "_co", None):
            _lib.lib().rs_coalescer_destroy(self._co)
            self._co = None
        super().close()
