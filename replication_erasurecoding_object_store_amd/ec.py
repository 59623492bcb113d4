"""Host-side mirror of the reference's ``internal/ec`` package over librsgpu.so.

Reference surface (kept name-for-name so tests read like the reference's):
  internal/ec/ec.go:15-17   type Service struct { driver reedsolomon.Encoder }
  internal/ec/ec.go:21-44   func NewService() interfaces.IEcDriver
  internal/ec/ec.go:48-50   func (s *Service) Split(data []byte) ([][]byte, error)
  internal/ec/ec.go:54-56   func (s *Service) Encode(shards [][]byte) error
  internal/ec/ec.go:59-61   func (s *Service) Reconstruct(shards [][]byte) error
  internal/interfaces/interfaces.go:41-52  IEcDriver
  internal/config/config.go:20-23          K = 4, M = 2

Go's ``[][]byte`` maps to a Python list whose entries are ``bytearray`` (or
``None``/empty for a nil shard); Go's ``error`` maps to :class:`ECError`, whose
message is klauspost's sentinel text.  Every parity / reconstructed byte is
computed by the HIP kernels behind the C-ABI; this module only marshals.
"""
from __future__ import annotations

import ctypes
import weakref
from typing import List, Optional, Sequence, Union

from . import _lib

K = 4  # internal/config/config.go:21
M = 2  # internal/config/config.go:22


class ECError(Exception):
    """A codec error; ``str(e)`` is the klauspost sentinel message."""

    def __init__(self, code: int):
        self.code = code
        super().__init__(_lib.strerror(code))


# klauspost v1.12.1 errors.go: Split's sentinel is produced on the host.
ErrShortData = _lib.RS_ERR_SHORT_DATA
ErrTooFewShards = _lib.RS_ERR_TOO_FEW_SHARDS
ErrShardNoData = _lib.RS_ERR_SHARD_NO_DATA
ErrShardSize = _lib.RS_ERR_SHARD_SIZE


def _check(rc: int) -> None:
    if rc != _lib.RS_OK:
        raise ECError(rc)


def _shard_array(shards: Sequence[Optional[bytearray]], S: int, fill_missing: bool):
    """Build (u8** ptrs, size_t* lens, keepalive) for a K+M shard list."""
    n = len(shards)
    ptrs = (_lib._u8p * n)()
    lens = (ctypes.c_size_t * n)()
    keep = []
    for i, sh in enumerate(shards):
        if sh is None or len(sh) == 0:
            lens[i] = 0
            if fill_missing:
                buf = (ctypes.c_uint8 * max(S, 1))()
                keep.append(buf)
                ptrs[i] = ctypes.cast(buf, _lib._u8p)
            continue
        if not isinstance(sh, (bytearray, memoryview)) or (isinstance(sh, memoryview) and sh.readonly):
            raise TypeError("shards must be bytearray or a writable memoryview (mutable, like Go []byte) or None")
        buf = (ctypes.c_uint8 * len(sh)).from_buffer(sh)
        keep.append(buf)
        ptrs[i] = ctypes.cast(buf, _lib._u8p)
        lens[i] = len(sh)
    return ptrs, lens, keep


def _create(k: int, m: int, device: Union[int, str, Sequence[int]]) -> ctypes.c_void_p:
    """device: an ordinal (rs_create), "all" (rs_create_multi over every visible
    GPU) or a list of ordinals (rs_create_devices; repeats allowed)."""
    handle = ctypes.c_void_p()
    if isinstance(device, str):
        if device != "all":
            raise ValueError(f"device must be an ordinal, 'all' or a list, not {device!r}")
        _check(_lib.lib().rs_create_multi(k, m, 0, 0, ctypes.byref(handle)))
    elif isinstance(device, int):
        _check(_lib.lib().rs_create(k, m, device, 0, ctypes.byref(handle)))
    else:
        devs = (ctypes.c_int * len(device))(*device)
        _check(_lib.lib().rs_create_devices(k, m, devs, len(device), 0, ctypes.byref(handle)))
    return handle


class Service:
    """IEcDriver implementation on the MI355X engine (internal/ec/ec.go:15-17)."""

    def __init__(self, k: int = K, m: int = M, device: Union[int, str, Sequence[int]] = 0):
        self._ctx = _create(k, m, device)
        self.k, self.m = k, m
        self._arenas = weakref.WeakSet()  # invalidated before rs_destroy frees their memory

    def close(self) -> None:
        if getattr(self, "_ctx", None):
            for a in list(getattr(self, "_arenas", ())):
                a._invalidate()
            _lib.lib().rs_destroy(self._ctx)
            self._ctx = None

    def __del__(self):  # pragma: no cover - best effort
        try:
            self.close()
        except Exception:
            pass

    @property
    def ctx(self) -> ctypes.c_void_p:
        return self._ctx

    def backend(self) -> str:
        return _lib.lib().rs_backend(self._ctx).decode()

    def devices(self) -> List[int]:
        """HIP ordinals of the context's engines (one per GPU, or repeats)."""
        L = _lib.lib()
        return [L.rs_device_at(self._ctx, i) for i in range(L.rs_device_count(self._ctx))]

    def device_launches(self) -> List[int]:
        """Codec kernels launched on each engine since creation (rs_device_launches)."""
        L = _lib.lib()
        out = []
        for i in range(L.rs_device_count(self._ctx)):
            v = ctypes.c_uint64()
            _check(L.rs_device_launches(self._ctx, i, ctypes.byref(v)))
            out.append(v.value)
        return out

    def encode_matrix(self) -> List[List[int]]:
        t = self.k + self.m
        out = (ctypes.c_uint8 * (t * self.k))()
        _check(_lib.lib().rs_encode_matrix(self._ctx, out))
        return [list(out[r * self.k:(r + 1) * self.k]) for r in range(t)]

    def _call(self, op: str, *args) -> int:
        """Per-object entry point rs_<op> (the coalescing service swaps in rs_co_<op>)."""
        return getattr(_lib.lib(), "rs_" + op)(self._ctx, *args)

    # ---- IEcDriver -------------------------------------------------------------
    def Split(self, data: bytes) -> List[bytearray]:
        """[upstream reedsolomon.go Split]: perShard = ceil(len/K); data shards hold
        the payload zero-padded to K*perShard; parity shards are zeroed.  Go's
        aliasing of ``data`` cannot be expressed for Python ``bytes``; the byte
        contents are identical."""
        if len(data) == 0:
            raise ECError(ErrShortData)
        S = int(_lib.lib().rs_shard_size(self._ctx, len(data)))
        padded = bytes(data) + bytes(self.k * S - len(data))
        out = [bytearray(padded[i * S:(i + 1) * S]) for i in range(self.k)]
        out += [bytearray(S) for _ in range(self.m)]
        return out

    def Encode(self, shards: List[Optional[bytearray]]) -> None:
        if len(shards) != self.k + self.m:
            raise ECError(ErrTooFewShards)
        ptrs, lens, keep = _shard_array(shards, 0, fill_missing=False)
        _check(self._call("encode", ptrs, lens))
        del keep

    def _reconstruct(self, shards: List[Optional[bytearray]], data_only: bool) -> None:
        if len(shards) != self.k + self.m:
            raise ECError(ErrTooFewShards)
        S = next((len(s) for s in shards if s is not None and len(s) > 0), 0)
        ptrs, lens, keep = _shard_array(shards, S, fill_missing=True)
        _check(self._call("reconstruct_data" if data_only else "reconstruct", ptrs, lens))
        for i, sh in enumerate(shards):
            if (sh is None or len(sh) == 0) and lens[i] == S and S > 0:
                shards[i] = bytearray(ctypes.string_at(ptrs[i], S))
        del keep

    def Reconstruct(self, shards: List[Optional[bytearray]]) -> None:
        """Fills every nil/empty entry (data and parity), as readservice.go:285 and
        poller.go:282 rely on."""
        self._reconstruct(shards, data_only=False)

    def ReconstructData(self, shards: List[Optional[bytearray]]) -> None:
        self._reconstruct(shards, data_only=True)

    def NewArena(self, size: int) -> "Arena":
        """Page-locked memory for in-place calls (the Go shim's NewArena)."""
        return Arena(self, size)

    def Verify(self, shards: List[bytearray]) -> bool:
        if len(shards) != self.k + self.m:
            raise ECError(ErrTooFewShards)
        ptrs, lens, keep = _shard_array(shards, 0, fill_missing=False)
        ok = ctypes.c_int(0)
        _check(self._call("verify", ptrs, lens, ctypes.byref(ok)))
        del keep
        return bool(ok.value)


class Arena:
    """The Go shim's Arena (ec_gpu.go): page-locked memory the context owns
    (rs_host_alloc).  Alloc(n) hands out writable memoryviews, 16-B aligned; a
    coalesced call whose shards all come from an arena runs in place on the GPU (no
    staging copies, parity written straight into the views).  A bump allocator:
    Alloc until full, Reset when no view is in use, Close to free.

    Reset and Close release every memoryview handed out, so a stale view raises
    ValueError instead of touching reused or freed memory.  Objects the caller built
    ON a view (numpy.frombuffer(view), ctypes from_buffer, ...) take their own
    reference to the memory that no Python API lets the arena see or revoke: drop
    them before Reset / Close, as the Go shim's callers drop their slices."""

    def __init__(self, svc: "Service", size: int):
        n = (size + 4095) // 4096 * 4096
        p = ctypes.c_void_p()
        _check(_lib.lib().rs_host_alloc(svc.ctx, n, ctypes.byref(p)))
        self._svc, self._base, self._size, self._off = svc, p.value, n, 0
        self._mem = (ctypes.c_uint8 * n).from_address(p.value)
        self._root: Optional[memoryview] = memoryview(self._mem).cast("B")  # one per arena
        self._views: List[memoryview] = []  # the slices handed out since the last Reset
        svc._arenas.add(self)

    def Alloc(self, n: int) -> Optional[memoryview]:
        off = (self._off + 15) // 16 * 16
        if n <= 0 or self._base is None or off + n > self._size:
            return None
        self._off = off + n
        v = self._root[off:off + n]
        self._views.append(v)
        return v

    def Reset(self) -> None:
        """Makes the whole arena free again (no view may be in use): the views handed
        out so far are released."""
        self._release_views()
        self._off = 0

    def _release_views(self) -> None:
        for v in self._views:
            try:
                v.release()
            except BufferError:  # a live PEP 3118 export of the view itself: cannot be revoked
                pass
        self._views = []

    def _invalidate(self) -> None:
        """The memory is about to be freed: every view handed out is released (using
        one afterwards raises ValueError instead of touching freed memory) and Alloc
        returns None."""
        self._release_views()
        if self._root is not None:
            try:
                self._root.release()
            except BufferError:
                pass
        self._base, self._mem, self._root = None, None, None

    def Close(self) -> None:
        """Frees the memory (no view may be in use); after the service closed,
        rs_destroy has freed it already."""
        if self._base is not None and self._svc.ctx:
            base = self._base
            self._invalidate()
            _check(_lib.lib().rs_host_free(self._svc.ctx, base))
        self._invalidate()


def NewService(k: int = K, m: int = M, device: Union[int, str, Sequence[int]] = 0) -> Service:
    """internal/ec/ec.go:21 NewService(): RS(K=4, M=2) on the GPU engine
    (device="all": one driver over every GPU of the node, as the Go shim builds it)."""
    return Service(k, m, device)
