"""ctypes front-end for the C oracle (oracle/librs_oracle.so).

TEST INFRASTRUCTURE ONLY -- only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may import this module.  The product package never does.

Parity status: pinned on the published known-answer tests of the codec the
reference wraps (klauspost/reedsolomon v1.12.1: galois_test.go, TestOneEncode;
reproduced in SURVEY.md Appendix A) and on an independent numpy restatement
(oracle/rs_oracle_np.py).  The reference's own tests pin no RS bytes
(SURVEY.md 8c), and its Go path cannot be built here (no Go toolchain).
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from typing import List, Optional, Sequence, Tuple

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "librs_oracle.so")

_u8p = ctypes.POINTER(ctypes.c_uint8)
_lib = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        L.rso_gf_mul.restype = ctypes.c_uint8
        L.rso_gf_exp.restype = ctypes.c_uint8
        L.rso_gf_inv.restype = ctypes.c_uint8
        L.rso_shard_size.restype = ctypes.c_size_t
        L.rso_shard_size.argtypes = [ctypes.c_int, ctypes.c_size_t]
        L.rso_encode_batch_scalar.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t,
                                              ctypes.c_size_t, ctypes.c_size_t, ctypes.c_size_t]
        L.rso_sha256.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
        L.rso_sha256_batch.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t,
                                       ctypes.c_size_t, ctypes.c_void_p]
        L.rso_baseline_sha256_batch.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_size_t,
                                                ctypes.c_void_p, ctypes.c_int]
        L.rso_baseline_apply_batch.argtypes = [
            ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
            ctypes.c_size_t, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_int]
        _lib = L
    return _lib


def gf_mul(a: int, b: int) -> int:
    return lib().rso_gf_mul(a, b)


def gf_exp(a: int, n: int) -> int:
    return lib().rso_gf_exp(a, n)


def build_matrix(k: int, m: int) -> np.ndarray:
    out = (ctypes.c_uint8 * ((k + m) * k))()
    rc = lib().rso_build_matrix(k, m, out)
    if rc:
        raise ValueError(f"rso_build_matrix rc={rc}")
    return np.frombuffer(bytes(out), np.uint8).reshape(k + m, k).copy()


def decode_rows(k: int, m: int, present: Sequence[int]) -> Tuple[List[int], List[int], np.ndarray]:
    t = k + m
    pres = (ctypes.c_uint8 * t)(*[1 if p else 0 for p in present])
    surv = (ctypes.c_int * k)()
    miss = (ctypes.c_int * t)()
    nm = ctypes.c_int(0)
    rows = (ctypes.c_uint8 * (t * k))()
    rc = lib().rso_decode_rows(k, m, pres, surv, miss, ctypes.byref(nm), rows)
    if rc:
        raise ValueError(f"rso_decode_rows rc={rc}")
    n = nm.value
    return list(surv), list(miss[:n]), np.frombuffer(bytes(rows), np.uint8)[: n * k].reshape(n, k).copy()


def _ptrs(shards: List[bytearray], S: int):
    n = len(shards)
    ptrs = (_u8p * n)()
    lens = (ctypes.c_size_t * n)()
    keep = []
    for i, sh in enumerate(shards):
        if sh is None or len(sh) == 0:
            buf = (ctypes.c_uint8 * max(S, 1))()
            lens[i] = 0
        else:
            buf = (ctypes.c_uint8 * len(sh)).from_buffer(sh)
            lens[i] = len(sh)
        keep.append(buf)
        ptrs[i] = ctypes.cast(buf, _u8p)
    return ptrs, lens, keep


def split(k: int, m: int, data: bytes) -> List[bytearray]:
    """[upstream reedsolomon.go Split] byte contents."""
    S = lib().rso_shard_size(k, len(data))
    if S == 0:
        raise ValueError("not enough data to fill the number of requested shards")
    padded = bytes(data) + bytes(k * S - len(data))
    return [bytearray(padded[i * S:(i + 1) * S]) for i in range(k)] + [bytearray(S) for _ in range(m)]


def encode(k: int, m: int, shards: List[bytearray]) -> int:
    ptrs, lens, keep = _ptrs(shards, 0)
    return lib().rso_encode(k, m, ptrs, lens)


def reconstruct(k: int, m: int, shards: List[Optional[bytearray]]) -> int:
    S = next((len(s) for s in shards if s is not None and len(s) > 0), 0)
    ptrs, lens, keep = _ptrs(shards, S)
    rc = lib().rso_reconstruct(k, m, ptrs, lens)
    if rc == 0:
        for i, sh in enumerate(shards):
            if (sh is None or len(sh) == 0) and lens[i] == S:
                shards[i] = bytearray(ctypes.string_at(ptrs[i], S))
    return rc


def verify(k: int, m: int, shards: List[bytearray]) -> Tuple[int, bool]:
    ptrs, lens, keep = _ptrs(shards, 0)
    ok = ctypes.c_int(0)
    rc = lib().rso_verify(k, m, ptrs, lens, ctypes.byref(ok))
    return rc, bool(ok.value)


def encode_batch_scalar(k: int, m: int, buf: np.ndarray, stripe_pitch: int, shard_pitch: int, S: int, N: int) -> None:
    """In-place encode of a unified (k+m slots per stripe) host buffer."""
    assert buf.dtype == np.uint8 and buf.flags.c_contiguous
    assert buf.nbytes >= (N - 1) * stripe_pitch + (k + m - 1) * shard_pitch + S
    lib().rso_encode_batch_scalar(k, m, buf.ctypes.data, stripe_pitch, shard_pitch, S, N)


def baseline_apply_batch(k: int, rows: np.ndarray, in_idx: Sequence[int], out_idx: Sequence[int], buf: np.ndarray,
                         stripe_pitch: int, shard_pitch: int, S: int, N: int, threads: int) -> int:
    """SIMD CPU baseline (AVX-512 GFNI / AVX2 split-nibble), returns SIMD level."""
    e = len(out_idx)
    rows = np.ascontiguousarray(rows, np.uint8)
    assert rows.shape == (e, k)
    ii = (ctypes.c_int * k)(*in_idx)
    oo = (ctypes.c_int * max(e, 1))(*out_idx)
    assert buf.nbytes >= (N - 1) * stripe_pitch + (max(max(in_idx), max(out_idx)) * shard_pitch) + S
    return lib().rso_baseline_apply_batch(k, e, rows.ctypes.data, ctypes.cast(ii, ctypes.c_void_p),
                                          ctypes.cast(oo, ctypes.c_void_p), buf.ctypes.data, stripe_pitch,
                                          shard_pitch, S, N, threads)


def sha256(msg: bytes) -> bytes:
    """FIPS 180-4 SHA-256 (writeservice.go:51-54 computeSHA256Hex's Sum256)."""
    buf = (ctypes.c_uint8 * max(1, len(msg))).from_buffer_copy(msg or b"\0")
    out = (ctypes.c_uint8 * 32)()
    lib().rso_sha256(ctypes.cast(buf, ctypes.c_void_p), len(msg), ctypes.cast(out, ctypes.c_void_p))
    return bytes(out)


def sha256_batch(base: np.ndarray, stride: int, n: int, length: int = 0, lens=None) -> np.ndarray:
    """Digests [n, 32] of n messages at base + i*stride (lens[i] or `length` bytes)."""
    out = np.zeros((n, 32), np.uint8)
    lp = None
    if lens is not None:
        lens = np.ascontiguousarray(lens, np.uint64)
        lp = lens.ctypes.data
    lib().rso_sha256_batch(base.ctypes.data, stride, lp, length, n, out.ctypes.data)
    return out


def baseline_sha256_batch(base: np.ndarray, stride: int, length: int, n: int, threads: int):
    """CPU baseline (SHA-NI on `threads` host threads): (digests [n, 32], used_sha_ni)."""
    assert base.nbytes >= (n - 1) * stride + length
    out = np.zeros((n, 32), np.uint8)
    ni = lib().rso_baseline_sha256_batch(base.ctypes.data, stride, length, n, out.ctypes.data, threads)
    return out, bool(ni)
