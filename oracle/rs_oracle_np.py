"""Independent numpy restatement of the reference codec (second oracle).

TEST INFRASTRUCTURE ONLY.  Written separately from rs_oracle.c (different table
construction, Gaussian elimination written over numpy rows) so that the two
restatements cross-check each other; both are pinned on the known-answer tests of
klauspost/reedsolomon v1.12.1 (the library internal/ec/ec.go:26 wraps).
"""
from __future__ import annotations

from typing import List, Optional

import numpy as np

POLY = 0x11D


def _tables():
    exp = np.zeros(512, np.int64)
    log = np.zeros(256, np.int64)
    x = 1
    for i in range(255):
        exp[i] = x
        log[x] = i
        x <<= 1
        if x & 0x100:
            x ^= POLY
    exp[255:510] = exp[0:255]
    return exp, log


EXP, LOG = _tables()
# full 256x256 product table [upstream galois.go mulTable]
MUL = np.zeros((256, 256), np.uint8)
_nz = np.arange(1, 256)
MUL[1:, 1:] = EXP[(LOG[_nz][:, None] + LOG[_nz][None, :])].astype(np.uint8)


def gf_exp(a: int, n: int) -> int:
    if n == 0:
        return 1
    if a == 0:
        return 0
    return int(EXP[(int(LOG[a]) * n) % 255])


def gf_inv(a: int) -> int:
    return int(EXP[(255 - LOG[a]) % 255])


def matmul(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    out = np.zeros((a.shape[0], b.shape[1]), np.uint8)
    for i in range(a.shape[1]):
        out ^= MUL[a[:, i][:, None], b[i, :][None, :]]
    return out


def invert(a: np.ndarray) -> np.ndarray:
    n = a.shape[0]
    w = np.concatenate([a.astype(np.uint8), np.eye(n, dtype=np.uint8)], axis=1)
    for col in range(n):
        nz = np.nonzero(w[col:, col])[0]
        if len(nz) == 0:
            raise ValueError("matrix is singular")
        p = col + int(nz[0])
        if p != col:
            w[[col, p]] = w[[p, col]]
        w[col] = MUL[gf_inv(int(w[col, col])), w[col]]
        for r in range(n):
            if r != col and w[r, col]:
                w[r] ^= MUL[int(w[r, col]), w[col]]
    return w[:, n:].copy()


def build_matrix(k: int, m: int) -> np.ndarray:
    v = np.array([[gf_exp(r, c) for c in range(k)] for r in range(k + m)], np.uint8)
    return matmul(v, invert(v[:k]))


def apply(rows: np.ndarray, inputs: np.ndarray) -> np.ndarray:
    """rows: e x k coefficients, inputs: k x S bytes -> e x S."""
    out = np.zeros((rows.shape[0], inputs.shape[1]), np.uint8)
    for c in range(rows.shape[1]):
        out ^= MUL[rows[:, c][:, None], inputs[c][None, :]]
    return out


def encode(k: int, m: int, data: np.ndarray) -> np.ndarray:
    """data: k x S -> parity m x S."""
    return apply(build_matrix(k, m)[k:], data)


def reconstruct(k: int, m: int, shards: List[Optional[np.ndarray]]) -> List[np.ndarray]:
    """Two-phase reconstruct like [upstream reedsolomon.go reconstruct]."""
    mat = build_matrix(k, m)
    present = [i for i, s in enumerate(shards) if s is not None and len(s) > 0]
    if len(present) < k:
        raise ValueError("too few shards given")
    surv = present[:k]
    dec = invert(mat[surv])
    sub = np.stack([shards[i] for i in surv])
    out = list(shards)
    for i in range(k):
        if out[i] is None or len(out[i]) == 0:
            out[i] = apply(dec[i:i + 1], sub)[0]
    data = np.stack(out[:k])
    for p in range(k, k + m):
        if out[p] is None or len(out[p]) == 0:
            out[p] = apply(mat[p:p + 1], data)[0]
    return out
