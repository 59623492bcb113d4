"""xoshiro256** byte streams for the seeded inputs of BASELINE.json's configs.

SURVEY.md 8d fixes the inputs as uniform random bytes from xoshiro256** with
per-config seeds (0x5EED0001 for the 1 MiB object, 0x5EED0002 for the 4 KiB
stripe batch, ...).  State is seeded with splitmix64(seed) x4; output words are
emitted little-endian.  Pure Python (about 1 M words/s): used for fixtures and
for the small/medium configs; the multi-GiB bench batches use on-device torch
RNG instead (bench.py says so in its "data" field).
"""
from __future__ import annotations

MASK = (1 << 64) - 1


def _rotl(x: int, k: int) -> int:
    return ((x << k) | (x >> (64 - k))) & MASK


def _splitmix64(state: int):
    while True:
        state = (state + 0x9E3779B97F4A7C15) & MASK
        z = state
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & MASK
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & MASK
        yield z ^ (z >> 31)


def xoshiro_bytes(seed: int, n: int) -> bytes:
    sm = _splitmix64(seed)
    s0, s1, s2, s3 = next(sm), next(sm), next(sm), next(sm)
    words = []
    for _ in range((n + 7) // 8):
        result = (_rotl((s1 * 5) & MASK, 7) * 9) & MASK
        t = (s1 << 17) & MASK
        s2 ^= s0
        s3 ^= s1
        s1 ^= s2
        s0 ^= s3
        s2 ^= t
        s3 = _rotl(s3, 45)
        words.append(result)
    out = b"".join(w.to_bytes(8, "little") for w in words)
    return out[:n]
