"""Batched SHA-256 (rs_sha256_batch / _var) vs the FIPS 180-4 oracle and hashlib.

Reference: writeservice.go:51-54 computeSHA256Hex = hex(crypto/sha256.Sum256(value)),
the "cold_hash" stored per EC write (:267) and compared to skip re-encoding (:326).
"""
import hashlib

import numpy as np
import pytest

from oracle import rs_oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng(gpu):
    from replication_erasurecoding_object_store_amd.batch import BatchEngine

    e = BatchEngine(4, 2, 0)
    yield e
    e.close()


LENS = [0, 1, 3, 4, 55, 56, 57, 63, 64, 65, 119, 120, 128, 1000, 1024, 4096, 65537]


@pytest.mark.parametrize("length", LENS)
@pytest.mark.parametrize("pad", [0, 3, 16])
def test_sha256_uniform_matches_oracle(eng, length, pad):
    import torch

    n = 97
    stride = length + pad  # pad 3: every other message starts unaligned
    rng = np.random.default_rng(length * 7 + pad)
    host = rng.integers(0, 256, max(1, n * stride + 8), dtype=np.uint8)
    dev = torch.from_numpy(host).cuda()
    d = eng.sha256(dev, length, n, stride=stride)
    torch.cuda.synchronize()
    got = d.cpu().numpy()
    ref = rs_oracle.sha256_batch(host, stride, n, length=length)
    assert np.array_equal(got, ref)
    for i in (0, n // 2, n - 1):
        assert got[i].tobytes() == hashlib.sha256(host[i * stride:i * stride + length].tobytes()).digest()
    assert eng.last_kernel() == "sha256_kernel"


def test_sha256_fips_vectors(eng):
    import torch

    vectors = [  # FIPS 180-2 Appendix B
        (b"abc", "ba7816bf8f01cfea414140de5dae2223b00361a396177a9cb410ff61f20015ad"),
        (b"", "e3b0c44298fc1c149afbf4c8996fb92427ae41e4649b934ca495991b7852b855"),
        (b"abcdbcdecdefdefgefghfghighijhijkijkljklmklmnlmnomnopnopq",
         "248d6a61d20638b8e5c026930c3e6039a33ce45964ff2167f6ecedd419db06c1"),
    ]
    for msg, hexd in vectors:
        dev = torch.tensor(list(msg) or [0], dtype=torch.uint8, device="cuda")
        d = eng.sha256(dev, len(msg), 1)
        torch.cuda.synchronize()
        assert d.cpu().numpy()[0].tobytes().hex() == hexd


def test_sha256_variable_lengths_and_offsets(eng):
    import torch

    rng = np.random.default_rng(11)
    n = 2000
    lens = rng.integers(0, 5000, n).astype(np.uint64)
    lens[:20] = [0, 1, 55, 56, 63, 64, 65, 119, 120, 127, 128, 129, 4096, 4095, 4097, 8, 9, 10, 11, 12]
    offsets = np.zeros(n, np.uint64)
    pos = 0
    for i in range(n):
        pos += int(rng.integers(0, 5))  # arbitrary (often unaligned) starts
        offsets[i] = pos
        pos += int(lens[i])
    host = rng.integers(0, 256, pos + 1, dtype=np.uint8)
    d = eng.sha256_var(torch.from_numpy(host).cuda(), torch.from_numpy(offsets.view(np.int64)).cuda(),
                       torch.from_numpy(lens.view(np.int64)).cuda())
    torch.cuda.synchronize()
    got = d.cpu().numpy()
    for i in range(n):
        o, ln = int(offsets[i]), int(lens[i])
        assert got[i].tobytes() == hashlib.sha256(host[o:o + ln].tobytes()).digest(), i


def test_sha256_config2_batch_and_split_view(eng):
    """65 536 x 4 KiB objects (config 2).  A value's K data shards are contiguous
    in the split layout when P == S, so the object hash runs on the encode input."""
    import torch

    from replication_erasurecoding_object_store_amd.batch import shard_pitch_for

    N, k, S = 65536, 4, 1024
    P = shard_pitch_for(S)
    assert P == S
    g = torch.Generator(device="cuda").manual_seed(0x5EED0002)
    data = torch.randint(0, 256, (N, k, P), dtype=torch.uint8, device="cuda", generator=g)
    d = eng.sha256(data, k * S, N, stride=k * P)
    torch.cuda.synchronize()
    got = d.cpu().numpy()
    host = data.cpu().numpy().reshape(N, -1)
    for i in np.random.default_rng(1).choice(N, 300, replace=False):
        assert got[i].tobytes() == hashlib.sha256(host[i].tobytes()).digest()
