"""Every batched kernel family against the CPU oracle, in one process.

rs_set_kernel_variant selects the family the specialised shapes launch:
  1  grid-stride apply_kernel + bitsliced encode (the default)
  2  pipe_kernel, one wave per SIMD, 2 task slots per wave
  3  pipe_kernel, 3 task slots
  4  grid-stride apply_kernel for encode too (no bitsliced program)
Each must give the oracle's bytes for encode, uniform reconstruct, per-stripe
reconstruct (host and device masks) and out-of-place reconstruct, with the slot
padding untouched, on the BASELINE shapes and a tail length (S % 16 != 0).
"""
import numpy as np
import pytest

from oracle import rs_oracle
from replication_erasurecoding_object_store_amd.batch import BatchEngine, shard_pitch_for

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engines(gpu):
    es = {}
    yield es
    for e in es.values():
        e.close()


def _masks(rng, N, t, m):
    masks = np.full(N, (1 << t) - 1, np.uint32)
    for i in range(N):
        for j in rng.choice(t, size=rng.integers(0, m + 1), replace=False):
            masks[i] &= ~np.uint32(1 << int(j))
    return masks


@pytest.mark.parametrize("variant", [1, 2, 3, 4])
@pytest.mark.parametrize("k,m,S", [(4, 2, 1024), (8, 4, 8192), (10, 4, 6554), (10, 4, 413), (6, 3, 1000)])
def test_variant_matches_oracle(engines, variant, k, m, S):
    import torch

    if (k, m) not in engines:
        engines[(k, m)] = BatchEngine(k, m, 0)
    eng = engines[(k, m)]
    eng.set_kernel_variant(variant)
    try:
        t, N, P = k + m, 300, shard_pitch_for(S)
        g = torch.Generator(device="cuda").manual_seed(variant * 1000 + k * 31 + S)
        data = torch.randint(0, 256, (N, k, P), dtype=torch.uint8, device="cuda", generator=g)
        parity = torch.full((N, m, P), 0xEE, dtype=torch.uint8, device="cuda")
        eng.encode(data, parity, S, N)
        torch.cuda.synchronize()
        uni = np.zeros((N, t, P), np.uint8)
        uni[:, :k] = data.cpu().numpy()
        rs_oracle.encode_batch_scalar(k, m, uni.reshape(-1), t * P, P, S, N)
        par = parity.cpu().numpy()
        assert np.array_equal(par[:, :, :S], uni[:, k:, :S]), "encode != oracle"
        assert (par[:, :, S:] == 0xEE).all(), "slot padding written"

        rng = np.random.default_rng(variant + S)
        # uniform pattern (two shards, one data one parity), in place
        one = np.uint32(((1 << t) - 1) & ~((1 << 1) | (1 << k)))
        d2, p2 = data.clone(), parity.clone()
        d2[:, 1, :S] = 0x33
        p2[:, 0, :S] = 0x33
        eng.reconstruct(d2, p2, S, N, one)
        torch.cuda.synchronize()
        assert torch.equal(d2[:, :, :S], data[:, :, :S]) and torch.equal(p2[:, :, :S], parity[:, :, :S])

        # per-stripe patterns, 0..m erasures: host masks then device masks, in place
        for use_dev in (False, True):
            masks = _masks(rng, N, t, m)
            lost = ((masks[:, None] >> np.arange(t)[None, :]) & 1) == 0
            d2, p2 = data.clone(), parity.clone()
            d2[:, :, :S][torch.from_numpy(lost[:, :k]).cuda()] = 0x33
            p2[:, :, :S][torch.from_numpy(lost[:, k:]).cuda()] = 0x33
            if use_dev:
                eng.reconstruct_devmask(d2, p2, S, N, torch.from_numpy(masks.view(np.int32)).cuda())
                eng.sync()
            else:
                eng.reconstruct(d2, p2, S, N, masks)
            torch.cuda.synchronize()
            assert torch.equal(d2[:, :, :S], data[:, :, :S]), (variant, use_dev)
            assert torch.equal(p2[:, :, :S], parity[:, :, :S]), (variant, use_dev)

        # out of place, device masks: the r-th missing shard at out[i, r]
        masks = _masks(rng, N, t, m)
        out = torch.full((N, m, P), 0xC3, dtype=torch.uint8, device="cuda")
        eng.reconstruct_out(data, parity, out, S, N, masks_dev=torch.from_numpy(masks.view(np.int32)).cuda())
        eng.sync()
        o = out.cpu().numpy()
        for i in range(N):
            miss = [s for s in range(t) if not (masks[i] >> s) & 1]
            for r, s in enumerate(miss):
                assert np.array_equal(o[i, r, :S], uni[i, s, :S]), (variant, i, s)
            assert (o[i, len(miss):] == 0xC3).all() and (o[i, :, S:] == 0xC3).all()
    finally:
        eng.set_kernel_variant(0)
