"""Shards of 2 GiB and more (the kernels' dropped-store descriptors span
2 GiB from a shard base, so a single launch could silently drop stores past it).
The reference passes whole objects to Split/Encode (writeservice.go:218-222): an
8 GiB object at RS(4+2) has 2 GiB shards.  launch_apply runs such shards as 1 GiB
column windows; RS is column-wise, so any column slice of the data shards encodes
to the same column slice of the parity, which the oracle checks around every
window boundary and at the partial last column."""
import numpy as np
import pytest

from oracle import rs_oracle
from replication_erasurecoding_object_store_amd.batch import BatchEngine, shard_pitch_for

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(300)]


def _oracle_cols(k, m, data_cols):
    """parity of a [k, n] column slice."""
    n = data_cols.shape[1]
    buf = np.zeros((1, k + m, n), np.uint8)
    buf[0, :k] = data_cols
    rs_oracle.encode_batch_scalar(k, m, buf.reshape(-1), (k + m) * n, n, n, 1)
    return buf[0, k:]


def test_encode_and_reconstruct_past_2GiB_shards(gpu):
    import torch

    k, m = 4, 2
    S = (1 << 31) + 4096 + 5  # past 2 GiB, partial last column
    P = shard_pitch_for(S)
    eng = BatchEngine(k, m, 0)
    try:
        g = torch.Generator(device="cuda").manual_seed(0x5EED0042)
        data = torch.randint(0, 256, (1, k, P), dtype=torch.uint8, device="cuda", generator=g)
        parity = torch.full((1, m, P), 0xC3, dtype=torch.uint8, device="cuda")
        eng.encode(data, parity, S, 1)
        torch.cuda.synchronize()
        assert (parity[0, :, S:] == 0xC3).all(), "nothing written past S"
        W = 1 << 30
        windows = [(0, 64), (W - 48, W + 48), (2 * W - 48, 2 * W + 48), (S - 70, S)]
        for lo, hi in windows:
            want = _oracle_cols(k, m, data[0, :, lo:hi].cpu().numpy())
            assert np.array_equal(parity[0, :, lo:hi].cpu().numpy(), want), (lo, hi)
        # 2-erasure reconstruct, out of place: data shard 1 and parity shard 5 lost
        out = torch.full((1, m, P), 0xC3, dtype=torch.uint8, device="cuda")
        eng.reconstruct_out(data, parity, out, S, 1, present_masks=0b011101)
        torch.cuda.synchronize()
        for lo, hi in windows:
            assert torch.equal(out[0, 0, lo:hi], data[0, 1, lo:hi]), (lo, hi)
            assert torch.equal(out[0, 1, lo:hi], parity[0, 1, lo:hi]), (lo, hi)
        assert torch.equal(out[0, 0, :S], data[0, 1, :S]) and torch.equal(out[0, 1, :S], parity[0, 1, :S])
        assert (out[0, :, min(P, (S + 127) // 128 * 128):] == 0xC3).all()  # rows end on whole lines
    finally:
        eng.close()


def test_plane_major_pitch_past_4GiB_unbounded_reconstruct(gpu):
    """the E = m per-stripe kernel loads each input through a buffer
    descriptor over its slot, whose range once came from the shard pitch truncated to
    32 bits -- a pitch of 4 GiB or more wrapped, and the loads past the wrapped range
    read zeros.  Plane-major layout (shard s of every stripe in its own plane), shard
    pitch 4 GiB + 4 KiB, device masks without a bound (apply_kernel<6,3,3,true>), two
    stripes; bytes vs the oracle.  ~36 GiB of device memory, mostly untouched."""
    import torch

    if torch.cuda.get_device_properties(0).total_memory < (64 << 30):
        pytest.skip("needs a 64 GiB+ GPU")
    k, m, S, N = 6, 3, 4096, 2
    P = (1 << 32) + 4096  # shard pitch past 32 bits
    sp = S  # stripe pitch inside a plane
    eng = BatchEngine(k, m, 0)
    try:
        data = torch.empty((k - 1) * P + N * sp, dtype=torch.uint8, device="cuda")
        parity = torch.empty((m - 1) * P + N * sp, dtype=torch.uint8, device="cuda")
        out = torch.full(((m - 1) * P + N * sp,), 0xC3, dtype=torch.uint8, device="cuda")
        rng = np.random.default_rng(44)
        host = rng.integers(0, 256, (N, k, S), dtype=np.uint8)
        for i in range(N):
            for s in range(k):
                data[s * P + i * sp: s * P + i * sp + S] = torch.from_numpy(host[i, s]).cuda()
        eng.encode(data, parity, S, N, shard_pitch=P, data_stripe_pitch=sp, parity_stripe_pitch=sp)
        torch.cuda.synchronize()
        want = np.zeros((N, k + m, S), np.uint8)
        want[:, :k] = host
        rs_oracle.encode_batch_scalar(k, m, want.reshape(-1), (k + m) * S, S, S, N)
        for i in range(N):
            for p in range(m):
                got = parity[p * P + i * sp: p * P + i * sp + S].cpu().numpy()
                assert np.array_equal(got, want[i, k + p]), ("encode", i, p)
        # stripe 0 misses data 0, 1 and parity 2; stripe 1 misses data 5
        full = (1 << (k + m)) - 1
        masks = np.array([full & ~0b100000011, full & ~0b000100000], np.uint32)
        from replication_erasurecoding_object_store_amd import _lib
        from replication_erasurecoding_object_store_amd.batch import _check

        md = torch.from_numpy(masks.view(np.int32)).cuda()
        _check(_lib.lib().rs_reconstruct_batch_out(eng.ctx, data.data_ptr(), sp, parity.data_ptr(), sp, P, S, N,
                                                   md.data_ptr(), N, 1, out.data_ptr(), sp, None))
        eng.sync()
        assert "apply_kernel<6,3,3,true>" in eng.last_kernel(), eng.last_kernel()
        for i in range(N):
            miss = [j for j in range(k + m) if not (masks[i] >> j) & 1]
            for r, j in enumerate(miss):
                got = out[r * P + i * sp: r * P + i * sp + S].cpu().numpy()
                assert np.array_equal(got, want[i, j]), ("reconstruct", i, r, j)
    finally:
        eng.close()
