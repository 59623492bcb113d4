"""Every batched kernel path of each specialised shape against the CPU oracle, in
one process.

The engine picks the kernel by shape and call: bitsliced or lookup encode,
stripe-aligned or flat-task per-stripe reconstruct, uniform-plan reconstruct (slots
resolved once per launch), and for device masks the erasure bound E of the launch
(rs_reconstruct_batch_out_devmask's max_missing; E <= 2 runs the input-outer flat
kernel).  Each must give the oracle's bytes, with slot padding untouched, on the
BASELINE shapes and a tail length (S % 16 != 0).
"""
import numpy as np
import pytest

from oracle import rs_oracle
from replication_erasurecoding_object_store_amd import _lib
from replication_erasurecoding_object_store_amd.batch import BatchEngine, shard_pitch_for
from replication_erasurecoding_object_store_amd.ec import ECError

pytestmark = pytest.mark.gpu

SHAPES = [(4, 2, 1024), (8, 4, 8192), (10, 4, 6554), (10, 4, 413), (6, 3, 1000), (4, 2, 1000), (10, 4, 8192)]


@pytest.fixture(scope="module")
def engines(gpu):
    es = {}
    yield es
    for e in es.values():
        e.close()


def _engine(engines, k, m):
    if (k, m) not in engines:
        engines[(k, m)] = BatchEngine(k, m, 0)
    return engines[(k, m)]


def _masks(rng, N, t, lo, hi):
    """Per-stripe present masks with lo..hi erasures each."""
    masks = np.full(N, (1 << t) - 1, np.uint32)
    for i in range(N):
        for j in rng.choice(t, size=rng.integers(lo, hi + 1), replace=False):
            masks[i] &= ~np.uint32(1 << int(j))
    return masks


def _codewords(eng, k, m, S, N, seed):
    import torch

    t, P = k + m, shard_pitch_for(S)
    g = torch.Generator(device="cuda").manual_seed(seed)
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
    return data, parity, uni


def _pad_end(S, P):
    """First byte of an out-of-place row that is never written: rows end on whole
    128-B lines within their slot (rs_set_out_pad_writes, on in BatchEngine)."""
    return min(P, (S + 127) // 128 * 128)


@pytest.mark.parametrize("k,m,S", SHAPES)
def test_paths_match_oracle(engines, k, m, S):
    import torch

    eng = _engine(engines, k, m)
    t, N, P = k + m, 300, shard_pitch_for(S)
    data, parity, uni = _codewords(eng, k, m, S, N, k * 31 + S)
    rng = np.random.default_rng(S)
    # uniform patterns (slots resolved once per launch), in place: one data + one
    # parity shard, two data shards, the parity shards only
    for lost in ((1, k), (0, 1), tuple(range(k, t))):
        one = np.uint32(((1 << t) - 1) & ~sum(1 << j for j in lost))
        d2, p2 = data.clone(), parity.clone()
        for j in lost:
            (d2[:, j] if j < k else p2[:, j - k])[:, :S] = 0x33
        eng.reconstruct(d2, p2, S, N, one)
        torch.cuda.synchronize()
        assert torch.equal(d2, data) and torch.equal(p2, parity), lost

    # per-stripe patterns, 0..m erasures: host masks then device masks, in place
    for use_dev in (False, True):
        masks = _masks(rng, N, t, 0, m)
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
        assert torch.equal(d2, data), use_dev
        assert torch.equal(p2, parity), use_dev

    # out of place: uniform host mask, then device masks with and without a bound
    for lost in ((0, 1), (1, k)):
        one = ((1 << t) - 1) & ~sum(1 << j for j in lost)
        out = torch.full((N, m, P), 0xC3, dtype=torch.uint8, device="cuda")
        eng.reconstruct_out(data, parity, out, S, N, present_masks=one)
        torch.cuda.synchronize()
        o = out.cpu().numpy()
        for r, s in enumerate(lost):
            assert np.array_equal(o[:, r, :S], uni[:, s, :S]), (lost, s)
        assert (o[:, len(lost):] == 0xC3).all() and (o[:, :, _pad_end(S, P):] == 0xC3).all()
    for bound in (0, 1, 2, m):
        hi = bound or m
        masks = _masks(rng, N, t, 1 if bound == 1 else 0, hi)
        out = torch.full((N, max(hi, 1), P), 0xC3, dtype=torch.uint8, device="cuda")
        eng.reconstruct_out(data, parity, out, S, N, masks_dev=torch.from_numpy(masks.view(np.int32)).cuda(),
                            max_missing=bound)
        eng.sync()
        o = out.cpu().numpy()
        for i in range(N):
            miss = [s for s in range(t) if not (masks[i] >> s) & 1]
            for r, s in enumerate(miss):
                assert np.array_equal(o[i, r, :S], uni[i, s, :S]), (bound, i, s)
            assert (o[i, len(miss):] == 0xC3).all() and (o[i, :, _pad_end(S, P):] == 0xC3).all()


@pytest.mark.parametrize("k,m,S", [(10, 4, 6554), (8, 4, 8192), (4, 2, 1024), (10, 4, 413)])
@pytest.mark.parametrize("bound", [1, 2])
def test_devmask_bound_flags_and_skips_excess(engines, k, m, S, bound):
    """Stripes missing more than max_missing shards are left untouched and reported
    by rs_sync as RS_ERR_INVALID_ARG; every other stripe is still rebuilt; a stripe
    with < k present wins as RS_ERR_TOO_FEW_SHARDS."""
    import torch

    if bound >= m:
        pytest.skip("a stripe beyond a bound of m has fewer than k shards: covered by TOO_FEW_SHARDS")
    eng = _engine(engines, k, m)
    t, N, P = k + m, 257, shard_pitch_for(S)
    data, parity, uni = _codewords(eng, k, m, S, N, 77 + bound)
    rng = np.random.default_rng(bound * 7 + S)
    masks = _masks(rng, N, t, 1, bound)
    over = [5, 64, 65, 200]  # neighbours of straddling flat tasks included
    for i in over:
        masks[i] = ((1 << t) - 1) & ~((1 << (bound + 1)) - 1)  # bound + 1 erasures
    out = torch.full((N, bound, P), 0xC3, dtype=torch.uint8, device="cuda")
    mdev = torch.from_numpy(masks.view(np.int32)).cuda()
    eng.reconstruct_out(data, parity, out, S, N, masks_dev=mdev, max_missing=bound)
    with pytest.raises(ECError) as ei:
        eng.sync()
    assert ei.value.code == _lib.RS_ERR_INVALID_ARG
    eng.sync()  # cleared
    o = out.cpu().numpy()
    for i in range(N):
        if i in over:
            assert (o[i] == 0xC3).all(), i
            continue
        miss = [s for s in range(t) if not (masks[i] >> s) & 1]
        for r, s in enumerate(miss):
            assert np.array_equal(o[i, r, :S], uni[i, s, :S]), (i, s)
    # a stripe with fewer than k present as well: TOO_FEW_SHARDS takes precedence
    masks[9] = (1 << (k - 1)) - 1
    eng.reconstruct_out(data, parity, out, S, N, masks_dev=torch.from_numpy(masks.view(np.int32)).cuda(),
                        max_missing=bound)
    with pytest.raises(ECError) as ei:
        eng.sync()
    assert ei.value.code == _lib.RS_ERR_TOO_FEW_SHARDS
    # the bound is checked against the out layout and m
    with pytest.raises(ECError):
        eng.reconstruct_out(data, parity, out, S, N, masks_dev=mdev, max_missing=-1)


# Sporadic-corruption guard for the output stores: every kernel stores with one
# cache policy (out_cpol); a per-lane mix of policies once returned wrong 64-B
# halves of rows on a few stripes per run (`HISTORY.md` §A.1 / §A.5, profiles/r03n_ab_cpol.log).
# Larger batches than the parity tests, two pattern draws each, every output row
# and every unused output slot compared (vectorised).
@pytest.mark.parametrize("k,m,S,bound", [(8, 4, 6554, 1), (10, 4, 6554, 2), (8, 4, 6554, 4), (8, 4, 8192, 1),
                                         (10, 4, 6554, 1), (8, 4, 8192, 4), (10, 4, 6554, 4), (4, 2, 1024, 2),
                                         (10, 4, 8192, 2), (10, 4, 8192, 4)])
def test_out_of_place_stress(engines, k, m, S, bound):
    import torch

    eng = _engine(engines, k, m)
    t, N, P = k + m, 2049, shard_pitch_for(S)
    g = torch.Generator(device="cuda").manual_seed(S * 7 + bound)
    data = torch.randint(0, 256, (N, k, P), dtype=torch.uint8, device="cuda", generator=g)
    parity = torch.empty((N, m, P), dtype=torch.uint8, device="cuda")
    eng.encode(data, parity, S, N)
    ref = torch.cat([data, parity], dim=1)[:, :, :S].cpu().numpy()  # [N, t, S], checked against the oracle above
    for trial in range(2):
        rng = np.random.default_rng(1000 * trial + S + bound)
        masks = _masks(rng, N, t, 0, bound)
        # expected out[i, r] = shard of the r-th missing index of stripe i
        missing = [[j for j in range(t) if not (int(masks[i]) >> j) & 1] for i in range(N)]
        # dev: the caller's bound (E = bound kernels); devu: no bound, the E = M kernels
        # (slot-descriptor loads, intact stripes and intact halves of straddling tasks
        # fetch nothing, round 4)
        for mode in ("host", "dev", "devu"):
            out = torch.full((N, m, P), 0xC3, dtype=torch.uint8, device="cuda")
            if mode == "host":
                eng.reconstruct_out(data, parity, out, S, N, present_masks=masks)
            else:
                eng.reconstruct_out(data, parity, out, S, N,
                                    masks_dev=torch.from_numpy(masks.view(np.int32)).cuda(),
                                    max_missing=bound if mode == "dev" else 0)
                eng.sync()
            torch.cuda.synchronize()
            got = out.cpu().numpy()
            for r in range(m):
                rows = np.array([i for i in range(N) if len(missing[i]) > r])
                if len(rows):
                    src = np.array([missing[i][r] for i in rows])
                    bad = np.nonzero((got[rows, r, :S] != ref[rows, src]).any(axis=1))[0]
                    assert len(bad) == 0, (mode, trial, r, rows[bad][:8].tolist())
                unused = np.array([i for i in range(N) if len(missing[i]) <= r])
                if len(unused):
                    assert (got[unused, r] == 0xC3).all(), (mode, trial, r, "unused output slot written")
            assert (got[:, :, _pad_end(S, P):] == 0xC3).all(), "output padding past the line written"


@pytest.mark.parametrize("k,m,S,bound", [(10, 4, 6554, 1), (10, 4, 6554, 2), (10, 4, 6554, 0), (8, 4, 8192, 2),
                                         (4, 2, 1000, 1), (6, 3, 413, 0)])
def test_out_pad_writes(engines, k, m, S, bound):
    """rs_set_out_pad_writes: every output row written keeps bytes [0, S) exact and
    may fill its padding up to the next 128-B line; bytes past that line and rows a
    stripe does not miss stay untouched.  Device masks, with the caller's bound and
    without (bound 0 -> E = M)."""
    import torch

    eng = _engine(engines, k, m)
    t, N = k + m, 777
    P = shard_pitch_for(S) + 256  # room past the 128-B line
    g = torch.Generator(device="cuda").manual_seed(S + k)
    data = torch.randint(0, 256, (N, k, P), dtype=torch.uint8, device="cuda", generator=g)
    parity = torch.empty((N, m, P), dtype=torch.uint8, device="cuda")
    eng.encode(data, parity, S, N)
    full = torch.cat([data, parity], dim=1).cpu().numpy()
    rng = np.random.default_rng(S * 7 + bound)
    masks = _masks(rng, N, t, 1, bound or m)
    rows = bound or m
    out = torch.full((N, rows, P), 0xC3, dtype=torch.uint8, device="cuda")
    mdev = torch.from_numpy(masks.view(np.int32)).cuda()
    eng.reconstruct_out(data, parity, out, S, N, masks_dev=mdev, max_missing=bound, shard_pitch=P)  # BatchEngine: on
    eng.sync()
    got = out.cpu().numpy()
    line_end = min(P, (S + 127) // 128 * 128)
    for i in range(N):
        missing = [j for j in range(t) if not (masks[i] >> j) & 1]
        for r, j in enumerate(missing):
            assert np.array_equal(got[i, r, :S], full[i, j, :S]), (i, r, j)
            assert (got[i, r, line_end:] == 0xC3).all(), ("past the line", i, r)
        assert (got[i, len(missing):] == 0xC3).all(), ("unused rows", i)
    # rs_set_out_pad_writes(0): exact rows, nothing past S
    out.fill_(0xC3)
    eng.set_out_pad_writes(False)
    try:
        eng.reconstruct_out(data, parity, out, S, N, masks_dev=mdev, max_missing=bound, shard_pitch=P)
        eng.sync()
    finally:
        eng.set_out_pad_writes(True)
    got = out.cpu().numpy()
    for i in range(N):
        missing = [j for j in range(t) if not (masks[i] >> j) & 1]
        for r, j in enumerate(missing):
            assert np.array_equal(got[i, r, :S], full[i, j, :S]), (i, r, j)
    assert (got[:, :, S:] == 0xC3).all(), "exact mode wrote past S"


@pytest.mark.parametrize("k,m,S", [(10, 4, 6554), (4, 2, 1000), (8, 4, 8200)])
def test_out_pad_never_crosses_a_stripe_slot(engines, k, m, S):
    """Dense 1-row outputs (bound 1, out stripe pitch = round_up(S, 16), below the
    128-B line end): whole-line rows would overwrite the next stripe's row, so the
    engine writes them exactly (the guard in launch()) -- with BatchEngine's padding on."""
    import torch

    eng = _engine(engines, k, m)
    t, N = k + m, 300
    P = shard_pitch_for(S)
    g = torch.Generator(device="cuda").manual_seed(S)
    data = torch.randint(0, 256, (N, k, P), dtype=torch.uint8, device="cuda", generator=g)
    parity = torch.empty((N, m, P), dtype=torch.uint8, device="cuda")
    eng.encode(data, parity, S, N)
    full = torch.cat([data, parity], dim=1)[:, :, :S].cpu().numpy()
    out_sp = (S + 15) // 16 * 16
    assert out_sp < (S + 127) // 128 * 128
    out = torch.full((N + 1, out_sp), 0xC3, dtype=torch.uint8, device="cuda")
    rng = np.random.default_rng(S)
    masks = _masks(rng, N, t, 1, 1)
    eng.reconstruct_out(data, parity, out[:N].view(N, 1, out_sp), S, N,
                        masks_dev=torch.from_numpy(masks.view(np.int32)).cuda(), max_missing=1, shard_pitch=P)
    eng.sync()
    got = out.cpu().numpy()
    for i in range(N):
        j = [s for s in range(t) if not (masks[i] >> s) & 1][0]
        assert np.array_equal(got[i, :S], full[i, j]), (i, j)
    assert (got[:N, S:] == 0xC3).all(), "a row's padding reached into the next stripe's row"
    assert (got[N] == 0xC3).all()


@pytest.mark.parametrize("k,m,S,bound", [(10, 4, 6554, 2), (10, 4, 6554, 0), (4, 2, 1000, 2), (8, 4, 8200, 1)])
def test_c_abi_default_rows_end_at_byte_s(k, m, S, bound):
    """a C / Go caller gets exact rows by default.  A context made
    through the plain C-ABI (no BatchEngine opt-in) writes no byte past S of any
    output row, so an output buffer that ends exactly at the last row's byte S --
    (N-1)*out_sp + (e-1)*pitch + S -- is enough: the bytes after it keep their
    sentinel, and every row equals the erased shard."""
    import ctypes

    import torch

    from replication_erasurecoding_object_store_amd.ec import Service

    svc = Service(k, m, 0)  # rs_create: the library's defaults
    try:
        t, N = k + m, 257
        P = shard_pitch_for(S)
        e = bound or m
        g = torch.Generator(device="cuda").manual_seed(S + 11)
        data = torch.randint(0, 256, (N, k, P), dtype=torch.uint8, device="cuda", generator=g)
        parity = torch.empty((N, m, P), dtype=torch.uint8, device="cuda")
        L = _lib.lib()
        st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        assert L.rs_encode_batch(svc.ctx, data.data_ptr(), k * P, parity.data_ptr(), m * P, P, S, N,
                                 _lib.RS_MEM_DEVICE, st) == 0
        full = torch.cat([data, parity], dim=1)[:, :, :S].cpu().numpy()
        rng = np.random.default_rng(S + bound)
        masks = _masks(rng, N, t, e, e)  # every stripe misses e shards: the last row is row e-1
        out_sp = e * P
        need = (N - 1) * out_sp + (e - 1) * P + S
        guard = 4096
        buf = torch.full((need + guard,), 0xC3, dtype=torch.uint8, device="cuda")
        mdev = torch.from_numpy(masks.view(np.int32)).cuda()
        assert L.rs_reconstruct_batch_out_devmask(svc.ctx, data.data_ptr(), k * P, parity.data_ptr(), m * P, P, S,
                                                  N, mdev.data_ptr(), bound, buf.data_ptr(), out_sp, st) == 0
        assert L.rs_sync(svc.ctx, st) == 0
        got = buf.cpu().numpy()
        assert (got[need:] == 0xC3).all(), "a byte past the last row's byte S was written"
        for i in range(N):
            missing = [j for j in range(t) if not (masks[i] >> j) & 1]
            for r, j in enumerate(missing):
                o = i * out_sp + r * P
                assert np.array_equal(got[o:o + S], full[i, j]), (i, r, j)
                if o + S < need:
                    assert (got[o + S:min(o + P, need)] == 0xC3).all(), ("row padding written", i, r)
    finally:
        svc.close()


@pytest.mark.parametrize("k,m,S,N", [(10, 4, 6554, 2049), (8, 4, 8192, 2049), (4, 2, 1024, 2049), (10, 4, 413, 2049),
                                     (6, 3, 1000, 777), (4, 2, 16384, 1025), (4, 2, 100, 40000)])
@pytest.mark.parametrize("where", ["dev", "host"])
def test_packed_rows_match_oracle(engines, k, m, S, N, where):
    """rs_reconstruct_batch_out_packed: stripes missing 0..m shards (scan batches);
    row_offsets = the exclusive prefix sum of the erasure counts (stripes with < k
    present take none), stripe i's r-th missing shard at row row_offsets[i] + r,
    equal to the encoded shard; bytes past each row's 128-B line and rows past the
    total stay untouched.  N = 40000 walks the scan kernel's 16384-mask chunks."""
    import torch

    eng = _engine(engines, k, m)
    t, P = k + m, shard_pitch_for(S)
    g = torch.Generator(device="cuda").manual_seed(S * 3 + N)
    data = torch.randint(0, 256, (N, k, P), dtype=torch.uint8, device="cuda", generator=g)
    parity = torch.empty((N, m, P), dtype=torch.uint8, device="cuda")
    eng.encode(data, parity, S, N)
    ref = torch.cat([data, parity], dim=1)[:, :, :S].cpu().numpy()
    rng = np.random.default_rng(S + N + (where == "dev"))
    masks = _masks(rng, N, t, 0, m)
    invalid = [7, 64, 65, N - 1] if where == "dev" else []
    for i in invalid:  # fewer than k present: reported by rs_sync, no rows
        masks[i] = (1 << (k - 1)) - 1
    nmiss = np.array([bin(int(x) ^ ((1 << t) - 1)).count("1") for x in masks])
    cnt = np.where(nmiss > m, 0, nmiss)
    want = np.concatenate([[0], np.cumsum(cnt)]).astype(np.uint32)
    out = torch.full((N * m + 2, P), 0xC3, dtype=torch.uint8, device="cuda")
    roffs = torch.full((N + 1,), -1, dtype=torch.int32, device="cuda")
    if where == "dev":
        eng.reconstruct_packed(data, parity, out, roffs, S, N, masks_dev=torch.from_numpy(masks.view(np.int32)).cuda())
        with pytest.raises(ECError) as ei:
            eng.sync()
        assert ei.value.code == _lib.RS_ERR_TOO_FEW_SHARDS
    else:
        eng.reconstruct_packed(data, parity, out, roffs, S, N, present_masks=masks)
    torch.cuda.synchronize()
    assert np.array_equal(roffs.cpu().numpy().view(np.uint32), want)
    got = out.cpu().numpy()
    rows = np.concatenate([want[i] + np.arange(cnt[i]) for i in range(N)]).astype(np.int64)
    src = np.concatenate([[(i, j) for j in range(t) if not (int(masks[i]) >> j) & 1] if cnt[i] else
                          np.zeros((0, 2), np.int64) for i in range(N)]).astype(np.int64)
    assert len(rows) == len(src) == int(want[N])
    bad = np.nonzero((got[rows, :S] != ref[src[:, 0], src[:, 1]]).any(axis=1))[0]
    assert len(bad) == 0, rows[bad][:8].tolist()
    assert (got[int(want[N]):] == 0xC3).all(), "a row past the batch's total was written"
    assert (got[:, _pad_end(S, P):] == 0xC3).all(), "row padding past the line written"
    # host masks with a stripe below k: refused before anything runs
    if where == "host":
        masks[3] = (1 << (k - 1)) - 1
        with pytest.raises(ECError) as ei:
            eng.reconstruct_packed(data, parity, out, roffs, S, N, present_masks=masks)
        assert ei.value.code == _lib.RS_ERR_TOO_FEW_SHARDS


@pytest.mark.parametrize("nbytes", [16, 4080, 4096, 4112, (1 << 20) + 16, 201326592])
def test_device_copy_exact(engines, nbytes):
    """rs_device_copy (the bench's HBM yardstick): 4 KiB wave tasks whose descriptors
    end with the buffer -- every byte copied, nothing past the end written."""
    import torch

    eng = _engine(engines, 4, 2)
    g = torch.Generator(device="cuda").manual_seed(nbytes % 1000)
    src = torch.randint(0, 256, (nbytes + 4096,), dtype=torch.uint8, device="cuda", generator=g)
    dst = torch.full((nbytes + 4096,), 0x5A, dtype=torch.uint8, device="cuda")
    eng.device_copy(dst, src, nbytes)
    torch.cuda.synchronize()
    assert torch.equal(dst[:nbytes], src[:nbytes])
    assert (dst[nbytes:] == 0x5A).all(), "bytes past the copy written"


@pytest.mark.parametrize("k,m,S", [(10, 4, 6554), (4, 2, 16384), (8, 4, 8192), (4, 2, 1024)])
def test_occupancy_cap_never_changes_bytes(engines, k, m, S):
    """rs_set_occupancy_cap (dynamic-LDS reservation per launch): every cap, the
    tuned defaults (-1) and none (0) give the oracle's bytes on the encode, bounded,
    unbounded and mixed per-stripe paths; caps outside -1..32 are refused."""
    import torch

    eng = BatchEngine(k, m, 0)  # its own context: the cap is context-wide
    try:
        t, N, P = k + m, 257, shard_pitch_for(S)
        data, parity, uni = _codewords(eng, k, m, S, N, 4242 + S)
        rng = np.random.default_rng(S + 1)
        mixed = _masks(rng, N, t, 0, m)
        for cap in (-1, 0, 2, 3, 4, 8, 32):
            eng.set_occupancy_cap(cap)
            p2 = torch.full_like(parity, 0xEE)
            eng.encode(data, p2, S, N)
            torch.cuda.synchronize()
            assert np.array_equal(p2.cpu().numpy()[:, :, :S], uni[:, k:, :S]), ("encode", cap)
            for bound, masks in ((1, _masks(rng, N, t, 1, 1)), (0, mixed)):
                out = torch.full((N, m, P), 0xC3, dtype=torch.uint8, device="cuda")
                eng.reconstruct_out(data, parity, out, S, N, masks_dev=torch.from_numpy(masks.view(np.int32)).cuda(),
                                    max_missing=bound)
                eng.sync()
                o = out.cpu().numpy()
                for i in range(N):
                    miss = [s for s in range(t) if not (masks[i] >> s) & 1]
                    for r, s in enumerate(miss):
                        assert np.array_equal(o[i, r, :S], uni[i, s, :S]), (cap, bound, i, s)
        for bad in (-2, 33):
            with pytest.raises(ECError):
                eng.set_occupancy_cap(bad)
    finally:
        eng.close()
