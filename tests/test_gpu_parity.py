"""GPU parity: the HIP engine (through the C-ABI) vs the CPU oracle, bit-exact.

Reference path: internal/ec/ec.go:48-61 -> klauspost/reedsolomon v1.12.1.  The
callers whose contract these cases mirror: writeservice.go:218-222 (Split+Encode),
readservice.go:285 / poller.go:282 (Reconstruct fills every nil entry).
"""
import itertools
import os
import threading

import numpy as np
import pytest

from oracle import rs_oracle
from replication_erasurecoding_object_store_amd import _lib
from replication_erasurecoding_object_store_amd.batch import BatchEngine, shard_pitch_for
from replication_erasurecoding_object_store_amd.ec import ECError, NewService
from replication_erasurecoding_object_store_amd.xoshiro import xoshiro_bytes

pytestmark = pytest.mark.gpu

KM = [(4, 2), (8, 4), (10, 4), (6, 3), (5, 5), (3, 1), (12, 4), (17, 3)]


@pytest.fixture(scope="module")
def engines(gpu):
    engs = {}
    yield engs
    for e in engs.values():
        e.close()


def eng_for(engines, k, m):
    if (k, m) not in engines:
        engines[(k, m)] = BatchEngine(k, m, 0)
    return engines[(k, m)]


def _pad_end(S, P):
    """First byte of an out-of-place row that is never written: rows end on whole
    128-B lines within their slot (rs_set_out_pad_writes, on in BatchEngine)."""
    return min(P, (S + 127) // 128 * 128)


def _host_diff(got, want):
    """'' when equal, else where a host-resident result differs (stripe / shard / byte
    ranges, how many differing bytes are zero) and whether it still differs 20 ms
    later: in-place zero-copy writes that land late vs bytes that are wrong."""
    import time

    def where():
        bad = np.argwhere(got != want)
        if bad.size == 0:
            return ""
        z = int((got[got != want] == 0).sum())
        return (f"{len(bad)} bytes differ ({z} zero) in {np.unique(bad[:, 0]).size} stripes, "
                f"shards {sorted(set(bad[:, 1].tolist()))}, bytes {bad[:, 2].min()}..{bad[:, 2].max()}, "
                f"first {bad[:4].tolist()}")

    d = where()
    if d:
        time.sleep(0.02)
        d += " | after 20 ms: " + (where() or "equal")
    return d


# ---- per-object IEcDriver surface ------------------------------------------------
@pytest.mark.parametrize("k,m", KM)
@pytest.mark.parametrize("length", [1, 2, 3, 10, 410, 4096, 6554 * 4 + 3, 65536])
def test_split_encode_matches_oracle(engines, k, m, length):
    svc = eng_for(engines, k, m)
    data = xoshiro_bytes(0x5EED0000 + length, length)
    shards = svc.Split(data)
    ref = rs_oracle.split(k, m, data)
    assert [bytes(s) for s in shards] == [bytes(s) for s in ref]
    svc.Encode(shards)
    assert rs_oracle.encode(k, m, ref) == 0
    assert [bytes(s) for s in shards] == [bytes(s) for s in ref]
    assert svc.Verify(shards)


def test_one_encode_kat(engines):
    """[upstream reedsolomon_test.go TestOneEncode] New(5,5) vectors."""
    svc = eng_for(engines, 5, 5)
    shards = [bytearray(x) for x in ([0, 1], [4, 5], [2, 3], [6, 7], [8, 9])] + [bytearray(2) for _ in range(5)]
    svc.Encode(shards)
    assert [list(s[:]) for s in shards[5:]] == [[12, 13], [10, 11], [14, 15], [90, 91], [94, 95]]


def test_reconstruct_all_21_patterns_rs42(engines):
    svc = eng_for(engines, 4, 2)
    data = xoshiro_bytes(0x5EED0003, 4096)
    full = svc.Split(data)
    svc.Encode(full)
    patterns = [c for e in (1, 2) for c in itertools.combinations(range(6), e)]
    assert len(patterns) == 21
    for pat in patterns:
        shards = [bytearray(s) for s in full]
        for i in pat:
            shards[i] = None if i % 2 else bytearray()
        svc.Reconstruct(shards)
        assert [bytes(s) for s in shards] == [bytes(s) for s in full], pat
        # ReconstructData fills only the data shards
        shards = [bytearray(s) for s in full]
        for i in pat:
            shards[i] = None
        svc.ReconstructData(shards)
        for i in range(6):
            if i < 4 or i not in pat:
                assert bytes(shards[i]) == bytes(full[i])
            else:
                assert shards[i] is None


@pytest.mark.parametrize("k,m", [(8, 4), (10, 4), (12, 4)])
def test_reconstruct_max_erasures(engines, k, m):
    svc = eng_for(engines, k, m)
    rng = np.random.default_rng(k * 100 + m)
    data = rng.integers(0, 256, 3000, dtype=np.uint8).tobytes()
    full = svc.Split(data)
    svc.Encode(full)
    for trial in range(12):
        pat = rng.choice(k + m, size=rng.integers(1, m + 1), replace=False)
        shards = [bytearray(s) for s in full]
        for i in pat:
            shards[i] = None
        ref = [None if s is None else bytearray(s) for s in shards]
        svc.Reconstruct(shards)
        assert rs_oracle.reconstruct(k, m, ref) == 0
        assert [bytes(s) for s in shards] == [bytes(s) for s in ref] == [bytes(s) for s in full]


def test_errors_match_klauspost_sentinels(engines):
    svc = eng_for(engines, 4, 2)
    with pytest.raises(ECError, match="not enough data to fill the number of requested shards"):
        svc.Split(b"")
    with pytest.raises(ECError, match="too few shards given"):
        svc.Encode([bytearray(4)] * 5)
    with pytest.raises(ECError, match="shard sizes do not match"):
        svc.Encode([bytearray(4)] * 5 + [bytearray(3)])
    with pytest.raises(ECError, match="shard sizes do not match"):
        svc.Encode([bytearray(4)] * 5 + [None])  # Encode does not accept nil
    with pytest.raises(ECError, match="no shard data"):
        svc.Encode([None] * 6)
    with pytest.raises(ECError, match="too few shards given"):
        svc.Reconstruct([bytearray(4)] * 3 + [None] * 3)
    with pytest.raises(ECError, match="shard sizes do not match"):
        svc.Reconstruct([bytearray(4)] * 4 + [bytearray(5), None])
    with pytest.raises(ECError, match="no shard data"):
        svc.Reconstruct([None] * 6)
    # all present: no-op, no error (upstream quick check)
    sh = svc.Split(b"hello world")
    svc.Encode(sh)
    before = [bytes(s) for s in sh]
    svc.Reconstruct(sh)
    assert [bytes(s) for s in sh] == before


@pytest.mark.parametrize("kind", ["zeros", "ff", "ascii_x", "ascii_A"])
def test_value_distributions(engines, kind):
    svc = eng_for(engines, 4, 2)
    n = 100 * 1024
    data = {"zeros": bytes(n), "ff": b"\xff" * n, "ascii_x": b"x" * n, "ascii_A": b"A" * n}[kind]
    shards = svc.Split(data)
    svc.Encode(shards)
    ref = rs_oracle.split(4, 2, data)
    rs_oracle.encode(4, 2, ref)
    assert [bytes(s) for s in shards] == [bytes(s) for s in ref]


def test_concurrent_callers(engines):
    """One shared IEcDriver, many goroutines (cmd/api/main.go:206 + gin)."""
    svc = eng_for(engines, 4, 2)
    errors = []

    def worker(seed):
        try:
            for j in range(20):
                data = xoshiro_bytes(seed * 1000 + j, 1000 + 37 * j)
                sh = svc.Split(data)
                svc.Encode(sh)
                ref = rs_oracle.split(4, 2, data)
                rs_oracle.encode(4, 2, ref)
                assert [bytes(s) for s in sh] == [bytes(s) for s in ref]
                sh[1] = None
                sh[4] = None
                svc.Reconstruct(sh)
                assert [bytes(s) for s in sh] == [bytes(s) for s in ref]
        except Exception as exc:  # pragma: no cover - reported below
            errors.append(exc)

    ts = [threading.Thread(target=worker, args=(i,)) for i in range(12)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errors, errors[0]


# ---- batched device path -----------------------------------------------------------
def _rand_batch(torch, n, t, pitch, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    return torch.randint(0, 256, (n, t, pitch), dtype=torch.uint8, device="cuda", generator=g)


@pytest.mark.parametrize("k,m", KM)
@pytest.mark.parametrize("S", [1, 15, 16, 17, 410, 1024, 1040, 6554, 16384])
def test_batch_encode_device(engines, k, m, S):
    import torch

    eng = eng_for(engines, k, m)
    N = max(3, min(300, (4 << 20) // (S * (k + m))))
    P = shard_pitch_for(S)
    buf = _rand_batch(torch, N, k + m, P, seed=S * 31 + k)
    eng.encode_unified(buf, S, P, N)
    torch.cuda.synchronize()
    got = buf.cpu().numpy()
    exp = got.copy()
    exp[:, k:, :] = 0
    rs_oracle.encode_batch_scalar(k, m, exp.reshape(-1), (k + m) * P, P, S, N)
    assert np.array_equal(got[:, :, :S], exp[:, :, :S])


def test_batch_encode_separate_parity_buffer(engines):
    import torch

    k, m, S, N = 4, 2, 1000, 257
    eng = eng_for(engines, k, m)
    P = shard_pitch_for(S)
    data = _rand_batch(torch, N, k, P, seed=5)
    parity = torch.full((N, m, P), 0xAB, dtype=torch.uint8, device="cuda")
    eng.encode(data, parity, S, N, P, k * P, m * P)
    torch.cuda.synchronize()
    uni = np.zeros((N, k + m, P), np.uint8)
    uni[:, :k] = data.cpu().numpy()
    rs_oracle.encode_batch_scalar(k, m, uni.reshape(-1), (k + m) * P, P, S, N)
    got = parity.cpu().numpy()
    assert np.array_equal(got[:, :, :S], uni[:, k:, :S])
    assert (got[:, :, S:] == 0xAB).all(), "padding of output slots must not be written"


@pytest.mark.parametrize("k,m", [(4, 2), (8, 4), (10, 4)])
@pytest.mark.parametrize("S", [1024, 6554])
def test_batch_reconstruct_uniform_all_patterns(engines, k, m, S):
    import torch

    eng = eng_for(engines, k, m)
    t = k + m
    N = 64
    P = shard_pitch_for(S)
    buf = _rand_batch(torch, N, t, P, seed=11 + k)
    eng.encode_unified(buf, S, P, N)
    torch.cuda.synchronize()
    orig = buf.clone()
    pats = [c for e in range(1, m + 1) for c in itertools.combinations(range(t), e)]
    if len(pats) > 60:
        rng = np.random.default_rng(S + k)
        pats = [pats[i] for i in rng.choice(len(pats), 60, replace=False)]
    for pat in pats:
        work = orig.clone()
        mask = (1 << t) - 1
        for i in pat:
            work[:, i, :S] = 0x5A
            mask &= ~(1 << i)
        eng.reconstruct_unified(work, S, P, N, mask)
        torch.cuda.synchronize()
        assert torch.equal(work[:, :, :S], orig[:, :, :S]), pat


@pytest.mark.parametrize("k,m", [(4, 2), (8, 4), (10, 4)])
def test_batch_reconstruct_per_stripe_masks(engines, k, m):
    import torch

    eng = eng_for(engines, k, m)
    t, S, N = k + m, 1024, 2048
    P = shard_pitch_for(S)
    buf = _rand_batch(torch, N, t, P, seed=99 + k)
    eng.encode_unified(buf, S, P, N)
    torch.cuda.synchronize()
    orig = buf.clone()
    rng = np.random.default_rng(0x5EED0003)
    masks = np.full(N, (1 << t) - 1, np.uint32)
    for i in range(N):
        e = rng.integers(0, m + 1)
        for j in rng.choice(t, size=e, replace=False):
            masks[i] &= ~np.uint32(1 << int(j))
    lost = torch.from_numpy(((masks[:, None] >> np.arange(t)[None, :]) & 1) == 0).cuda()
    work = orig.clone()
    work[:, :, :S][lost] = 0
    eng.reconstruct_unified(work, S, P, N, masks)
    torch.cuda.synchronize()
    assert torch.equal(work[:, :, :S], orig[:, :, :S])
    # device-resident masks give the same result
    work2 = orig.clone()
    work2[:, :, :S][lost] = 0
    eng.reconstruct_unified_devmask(work2, S, P, N, torch.from_numpy(masks.view(np.int32)).cuda())
    eng.sync()
    assert torch.equal(work2[:, :, :S], orig[:, :, :S])


def test_batch_reconstruct_too_few(engines):
    import torch

    eng = eng_for(engines, 4, 2)
    S, N = 64, 4
    P = shard_pitch_for(S)
    buf = _rand_batch(torch, N, 6, P, seed=1)
    before = buf.clone()
    with pytest.raises(ECError, match="too few shards given"):
        eng.reconstruct_unified(buf, S, P, N, np.array([0b111111, 0b000111, 0b111100, 0b110011], np.uint32))
    torch.cuda.synchronize()
    assert torch.equal(buf, before), "a rejected batch must not be modified"
    masks = torch.tensor([0b111111, 0b000111, 0b111100, 0b110011], dtype=torch.int32, device="cuda")
    eng.reconstruct_unified_devmask(buf, S, P, N, masks)
    with pytest.raises(ECError, match="too few shards given"):
        eng.sync()


def _host_mem(eng, mem, shape):
    """A zeroed host array of `shape` in memory kind `mem`: "alloc" (rs_host_alloc,
    the only memory a kernel addresses in place), "register" (rs_host_register'ed
    numpy memory: recorded, staged) or "pageable"."""
    n = int(np.prod(shape))
    if mem == "alloc":
        a = eng.host_alloc(n).reshape(shape)
        a[:] = 0
        return a
    a = np.zeros(shape, np.uint8)
    if mem == "register":
        eng.host_register(a)
    return a


def _host_mem_free(eng, mem, a):
    if mem == "alloc":
        eng.host_free(a)
    elif mem == "register":
        eng.host_unregister(a)


@pytest.mark.parametrize("zero_copy", [True, False])
@pytest.mark.parametrize("mem", ["alloc", "register"])
def test_batch_host_paths_match_device(engines, zero_copy, mem):
    import torch

    k, m = 4, 2
    eng = eng_for(engines, k, m)
    S, N = 1024, 5000
    P = shard_pitch_for(S)
    buf = _rand_batch(torch, N, k + m, P, seed=3)
    host = _host_mem(eng, mem, (N, k + m, P))
    host[:] = buf.cpu().numpy()
    eng.encode_unified(buf, S, P, N)
    torch.cuda.synchronize()
    eng.set_host_zero_copy(zero_copy)
    path = "zero-copy" if zero_copy and mem == "alloc" else "staged"
    try:
        eng.encode_host_unified(host, S, P, N)
        assert eng.last_host_path() == path
        assert np.array_equal(host[:, :, :S], buf.cpu().numpy()[:, :, :S])
        orig = host.copy()
        host[:, 0, :S] = 0
        host[:, 3, :S] = 0
        eng.reconstruct_host_unified(host, S, P, N, 0b110110)
        assert not _host_diff(host[:, :, :S], orig[:, :, :S]), _host_diff(host[:, :, :S], orig[:, :, :S])
        rng = np.random.default_rng(5)
        masks = np.array([0b111111 & ~(1 << rng.integers(0, 6)) for _ in range(N)], np.uint32)
        for i in range(N):
            for j in range(6):
                if not (masks[i] >> j) & 1:
                    host[i, j, :S] = 0
        eng.reconstruct_host_unified(host, S, P, N, masks)
        assert not _host_diff(host[:, :, :S], orig[:, :, :S]), _host_diff(host[:, :, :S], orig[:, :, :S])
        assert eng.last_host_path() == path
    finally:
        eng.set_host_zero_copy(True)
        _host_mem_free(eng, mem, host)


@pytest.mark.parametrize("k,m", [(4, 2), (10, 4)])
def test_staged_per_stripe_never_writes_present_slots(engines, k, m):
    """Staged per-stripe host reconstruct (round 5, host_batch_ps): every present
    slot of the caller's memory is read-only (mprotect) during the call -- a write by
    DMA or by the host scatter would fail the call or fault -- and the missing slots
    come back equal to the oracle's codewords.  Intact stripes, 1..m erasures and
    slack bytes past S in every slot (guard pattern, never written) included."""
    import ctypes
    import mmap

    eng = eng_for(engines, k, m)
    t = k + m
    S, P, N = 4000, 4096, 48  # one page per slot: each present slot protected on its own
    mm = mmap.mmap(-1, N * t * P)
    host = np.frombuffer(mm, np.uint8).reshape(N, t, P)
    rng = np.random.default_rng(21)
    want = np.zeros((N, t, S), np.uint8)
    want[:, :k] = rng.integers(0, 256, (N, k, S), dtype=np.uint8)
    rs_oracle.encode_batch_scalar(k, m, want.reshape(-1), t * S, S, S, N)
    host[:, :, :S] = want
    host[:, :, S:] = 0xA5  # guard bytes past S
    masks = np.full(N, (1 << t) - 1, np.uint32)
    for i in range(N):
        ne = i % (m + 1)  # 0 (intact) .. m erasures
        for j in rng.choice(t, size=ne, replace=False):
            masks[i] &= ~np.uint32(1 << int(j))
            host[i, j, :S] = 0
    libc = ctypes.CDLL(None, use_errno=True)
    libc.mprotect.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    base = host.ctypes.data
    present = [(i, j) for i in range(N) for j in range(t) if (masks[i] >> j) & 1]
    for i, j in present:
        assert libc.mprotect(base + (i * t + j) * P, P, mmap.PROT_READ) == 0
    try:
        eng.reconstruct_host_unified(host, S, P, N, masks)
        assert eng.last_host_path() == "staged"
    finally:
        for i, j in present:
            libc.mprotect(base + (i * t + j) * P, P, mmap.PROT_READ | mmap.PROT_WRITE)
    assert not _host_diff(host[:, :, :S], want), _host_diff(host[:, :, :S], want)
    assert (host[:, :, S:] == 0xA5).all(), "bytes past S were written"
    del host
    mm.close()


def test_config2_full_size_roundtrip(engines):
    """BASELINE config 2/3 at full size (65 536 x 4 KiB stripes): encode, check a
    sample of stripes against the oracle, then erase 2 shards per stripe (seeded
    random pattern) and reconstruct -- must return the original bytes."""
    import torch

    k, m, S, N = 4, 2, 1024, 65536
    eng = eng_for(engines, k, m)
    P = shard_pitch_for(S)
    buf = _rand_batch(torch, N, k + m, P, seed=0x5EED0002)
    eng.encode_unified(buf, S, P, N)
    torch.cuda.synchronize()
    idx = np.random.default_rng(0).choice(N, 512, replace=False)
    got = buf[torch.from_numpy(idx).cuda()].cpu().numpy()
    exp = got.copy()
    rs_oracle.encode_batch_scalar(k, m, exp.reshape(-1), (k + m) * P, P, S, len(idx))
    assert np.array_equal(got[:, :, :S], exp[:, :, :S])
    orig = buf.clone()
    rng = np.random.default_rng(0x5EED0003)
    pairs = np.array(list(itertools.combinations(range(6), 2)))
    choice = pairs[rng.integers(0, len(pairs), N)]
    masks = (0b111111 & ~((1 << choice[:, 0]) | (1 << choice[:, 1]))).astype(np.uint32)
    rows = torch.arange(N, device="cuda")
    for col in range(2):
        buf[rows, torch.from_numpy(choice[:, col]).cuda(), :S] = 0
    eng.reconstruct_unified(buf, S, P, N, masks)
    torch.cuda.synchronize()
    assert torch.equal(buf[:, :, :S], orig[:, :, :S])


def test_config3_full_size_one_erasure(engines):
    """BASELINE configs[2], 1-missing leg, at full size: the 65 536 x 4 KiB batch
    with one erased shard per stripe (index uniform in [0, 6), seed 0x5EED0003).
    Sampled stripes are compared with rs_oracle.reconstruct (the oracle's own
    two-phase klauspost reconstruct, not a re-encode) and every stripe round-trips:
    in place with host masks, out of place with device masks (bound 1 and none)."""
    import torch

    k, m, S, N = 4, 2, 1024, 65536
    t = k + m
    eng = eng_for(engines, k, m)
    P = shard_pitch_for(S)
    buf = _rand_batch(torch, N, t, P, seed=0x5EED0002)
    eng.encode_unified(buf, S, P, N)
    torch.cuda.synchronize()
    orig = buf.clone()
    lost = np.random.default_rng(0x5EED0003).integers(0, t, N)
    masks = (((1 << t) - 1) & ~(1 << lost)).astype(np.uint32)
    rows = torch.arange(N, device="cuda")
    lost_d = torch.from_numpy(lost).cuda()
    buf[rows, lost_d, :S] = 0
    erased = buf.clone()
    eng.reconstruct_unified(buf, S, P, N, masks)
    torch.cuda.synchronize()
    assert torch.equal(buf[:, :, :S], orig[:, :, :S])
    # oracle on sampled stripes: its reconstruct from the erased shard lists
    idx = np.random.default_rng(3).choice(N, 256, replace=False)
    er = erased[torch.from_numpy(idx).cuda()].cpu().numpy()
    got = buf[torch.from_numpy(idx).cuda()].cpu().numpy()
    for j, i in enumerate(idx):
        sh = [bytearray(er[j, s, :S].tobytes()) if s != lost[i] else None for s in range(t)]
        assert rs_oracle.reconstruct(k, m, sh) == 0
        assert all(bytes(sh[s]) == got[j, s, :S].tobytes() for s in range(t)), i
    # out of place with device masks: split views of the same buffer
    data, parity = orig[:, :k], orig[:, k:]
    mdev = torch.from_numpy(masks.view(np.int32)).cuda()
    for bound in (1, 0):
        out = torch.full((N, 1 if bound else m, P), 0xC3, dtype=torch.uint8, device="cuda")
        eng.reconstruct_out(data.contiguous(), parity.contiguous(), out, S, N, masks_dev=mdev, max_missing=bound)
        eng.sync()
        assert torch.equal(out[:, 0, :S], orig[rows, lost_d, :S]), bound


def test_golden_fixtures_through_hip(engines):
    """The committed golden vectors (tests/golden/rs_golden.npz, the oracle's
    pinned fixtures) fed through the HIP path itself: Split + Encode of every
    stored object and a device batch of its data shards reproduce the stored
    parity, and every stored erasure pattern (dec_<k>_<m>_<pattern>) reconstructs
    the stored 4 KiB object of its code byte-exact."""
    import torch

    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "rs_golden.npz"))
    n_enc = n_dec = 0
    objs = {}
    for key in sorted(g.files):
        if not (key.startswith("enc_") and key.endswith("_data")):
            continue
        _, k, m, L, _ = key.split("_")
        k, m, L = int(k), int(m), int(L)
        value, parity = g[key].tobytes(), g[key[: -len("data")] + "parity"]
        eng = eng_for(engines, k, m)
        shards = eng.Split(value)
        eng.Encode(shards)
        S = len(shards[0])
        assert parity.shape == (m, S), key
        assert all(bytes(shards[k + r]) == parity[r].tobytes() for r in range(m)), key
        P = shard_pitch_for(S)
        d = torch.zeros((3, k, P), dtype=torch.uint8, device="cuda")
        d[:, :, :S] = torch.from_numpy(np.frombuffer(b"".join(bytes(x) for x in shards[:k]), np.uint8)
                                       .reshape(k, S)).cuda()
        p = torch.zeros((3, m, P), dtype=torch.uint8, device="cuda")
        eng.encode(d, p, S, 3)
        torch.cuda.synchronize()
        assert np.array_equal(p[:, :, :S].cpu().numpy(), np.broadcast_to(parity, (3, m, S))), key
        if L == 4096:
            objs[(k, m)] = shards
        n_enc += 1
    for key in sorted(g.files):
        if not key.startswith("dec_"):
            continue
        _, k, m, pat = key.split("_")
        k, m = int(k), int(m)
        lost = [int(x) for x in pat.split("-")]
        full = objs[(k, m)]
        sh = [None if i in lost else bytearray(s) for i, s in enumerate(full)]
        eng_for(engines, k, m).Reconstruct(sh)
        assert [bytes(x) for x in sh] == [bytes(x) for x in full], key
        n_dec += 1
    assert n_enc >= 18 and n_dec >= 40, (n_enc, n_dec)


# ---- split layout (data region + parity region): the bench layout -------------------
def _masks_upto(rng, N, t, m):
    masks = np.full(N, (1 << t) - 1, np.uint32)
    for i in range(N):
        for j in rng.choice(t, size=rng.integers(0, m + 1), replace=False):
            masks[i] &= ~np.uint32(1 << int(j))
    return masks


@pytest.mark.parametrize("k,m", [(4, 2), (8, 4), (10, 4), (6, 3), (12, 4)])
@pytest.mark.parametrize("S", [7, 1000, 1024, 6554])
def test_split_layout_device(engines, k, m, S):
    import torch

    eng = eng_for(engines, k, m)
    N = 777
    P = shard_pitch_for(S)
    g = torch.Generator(device="cuda").manual_seed(S + 17 * k)
    data = torch.randint(0, 256, (N, k, P), dtype=torch.uint8, device="cuda", generator=g)
    parity = torch.full((N, m, P), 0xEE, dtype=torch.uint8, device="cuda")
    eng.encode(data, parity, S, N)
    torch.cuda.synchronize()
    uni = np.zeros((N, k + m, P), np.uint8)
    uni[:, :k] = data.cpu().numpy()
    rs_oracle.encode_batch_scalar(k, m, uni.reshape(-1), (k + m) * P, P, S, N)
    par = parity.cpu().numpy()
    assert np.array_equal(par[:, :, :S], uni[:, k:, :S])
    assert (par[:, :, S:] == 0xEE).all(), "slot padding must never be written"
    # per-stripe erasures (0..m per stripe), host masks then device masks
    rng = np.random.default_rng(S * 3 + k)
    t = k + m
    for use_dev in (False, True):
        masks = _masks_upto(rng, N, t, m)
        lost = ((masks[:, None] >> np.arange(t)[None, :]) & 1) == 0
        d2, p2 = data.clone(), parity.clone()
        dl = torch.from_numpy(lost[:, :k]).cuda()
        pl = torch.from_numpy(lost[:, k:]).cuda()
        d2[:, :, :S][dl] = 0x33
        p2[:, :, :S][pl] = 0x33
        if use_dev and t <= 16:
            eng.reconstruct_devmask(d2, p2, S, N, torch.from_numpy(masks.view(np.int32)).cuda())
            eng.sync()
        elif not use_dev:
            if t > 16:
                # per-stripe patterns need the k+m <= 16 LUT: one uniform pattern instead
                one = np.uint32(((1 << t) - 1) & ~0b101)
                d2[:, 0, :S] = 0x33
                d2[:, 2, :S] = 0x33
                eng.reconstruct(d2, p2, S, N, one)
            else:
                eng.reconstruct(d2, p2, S, N, masks)
        torch.cuda.synchronize()
        assert torch.equal(d2[:, :, :S], data[:, :, :S])
        assert torch.equal(p2[:, :, :S], parity[:, :, :S])


def test_host_alloc_batches_zero_copy(engines):
    """Host batches in context-owned page-locked memory (rs_host_alloc): zero-copy,
    oracle bytes for encode, a uniform and a per-stripe reconstruct; the pointer is
    rs_host_free's alone (rs_host_unregister refuses it)."""
    from replication_erasurecoding_object_store_amd import _lib

    k, m, S, N = 4, 2, 1024, 3000
    eng = eng_for(engines, k, m)
    buf = eng.host_alloc(N * (k + m) * S)
    try:
        data = buf[:N * k * S].reshape(N, k, S)
        parity = buf[N * k * S:].reshape(N, m, S)
        data[:] = np.random.default_rng(77).integers(0, 256, (N, k, S), dtype=np.uint8)
        parity[:] = 0
        eng.encode_host(data, parity, S, N)
        assert eng.last_host_path() == "zero-copy"
        uni = np.concatenate([data, np.zeros_like(parity)], axis=1).copy()
        rs_oracle.encode_batch_scalar(k, m, uni.reshape(-1), (k + m) * S, S, S, N)
        assert not _host_diff(parity, uni[:, k:]), _host_diff(parity, uni[:, k:])
        d0, p0 = data.copy(), parity.copy()
        data[:, 2] = 0
        parity[:, 1] = 0
        eng.reconstruct_host(data, parity, S, N, 0b011011)
        assert not _host_diff(data, d0) and not _host_diff(parity, p0), (_host_diff(data, d0), _host_diff(parity, p0))
        masks = _masks_upto(np.random.default_rng(78), N, 6, 2)
        lost = ((masks[:, None] >> np.arange(6)[None, :]) & 1) == 0
        data[lost[:, :4]] = 0
        parity[lost[:, 4:]] = 0
        eng.reconstruct_host(data, parity, S, N, masks)
        assert eng.last_host_path() == "zero-copy"
        assert not _host_diff(data, d0) and not _host_diff(parity, p0), (_host_diff(data, d0), _host_diff(parity, p0))
        assert _lib.lib().rs_host_unregister(eng.ctx, buf.ctypes.data) == _lib.RS_ERR_INVALID_ARG
    finally:
        eng.host_free(buf)


def test_host_path_routing(engines):
    """Which host memory a kernel may address in place (`HISTORY.md` §A.1): only the
    context's own page-locked memory (rs_host_alloc) runs zero-copy.  Pageable,
    rs_host_register'ed and torch-pinned memory -- pages whose placement the library
    does not control -- are staged, and the bytes are the same either way."""
    import torch

    k, m, S, N = 4, 2, 1024, 256
    eng = eng_for(engines, k, m)
    src = np.random.default_rng(11).integers(0, 256, (N, k, S), dtype=np.uint8)
    want = np.concatenate([src, np.zeros((N, m, S), np.uint8)], axis=1)
    rs_oracle.encode_batch_scalar(k, m, want.reshape(-1), (k + m) * S, S, S, N)
    kinds = {"alloc": "zero-copy", "register": "staged", "pageable": "staged", "torch_pinned": "staged"}
    for mem, path in kinds.items():
        if mem == "torch_pinned":
            data = torch.empty((N, k, S), dtype=torch.uint8, pin_memory=True).numpy()
            parity = torch.zeros((N, m, S), dtype=torch.uint8, pin_memory=True).numpy()
        else:
            data, parity = _host_mem(eng, mem, (N, k, S)), _host_mem(eng, mem, (N, m, S))
        try:
            data[:] = src
            eng.encode_host(data, parity, S, N)
            assert eng.last_host_path() == path, mem
            assert np.array_equal(parity, want[:, k:]), mem
        finally:
            if mem != "torch_pinned":
                _host_mem_free(eng, mem, data)
                _host_mem_free(eng, mem, parity)
    # register: ranges may not overlap a known one; unregister only what was registered
    a = np.zeros(8192, np.uint8)
    L = _lib.lib()
    assert L.rs_host_register(eng.ctx, a.ctypes.data, 4096) == 0
    assert L.rs_host_register(eng.ctx, a.ctypes.data + 100, 4096) == _lib.RS_ERR_INVALID_ARG
    assert L.rs_host_unregister(eng.ctx, a.ctypes.data + 100) == _lib.RS_ERR_INVALID_ARG
    assert L.rs_host_unregister(eng.ctx, a.ctypes.data) == 0
    assert L.rs_host_unregister(eng.ctx, a.ctypes.data) == _lib.RS_ERR_INVALID_ARG


@pytest.mark.parametrize("zero_copy", [True, False])
@pytest.mark.parametrize("S,mem", [(1024, "alloc"), (1000, "alloc"), (1024, "register")])
def test_split_layout_host(engines, S, mem, zero_copy):
    k, m = 4, 2
    eng = eng_for(engines, k, m)
    N = 3000
    P = S  # host layout: shards back to back (the Split view), no padding
    rng = np.random.default_rng(S)
    data = _host_mem(eng, mem, (N, k, P))
    data[:] = rng.integers(0, 256, (N, k, P), dtype=np.uint8)
    parity = _host_mem(eng, mem, (N, m, P))
    eng.set_host_zero_copy(zero_copy)
    # zero-copy needs the context's own memory and 16-B slots
    path = "zero-copy" if zero_copy and S % 16 == 0 and mem == "alloc" else "staged"
    try:
        eng.encode_host(data, parity, S, N)
        assert eng.last_host_path() == path
        uni = np.concatenate([data, np.zeros_like(parity)], axis=1).copy()
        rs_oracle.encode_batch_scalar(k, m, uni.reshape(-1), (k + m) * P, P, S, N)
        assert np.array_equal(parity, uni[:, k:])
        d0, p0 = data.copy(), parity.copy()
        data[:, 1] = 0
        parity[:, 0] = 0
        eng.reconstruct_host(data, parity, S, N, 0b101101)
        assert not _host_diff(data, d0) and not _host_diff(parity, p0), (_host_diff(data, d0), _host_diff(parity, p0))
        masks = _masks_upto(rng, N, 6, 2)
        lost = ((masks[:, None] >> np.arange(6)[None, :]) & 1) == 0
        data[lost[:, :4]] = 0
        parity[lost[:, 4:]] = 0
        eng.reconstruct_host(data, parity, S, N, masks)
        assert not _host_diff(data, d0) and not _host_diff(parity, p0), (_host_diff(data, d0), _host_diff(parity, p0))
        # scrub, zero-copy or staged alike
        assert not eng.verify_host(data, parity, S, N).any()
        parity[17, 1, 3] ^= 4
        assert np.array_equal(np.nonzero(eng.verify_host(data, parity, S, N))[0], [17])
        assert eng.last_host_path() == path
    finally:
        eng.set_host_zero_copy(True)
        _host_mem_free(eng, mem, data)
        _host_mem_free(eng, mem, parity)


@pytest.mark.parametrize("k,m", [(4, 2), (8, 4), (10, 4), (12, 4)])
@pytest.mark.parametrize("S", [1024, 6554, 100])
def test_reconstruct_out_of_place(engines, k, m, S):
    """rs_reconstruct_batch_out: r-th missing shard of stripe i lands in out[i, r];
    the shard buffers are not written."""
    import torch

    eng = eng_for(engines, k, m)
    N, t = 513, k + m
    P = shard_pitch_for(S)
    g = torch.Generator(device="cuda").manual_seed(k * 1000 + S)
    data = torch.randint(0, 256, (N, k, P), dtype=torch.uint8, device="cuda", generator=g)
    parity = torch.empty((N, m, P), dtype=torch.uint8, device="cuda")
    eng.encode(data, parity, S, N)
    full = torch.cat([data, parity], dim=1)  # [N, t, P]
    rng = np.random.default_rng(S + k)
    modes = ["uniform", "host"] + (["dev"] if t <= 16 else [])
    for mode in modes:
        if mode == "uniform":
            miss = sorted(rng.choice(t, size=m, replace=False).tolist())
            masks = np.full(N, ((1 << t) - 1) & ~sum(1 << j for j in miss), np.uint32)
        else:
            masks = _masks_upto(rng, N, t, m)
            masks[0] = (1 << t) - 1  # a complete stripe: nothing written for it
        d0, p0 = data.clone(), parity.clone()
        out = torch.full((N, m, P), 0xC3, dtype=torch.uint8, device="cuda")
        if mode == "uniform":
            eng.reconstruct_out(data, parity, out, S, N, present_masks=masks[0])
        elif mode == "host":
            eng.reconstruct_out(data, parity, out, S, N, present_masks=masks)
        else:
            eng.reconstruct_out(data, parity, out, S, N, masks_dev=torch.from_numpy(masks.view(np.int32)).cuda())
            eng.sync()
        # a device fault is reported asynchronously: name the mode whose launch preceded it
        try:
            torch.cuda.synchronize()
            _ = out[0, 0, 0].item()
        except Exception as exc:
            raise AssertionError(f"device error after mode {mode} (last launch on this stream: "
                                 f"{eng.last_kernel_on()}): {exc}") from exc
        assert torch.equal(data, d0) and torch.equal(parity, p0), "inputs must be read-only"
        got = out.cpu().numpy()
        ref = full.cpu().numpy()
        for i in range(N):
            missing = [j for j in range(t) if not (masks[i] >> j) & 1]
            for r, j in enumerate(missing):
                assert np.array_equal(got[i, r, :S], ref[i, j, :S]), (mode, i, r, j)
            for r in range(len(missing), m):
                assert (got[i, r] == 0xC3).all(), "unused output slots untouched"
        assert (got[:, :, _pad_end(S, P):] == 0xC3).all()


# ---- batched verify / scrub (rs_verify_batch) -------------------------------------
def _oracle_bad(k, m, data_np, parity_np, S):
    """Expected mismatch bitmask per stripe: oracle re-encode vs stored parity."""
    N, _, P = data_np.shape
    uni = np.zeros((N, k + m, P), np.uint8)
    uni[:, :k] = data_np
    rs_oracle.encode_batch_scalar(k, m, uni.reshape(-1), (k + m) * P, P, S, N)
    diff = (uni[:, k:, :S] != parity_np[:, :, :S]).any(axis=2)  # [N, m]
    return (diff * (1 << np.arange(m))[None, :]).sum(axis=1).astype(np.uint32)


@pytest.mark.parametrize("k,m", [(4, 2), (8, 4), (10, 4), (6, 3), (5, 5), (12, 4)])
@pytest.mark.parametrize("S", [1, 15, 16, 100, 1024, 1040, 6554, 10923])
def test_verify_batch_device(engines, k, m, S):
    """Clean stripes report 0; corrupting a data or parity byte flags exactly the
    parity rows the oracle's re-encode disagrees with; slot padding is ignored."""
    import torch

    eng = eng_for(engines, k, m)
    N = 300
    P = shard_pitch_for(S)
    g = torch.Generator(device="cuda").manual_seed(S * 31 + k)
    data = torch.randint(0, 256, (N, k, P), dtype=torch.uint8, device="cuda", generator=g)
    parity = torch.empty((N, m, P), dtype=torch.uint8, device="cuda")
    eng.encode(data, parity, S, N)
    bad = torch.full((N,), -1, dtype=torch.int32, device="cuda")
    eng.verify(data, parity, bad, S, N)
    torch.cuda.synchronize()
    assert int(bad.abs().sum()) == 0, "intact stripes must verify clean"
    # ragged shard lengths (columns not a multiple of 64) on the specialised shapes run
    # the flat-task kernel, whose tasks straddle stripes
    cols = -(-S // 16)
    flat = cols >= 64 and cols % 64 != 0 and (k, m) in [(4, 2), (8, 4), (10, 4), (6, 3)]
    assert eng.last_kernel().startswith("verify_flat_kernel" if flat else "verify_kernel"), eng.last_kernel()
    # corrupt: one random byte in a data shard or a parity shard of ~1/3 of stripes;
    # garbage in the slot padding of every stripe must not count
    rng = np.random.default_rng(S + k * 7)
    d_np, p_np = data.cpu().numpy(), parity.cpu().numpy()
    if P > S:
        d_np[:, :, S:] ^= 0x5A
        p_np[:, :, S:] ^= 0xA5
    hit = rng.random(N) < 0.33
    for i in np.nonzero(hit)[0]:
        b = int(rng.integers(0, S))
        flip = np.uint8(rng.integers(1, 256))
        if rng.random() < 0.5:
            d_np[i, int(rng.integers(0, k)), b] ^= flip
        else:
            p_np[i, int(rng.integers(0, m)), b] ^= flip
    exp = _oracle_bad(k, m, d_np, p_np, S)
    assert (exp[hit] != 0).all() and (exp[~hit] == 0).all()
    data.copy_(torch.from_numpy(d_np))
    parity.copy_(torch.from_numpy(p_np))
    eng.verify(data, parity, bad, S, N)
    torch.cuda.synchronize()
    assert np.array_equal(bad.cpu().numpy().view(np.uint32), exp)


def test_verify_batch_host_and_per_object(engines):
    k, m, S, N = 4, 2, 1000, 2500
    eng = eng_for(engines, k, m)
    rng = np.random.default_rng(99)
    data = rng.integers(0, 256, (N, k, S), dtype=np.uint8)
    parity = np.zeros((N, m, S), np.uint8)
    eng.encode_host(data, parity, S, N)
    assert not eng.verify_host(data, parity, S, N).any()
    parity[7, 1, 999] ^= 1
    data[1234, 0, 0] ^= 0x80
    bad = eng.verify_host(data, parity, S, N)
    exp = _oracle_bad(k, m, data, parity, S)
    assert np.array_equal(bad, exp) and bad[7] == 0b10 and bad[1234] != 0
    assert np.count_nonzero(bad) == 2
    # per-object Verify agrees (klauspost Verify -> false on any parity mismatch)
    for i in (6, 7, 1234):
        shards = [bytearray(data[i, j]) for j in range(k)] + [bytearray(parity[i, j]) for j in range(m)]
        assert eng.Verify(shards) == (bad[i] == 0)


@pytest.mark.parametrize("k,m,S", [(4, 2, 1024), (10, 4, 6554), (4, 2, 100)])
def test_soa_layout_device(engines, k, m, S):
    """SURVEY §8d config 2's strided SoA variant: shard s of every stripe in one
    plane, data [K, N, P] / parity [M, N, P] (shard pitch = N*P, stripe pitch = P).
    Same bytes as the split layout."""
    import torch

    eng = eng_for(engines, k, m)
    N = 999
    P = shard_pitch_for(S)
    g = torch.Generator(device="cuda").manual_seed(S + k)
    data = torch.randint(0, 256, (k, N, P), dtype=torch.uint8, device="cuda", generator=g)
    parity = torch.full((m, N, P), 0x77, dtype=torch.uint8, device="cuda")
    eng.encode(data, parity, S, N, shard_pitch=N * P, data_stripe_pitch=P, parity_stripe_pitch=P)
    ref_d = data.permute(1, 0, 2).contiguous()
    ref_p = torch.empty((N, m, P), dtype=torch.uint8, device="cuda")
    eng.encode(ref_d, ref_p, S, N)
    torch.cuda.synchronize()
    assert torch.equal(parity.permute(1, 0, 2)[:, :, :S], ref_p[:, :, :S])
    assert (parity[:, :, S:] == 0x77).all()
    # per-stripe 2-erasure reconstruct, out of place, SoA out [M, N, P]
    rng = np.random.default_rng(S)
    t = k + m
    masks = _masks_upto(rng, N, t, m)
    out = torch.full((m, N, P), 0x55, dtype=torch.uint8, device="cuda")
    _lib_out = __import__("replication_erasurecoding_object_store_amd._lib", fromlist=["lib"])
    rc = _lib_out.lib().rs_reconstruct_batch_out(
        eng.ctx, data.data_ptr(), P, parity.data_ptr(), P, N * P, S, N,
        masks.ctypes.data, N, 0, out.data_ptr(), P, torch.cuda.current_stream().cuda_stream)
    assert rc == 0
    torch.cuda.synchronize()
    full = torch.cat([data, parity], dim=0).cpu().numpy()  # [t, N, P]
    got = out.cpu().numpy()
    for i in range(N):
        missing = [j for j in range(t) if not (masks[i] >> j) & 1]
        for r, j in enumerate(missing):
            assert np.array_equal(got[r, i, :S], full[j, i, :S]), (i, r, j)


# ---- bitsliced encode over flat 128-column tasks (tasks straddle stripes) -----------
@pytest.mark.parametrize("k,m", [(8, 4), (10, 4)])
@pytest.mark.parametrize("S,N", [(2048, 1), (2048, 3), (2049, 2), (6554, 1), (6554, 5), (6554, 37),
                                 (4000, 7), (3000, 129), (16383, 3), (2047, 4), (2032, 4)])
def test_bitsliced_flat_tasks(engines, k, m, S, N):
    """Every stripe boundary position inside a task, batches whose column count is not
    a multiple of 128, partial last columns at every offset, one-stripe batches, and a
    shard length just below the flat kernel's 128-column minimum (2032: lookup kernel)."""
    import torch

    eng = eng_for(engines, k, m)
    P = shard_pitch_for(S)
    g = torch.Generator(device="cuda").manual_seed(S * 7 + N + k)
    data = torch.randint(0, 256, (N, k, P), dtype=torch.uint8, device="cuda", generator=g)
    parity = torch.full((N, m, P), 0xEE, dtype=torch.uint8, device="cuda")
    eng.encode(data, parity, S, N)
    torch.cuda.synchronize()
    kname = eng.last_kernel()
    bitsliced = "bitsliced" in kname or "bs16" in kname  # 2 KiB-row or 1 KiB-task pair kernel
    assert bitsliced == (S >= 2033), kname  # 128 columns = S > 2032
    uni = np.zeros((N, k + m, P), np.uint8)
    uni[:, :k] = data.cpu().numpy()
    rs_oracle.encode_batch_scalar(k, m, uni.reshape(-1), (k + m) * P, P, S, N)
    par = parity.cpu().numpy()
    assert np.array_equal(par[:, :, :S], uni[:, k:, :S]), kname
    assert (par[:, :, S:] == 0xEE).all(), "slot padding must never be written"
    # unified K+M-slot layout: the next stripe's parity is data_sp (not parity_sp) away
    buf = torch.from_numpy(uni.copy()).cuda()
    buf[:, k:, :] = 0xEE
    eng.encode_unified(buf, S, P, N)
    torch.cuda.synchronize()
    out = buf.cpu().numpy()
    assert np.array_equal(out[:, k:, :S], uni[:, k:, :S])
    assert (out[:, k:, S:] == 0xEE).all()


@pytest.mark.parametrize("k,m,S,P", [(10, 4, 6554, 6656), (10, 4, 6554, 6912), (8, 4, 2049, 2304),
                                     (4, 2, 1000, 1280), (4, 2, 1000, 1008), (10, 4, 6656, 6656)])
def test_parity_pad_writes(engines, k, m, S, P):
    """rs_set_parity_pad_writes: encode writes parity bytes [S, min(P, round_up(S, 128)))
    -- the code of the data padding -- and nothing past that; reconstruct is unaffected."""
    import torch

    eng = eng_for(engines, k, m)
    N = 23
    s_eff = min(P, (S + 127) // 128 * 128)
    g = torch.Generator(device="cuda").manual_seed(S + P + k)
    data = torch.randint(0, 256, (N, k, P), dtype=torch.uint8, device="cuda", generator=g)
    parity = torch.full((N, m, P), 0xEE, dtype=torch.uint8, device="cuda")
    eng.set_parity_pad_writes(True)
    try:
        eng.encode(data, parity, S, N, shard_pitch=P)
        torch.cuda.synchronize()
        uni = np.zeros((N, k + m, P), np.uint8)
        uni[:, :k] = data.cpu().numpy()
        rs_oracle.encode_batch_scalar(k, m, uni.reshape(-1), (k + m) * P, P, s_eff, N)
        par = parity.cpu().numpy()
        assert np.array_equal(par[:, :, :s_eff], uni[:, k:, :s_eff])
        assert (par[:, :, s_eff:] == 0xEE).all(), "written past the 128-B line / pitch"
        # per-stripe reconstruct with the option on still writes exactly S bytes
        d2, p2 = data.clone(), parity.clone()
        d2[:, 1, :] = 0x55
        p2[:, 0, :] = 0x55
        t = k + m
        eng.reconstruct(d2, p2, S, N, np.full(N, ((1 << t) - 1) & ~((1 << 1) | (1 << k)), np.uint32),
                        shard_pitch=P)
        torch.cuda.synchronize()
        assert torch.equal(d2[:, :, :S], data[:, :, :S]) and torch.equal(p2[:, :, :S], parity[:, :, :S])
        assert (d2[:, 1, S:] == 0x55).all() and (p2[:, 0, S:] == 0x55).all()
    finally:
        eng.set_parity_pad_writes(False)


@pytest.mark.parametrize("zero_copy", [True, False])
@pytest.mark.parametrize("S", [6560, 6554])
def test_flat_kernels_host(engines, S, zero_copy):
    """The flat-task encode and scrub kernels on host-resident batches with no slot
    padding (P = S): zero-copy (the kernels address rs_host_alloc'ed memory through
    their buffer descriptors) and staged."""
    k, m = 10, 4
    eng = eng_for(engines, k, m)
    N = 203
    P = S
    rng = np.random.default_rng(S + zero_copy)
    data = _host_mem(eng, "alloc", (N, k, P))
    data[:] = rng.integers(0, 256, (N, k, P), dtype=np.uint8)
    parity = _host_mem(eng, "alloc", (N, m, P))
    eng.set_host_zero_copy(zero_copy)
    path = "zero-copy" if zero_copy and S % 16 == 0 else "staged"
    try:
        eng.encode_host(data, parity, S, N)
        assert eng.last_host_path() == path
        assert any(n in eng.last_kernel() for n in ("bitsliced", "bs16")), eng.last_kernel()
        uni = np.concatenate([data, np.zeros_like(parity)], axis=1).copy()
        rs_oracle.encode_batch_scalar(k, m, uni.reshape(-1), (k + m) * P, P, S, N)
        assert np.array_equal(parity, uni[:, k:])
        assert not eng.verify_host(data, parity, S, N).any()
        assert eng.last_kernel().startswith("verify_flat_kernel"), eng.last_kernel()
        for i, b in [(0, 0), (1, S - 1), (100, S // 2), (N - 1, S - 1)]:
            parity[i, 3, b] ^= 0x40
        bad = eng.verify_host(data, parity, S, N)
        assert np.array_equal(np.nonzero(bad)[0], [0, 1, 100, N - 1]) and (bad[bad != 0] == 8).all()
    finally:
        eng.set_host_zero_copy(True)
        eng.host_free(data)
        eng.host_free(parity)


@pytest.mark.parametrize("k,m", [(10, 4), (8, 4), (4, 2), (6, 3)])
@pytest.mark.parametrize("S,N", [(1040, 37), (2049, 3), (6554, 1), (6554, 29), (10923, 5)])
def test_flat_reconstruct_tasks(engines, k, m, S, N):
    """Per-stripe out-of-place reconstruct on ragged shard lengths (flat 64-column
    tasks that straddle stripes): neighbours with equal and with different erasure
    patterns, complete stripes, and invalid stripes (> m missing) next to valid ones
    -- the invalid ones write nothing and the call reports "too few shards given"."""
    import torch

    eng = eng_for(engines, k, m)
    t = k + m
    P = shard_pitch_for(S)
    g = torch.Generator(device="cuda").manual_seed(S * 3 + N + k)
    data = torch.randint(0, 256, (N, k, P), dtype=torch.uint8, device="cuda", generator=g)
    parity = torch.empty((N, m, P), dtype=torch.uint8, device="cuda")
    eng.encode(data, parity, S, N)
    ref = torch.cat([data, parity], dim=1).cpu().numpy()
    rng = np.random.default_rng(S + N + t)
    masks = _masks_upto(rng, N, t, m)
    for i in range(0, N - 1, 4):
        masks[i + 1] = masks[i]  # equal patterns across some boundaries
    invalid = []
    if N >= 3:
        invalid = [N // 2]
        masks[N // 2] = (1 << k) - 1 - 1  # k-1 present: too few
    out = torch.full((N, m, P), 0xC3, dtype=torch.uint8, device="cuda")
    eng.reconstruct_out(data, parity, out, S, N, masks_dev=torch.from_numpy(masks.view(np.int32)).cuda())
    if invalid:
        with pytest.raises(ECError, match="too few shards given"):
            eng.sync()
    else:
        eng.sync()
    torch.cuda.synchronize()
    kname = eng.last_kernel()
    cols = -(-S // 16)
    assert ("flat_seg" in kname) == (cols >= 64 and cols % 64 != 0), kname
    got = out.cpu().numpy()
    for i in range(N):
        if i in invalid:
            assert (got[i] == 0xC3).all(), "an invalid stripe writes nothing"
            continue
        missing = [j for j in range(t) if not (masks[i] >> j) & 1]
        for r, j in enumerate(missing):
            assert np.array_equal(got[i, r, :S], ref[i, j, :S]), (kname, i, r, j)
        for r in range(len(missing), m):
            assert (got[i, r] == 0xC3).all(), "unused output slots untouched"
    assert (got[:, :, _pad_end(S, P):] == 0xC3).all(), "output padding untouched"


@pytest.mark.parametrize("k,m", [(10, 4), (8, 4), (4, 2), (6, 3)])
@pytest.mark.parametrize("S,N", [(1040, 37), (6554, 29), (10923, 5)])
def test_flat_reconstruct_inplace(engines, k, m, S, N):
    """In-place per-stripe reconstruct (device masks) on ragged shard lengths: every
    missing slot refilled with its original bytes, in the data and the parity region,
    nothing past S written, invalid stripes left alone.  (In place runs the
    stripe-aligned kernel: an in-place flat-task form measured 5 points slower,
    profiles/r02c_ab_flat_ps_inplace_rejected.log.)"""
    import torch

    eng = eng_for(engines, k, m)
    t = k + m
    P = shard_pitch_for(S)
    g = torch.Generator(device="cuda").manual_seed(S * 5 + N + k)
    data = torch.randint(0, 256, (N, k, P), dtype=torch.uint8, device="cuda", generator=g)
    parity = torch.empty((N, m, P), dtype=torch.uint8, device="cuda")
    eng.encode(data, parity, S, N)
    rng = np.random.default_rng(S * 7 + N + t)
    masks = _masks_upto(rng, N, t, m)
    for i in range(0, N - 1, 5):
        masks[i + 1] = masks[i]
    inv = N // 3
    masks[inv] = (1 << t) - 1 - sum(1 << j for j in range(m + 1))  # m+1 missing: too few
    lost = ((masks[:, None] >> np.arange(t)[None, :]) & 1) == 0
    d2, p2 = data.clone(), parity.clone()
    d2[torch.from_numpy(lost[:, :k]).cuda()] = 0x33
    p2[torch.from_numpy(lost[:, k:]).cuda()] = 0x33
    eng.reconstruct_devmask(d2, p2, S, N, torch.from_numpy(masks.view(np.int32)).cuda())
    with pytest.raises(ECError, match="too few shards given"):
        eng.sync()
    torch.cuda.synchronize()
    ok = np.ones(N, bool)
    ok[inv] = False
    okt = torch.from_numpy(ok).cuda()
    assert torch.equal(d2[okt][:, :, :S], data[okt][:, :, :S])
    assert torch.equal(p2[okt][:, :, :S], parity[okt][:, :, :S])
    # padding past S of refilled slots keeps the 0x33 fill; the invalid stripe is untouched
    assert (d2[okt][:, :, S:][torch.from_numpy(lost[ok, :k]).cuda()] == 0x33).all()
    assert (p2[okt][:, :, S:][torch.from_numpy(lost[ok, k:]).cuda()] == 0x33).all()
    li = torch.from_numpy(lost[inv]).cuda()
    assert (torch.cat([d2[inv], p2[inv]])[li] == 0x33).all()


@pytest.mark.parametrize("k,m", [(10, 4), (8, 4), (6, 3)])
@pytest.mark.parametrize("S,N", [(6554, 29), (1040, 9), (10923, 4)])
def test_flat_reconstruct_host_masks_e2(engines, k, m, S, N):
    """Host masks of at most 2 erasures on ragged shard lengths: the batch is sized
    for 2 outputs (the flat-task kernel's E = 2 form); straddling stripes with equal
    and different patterns."""
    import torch

    eng = eng_for(engines, k, m)
    t = k + m
    P = shard_pitch_for(S)
    g = torch.Generator(device="cuda").manual_seed(S * 11 + N + k)
    data = torch.randint(0, 256, (N, k, P), dtype=torch.uint8, device="cuda", generator=g)
    parity = torch.empty((N, m, P), dtype=torch.uint8, device="cuda")
    eng.encode(data, parity, S, N)
    ref = torch.cat([data, parity], dim=1).cpu().numpy()
    rng = np.random.default_rng(S + N * 3 + t)
    masks = _masks_upto(rng, N, t, 2)
    masks[0] = ((1 << t) - 1) & ~0b11  # at least one 2-erasure stripe
    for i in range(1, N - 1, 3):
        masks[i + 1] = masks[i]
    out = torch.full((N, m, P), 0xC3, dtype=torch.uint8, device="cuda")
    eng.reconstruct_out(data, parity, out, S, N, present_masks=masks)
    torch.cuda.synchronize()
    cols = -(-S // 16)
    assert ("flat_seg" in eng.last_kernel()) == (cols % 64 != 0), eng.last_kernel()
    got = out.cpu().numpy()
    for i in range(N):
        missing = [j for j in range(t) if not (masks[i] >> j) & 1]
        for r, j in enumerate(missing):
            assert np.array_equal(got[i, r, :S], ref[i, j, :S]), (i, r, j)
        for r in range(len(missing), m):
            assert (got[i, r] == 0xC3).all()
    assert (got[:, :, _pad_end(S, P):] == 0xC3).all()
