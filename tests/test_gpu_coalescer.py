"""Batch coalescer (rs_coalescer_*, rs_co_*): concurrent per-object IEcDriver calls
merged into device batches must give exactly the per-object results and errors.

Contract mirrored: internal/ec/ec.go:54-61 called from a goroutine per request
(writeservice.go:218-222, readservice.go:144,285) and healer workers
(poller.go:282).  Checked against the CPU oracle.
"""
import threading

import numpy as np
import pytest

from oracle import rs_oracle
from replication_erasurecoding_object_store_amd.coalescer import CoalescingService
from replication_erasurecoding_object_store_amd.ec import ECError, ErrShardNoData, ErrShardSize, ErrTooFewShards
from replication_erasurecoding_object_store_amd.xoshiro import xoshiro_bytes

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(300)]


def _run_threads(n, fn):
    errs = []

    def wrap(t):
        try:
            fn(t)
        except Exception as e:  # surfaced below
            errs.append(e)

    ts = [threading.Thread(target=wrap, args=(t,)) for t in range(n)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    if errs:
        raise errs[0]


@pytest.mark.parametrize("staged_dma", [False, True])
@pytest.mark.parametrize("k,m", [(4, 2), (10, 4), (17, 3)])
def test_concurrent_mixed_ops_match_oracle(gpu, k, m, staged_dma):
    svc = CoalescingService(k, m, max_batch=64, max_wait_us=500, inflight=3, staged_dma=staged_dma)
    try:
        sizes = [4096, 1000, 65536 + 5]

        def worker(t):
            rng = np.random.default_rng(t)
            for j in range(12):
                length = sizes[(t + j) % len(sizes)]
                data = xoshiro_bytes(t * 1000 + j, length)
                shards = svc.Split(data)
                ref = rs_oracle.split(k, m, data)
                assert rs_oracle.encode(k, m, ref) == 0
                svc.Encode(shards)
                assert [bytes(s) for s in shards] == [bytes(s) for s in ref]
                assert svc.Verify(shards)
                # erase 0..m shards, full Reconstruct then ReconstructData
                lost = rng.choice(k + m, size=int(rng.integers(0, m + 1)), replace=False)
                got = [None if i in lost else bytearray(s) for i, s in enumerate(shards)]
                svc.Reconstruct(got)
                assert [bytes(s) for s in got] == [bytes(s) for s in ref]
                got = [None if i in lost else bytearray(s) for i, s in enumerate(shards)]
                svc.ReconstructData(got)
                for i in range(k + m):
                    if i < k or i not in lost:
                        assert bytes(got[i]) == bytes(ref[i])
                    else:
                        assert got[i] is None, "ReconstructData leaves parity nil"
                # bit rot in one parity shard -> Verify false
                bad = [bytearray(s) for s in shards]
                bad[k + int(rng.integers(0, m))][int(rng.integers(0, len(bad[k])))] ^= 0x10
                assert not svc.Verify(bad)

        _run_threads(16, worker)
        st = svc.stats()
        assert st["calls"] > 0 and 0 < st["batches"] <= st["calls"]
        assert st["max_batch"] <= 64
    finally:
        svc.close()


def test_batch_fills_then_closes(gpu):
    """16 callers, max_batch 16, a long wait: one launch carries all 16."""
    svc = CoalescingService(4, 2, max_batch=16, max_wait_us=2_000_000, inflight=2)
    try:
        barrier = threading.Barrier(16)
        out = [None] * 16

        def worker(t):
            shards = svc.Split(xoshiro_bytes(0x5EED0002 + t, 4096))
            barrier.wait()
            svc.Encode(shards)
            out[t] = shards

        _run_threads(16, worker)
        st = svc.stats()
        assert st == {"calls": 16, "batches": 1, "stripes": 16, "max_batch": 16}
        for t in range(16):
            ref = rs_oracle.split(4, 2, xoshiro_bytes(0x5EED0002 + t, 4096))
            rs_oracle.encode(4, 2, ref)
            assert [bytes(s) for s in out[t]] == [bytes(s) for s in ref]
    finally:
        svc.close()


@pytest.mark.parametrize("data_only", [False, True])
def test_plan_mode_coalesces_reconstruct(gpu, data_only):
    """k+m > 16 (no all-pattern LUT): 16 concurrent Reconstruct / ReconstructData
    calls with 16 different erasure patterns still ride one launch, each object with
    its own plan, and match the oracle."""
    k, m = 17, 3
    svc = CoalescingService(k, m, max_batch=16, max_wait_us=2_000_000, inflight=2)
    try:
        barrier = threading.Barrier(16)
        refs, outs, losts = [None] * 16, [None] * 16, [None] * 16

        def worker(t):
            ref = rs_oracle.split(k, m, xoshiro_bytes(0x5EED0017 + t, 5000 + 7 * t))
            rs_oracle.encode(k, m, ref)
            rng = np.random.default_rng(t)
            lost = set(rng.choice(k + m, size=1 + t % m, replace=False).tolist())
            got = [None if i in lost else bytearray(s) for i, s in enumerate(ref)]
            barrier.wait()
            (svc.ReconstructData if data_only else svc.Reconstruct)(got)
            refs[t], outs[t], losts[t] = ref, got, lost

        _run_threads(16, worker)
        # objects of 16 different lengths: one batch per shard length
        for ref, got, lost in zip(refs, outs, losts):
            for i in range(k + m):
                if data_only and i >= k and i in lost:
                    assert got[i] is None
                else:
                    assert bytes(got[i]) == bytes(ref[i])
        # same length, different patterns: one launch
        svc2 = CoalescingService(k, m, max_batch=16, max_wait_us=2_000_000, inflight=2)
        try:
            barrier2 = threading.Barrier(16)
            ok = [False] * 16

            def worker2(t):
                ref = rs_oracle.split(k, m, xoshiro_bytes(0x5EED0117 + t, 17 * 300))
                rs_oracle.encode(k, m, ref)
                lost = {t % (k + m), (t + 5) % (k + m)}
                got = [None if i in lost else bytearray(s) for i, s in enumerate(ref)]
                barrier2.wait()
                (svc2.ReconstructData if data_only else svc2.Reconstruct)(got)
                ok[t] = all((data_only and i >= k and i in lost and got[i] is None) or bytes(got[i]) == bytes(ref[i])
                            for i in range(k + m))

            _run_threads(16, worker2)
            assert all(ok)
            assert svc2.stats() == {"calls": 16, "batches": 1, "stripes": 16, "max_batch": 16}
        finally:
            svc2.close()
    finally:
        svc.close()


def test_errors_identical_to_per_object(gpu):
    svc = CoalescingService(4, 2, max_wait_us=0)
    try:
        with pytest.raises(ECError) as e:
            svc.Encode([bytearray(8)] * 5)
        assert e.value.code == ErrTooFewShards
        with pytest.raises(ECError) as e:
            svc.Encode([bytearray(8)] * 5 + [bytearray(7)])
        assert e.value.code == ErrShardSize and str(e.value) == "shard sizes do not match"
        with pytest.raises(ECError) as e:
            svc.Encode([bytearray()] * 6)
        assert e.value.code == ErrShardNoData
        with pytest.raises(ECError) as e:
            svc.Reconstruct([bytearray(8), None, None, None, bytearray(8), bytearray(8)])
        assert e.value.code == ErrTooFewShards and str(e.value) == "too few shards given"
        full = [bytearray(8) for _ in range(6)]
        svc.Reconstruct(full)  # nothing missing: no-op
        assert svc.stats()["batches"] == 0, "rejected and no-op calls never reach the device"
    finally:
        svc.close()


@pytest.mark.parametrize("k,m", [(4, 2), (10, 4), (17, 3)])
def test_reconstruct_many_matches_oracle(gpu, k, m):
    """rs_co_reconstruct_many: per object exactly Reconstruct's result / error."""
    svc = CoalescingService(k, m, max_batch=50)
    try:
        rng = np.random.default_rng(k)
        objs, refs, expect_err = [], [], []
        for i in range(300):
            length = int(rng.choice([1, 100, 4096, 65536, 5000]))
            ref = rs_oracle.split(k, m, xoshiro_bytes(i, length))
            rs_oracle.encode(k, m, ref)
            nlost = int(rng.integers(0, m + 2))  # m+1 erasures -> too few shards
            lost = set(rng.choice(k + m, size=nlost, replace=False).tolist())
            objs.append([None if j in lost else bytearray(s) for j, s in enumerate(ref)])
            refs.append(ref)
            expect_err.append(nlost > m)
        objs.append([bytearray(4)] * (k + m - 1))  # wrong shard count
        errs = svc.ReconstructMany(objs)
        assert errs[-1] is not None and errs[-1].code == ErrTooFewShards
        for o, ref, bad, err in zip(objs, refs, expect_err, errs):
            if bad:
                assert err is not None and err.code == ErrTooFewShards
            else:
                assert err is None
                assert [bytes(s) for s in o] == [bytes(s) for s in ref]
        st = svc.stats()
        assert st["batches"] < 300 and st["max_batch"] <= 50
        # EncodeMany
        enc = [rs_oracle.split(k, m, xoshiro_bytes(1000 + i, 3000 + i)) for i in range(40)]
        mine = [[bytearray(s) for s in e] for e in enc]
        assert svc.EncodeMany(mine) == [None] * 40
        for e, o in zip(enc, mine):
            rs_oracle.encode(k, m, e)
            assert [bytes(s) for s in o] == [bytes(s) for s in e]
    finally:
        svc.close()


def test_batch_healer_poller_semantics(gpu):
    """cmd/healer/poller.go:227-309 rules over a scan's audits, repaired in batch."""
    from replication_erasurecoding_object_store_amd.healer import DATA_LOSS, HEALTHY, REPAIRED, BatchHealer

    svc = CoalescingService(4, 2)
    try:
        healer = BatchHealer(svc)
        audits, fulls = [], []
        rng = np.random.default_rng(0x5EED0005)
        for i in range(200):
            full = rs_oracle.split(4, 2, xoshiro_bytes(0x5EED0005 + i, 4096))
            rs_oracle.encode(4, 2, full)
            nlost = [0, 1, 2, 3][i % 4]
            lost = set(rng.choice(6, size=nlost, replace=False).tolist())
            audits.append((f"metadata/obj{i}", [None if j in lost else bytes(s) for j, s in enumerate(full)]))
            fulls.append((full, sorted(lost)))
        res = healer.repair(audits)
        for r, (full, lost) in zip(res, fulls):
            if not lost:
                assert r.status == HEALTHY
            elif len(lost) > 2:
                assert r.status == DATA_LOSS and r.error == "critical data loss: not enough shards"
            else:
                assert r.status == REPAIRED and sorted(r.repaired) == lost == r.missing
                for j in lost:
                    assert r.repaired[j] == bytes(full[j])
        assert svc.stats()["batches"] == 1, "100 repairs of one shard length -> one launch"
    finally:
        svc.close()


@pytest.mark.parametrize("max_batch,inflight", [(5, 2), (64, 4), (4096, 16)])
def test_reservation_stress(gpu, max_batch, inflight):
    """64 threads x 60 encodes of two interleaved shard lengths: the lock-free slot
    reservation (CAS ticket, hot batch), full-batch closes and batch recycling
    under contention; every result checked, every call accounted for."""
    svc = CoalescingService(4, 2, max_batch=max_batch, inflight=inflight)
    try:
        refs = {}
        for length in (4096, 1000):
            data = xoshiro_bytes(length, length)
            ref = rs_oracle.split(4, 2, data)
            rs_oracle.encode(4, 2, ref)
            refs[length] = (data, [bytes(x) for x in ref])

        def worker(t):
            for j in range(60):
                length = 4096 if (t + j) % 3 else 1000
                data, ref = refs[length]
                shards = svc.Split(data)
                svc.Encode(shards)
                assert [bytes(x) for x in shards] == ref

        _run_threads(64, worker)
        st = svc.stats()
        assert st["calls"] == 64 * 60 and st["stripes"] == 64 * 60
        assert st["max_batch"] <= max_batch
    finally:
        svc.close()


def test_many_and_single_callers_share_batches(gpu):
    """Multi-object calls (one caller holding many slots, so whole wake-up groups
    with no sleeper) interleaved with single-object callers in the same batches:
    every caller must be woken and get its own bytes."""
    svc = CoalescingService(4, 2, max_batch=64, max_wait_us=200, inflight=4)
    try:
        def worker(t):
            for j in range(20):
                if t % 4 == 0:
                    objs = [rs_oracle.split(4, 2, xoshiro_bytes(t * 1000 + j * 50 + i, 4096)) for i in range(13)]
                    mine = [[bytearray(s) for s in o] for o in objs]
                    assert svc.EncodeMany(mine) == [None] * 13
                    for o, got in zip(objs, mine):
                        rs_oracle.encode(4, 2, o)
                        assert [bytes(s) for s in got] == [bytes(s) for s in o]
                else:
                    data = xoshiro_bytes(t * 1000 + j, 4096)
                    sh = svc.Split(data)
                    svc.Encode(sh)
                    ref = rs_oracle.split(4, 2, data)
                    rs_oracle.encode(4, 2, ref)
                    assert [bytes(s) for s in sh] == [bytes(s) for s in ref]

        _run_threads(48, worker)
        st = svc.stats()
        assert st["stripes"] == 12 * 20 * 13 + 36 * 20
    finally:
        svc.close()


@pytest.mark.parametrize("staged_dma", [False, True])
@pytest.mark.parametrize("k,m", [(4, 2), (10, 4), (17, 3)])
def test_encode_hash_matches_hashlib_and_oracle(gpu, k, m, staged_dma):
    """rs_co_encode_hash: the write path's Split -> Encode -> cold_hash
    (writeservice.go:218-222, :267) in one coalesced batch.  Parity = the oracle's,
    digest = hashlib.sha256(value), for values whose shard length is and is not a
    multiple of 16 (the staged shards then sit at a 16-B pitch with gaps: the
    kernel reads the value across them), mixed in batches with plain encodes and
    reconstructs from concurrent callers."""
    import hashlib

    svc = CoalescingService(k, m, max_batch=48, max_wait_us=300, inflight=3, staged_dma=staged_dma)
    try:
        sizes = [1, 2, 3, 63, 64, 65, 1000, 4096, 4097, 10 * 1024 + 7, 100 * 1024, 65536 + 5]

        def worker(t):
            rng = np.random.default_rng(100 + t)
            for j in range(len(sizes)):
                length = sizes[(t + j) % len(sizes)]
                data = xoshiro_bytes(t * 7919 + j, length)
                shards = svc.Split(data)
                ref = rs_oracle.split(k, m, data)
                assert rs_oracle.encode(k, m, ref) == 0
                if j % 3 == 2:  # a plain encode / a repair in the same batches
                    svc.Encode(shards)
                    gone = int(rng.integers(0, k + m))
                    got = [None if i == gone else bytearray(s) for i, s in enumerate(shards)]
                    svc.Reconstruct(got)
                    assert [bytes(s) for s in got] == [bytes(s) for s in ref]
                    continue
                digest = svc.EncodeHash(shards, len(data))
                assert [bytes(s) for s in shards] == [bytes(s) for s in ref], (length, "parity")
                assert digest == hashlib.sha256(data).digest(), (length, "cold_hash")

        _run_threads(8, worker)
        # many objects in one call; value_len may stop short of the padded shards
        objs, vals = [], []
        for i, length in enumerate(sizes):
            data = xoshiro_bytes(555 + i, length)
            objs.append(svc.Split(data))
            vals.append(data)
        res = svc.EncodeHashMany(objs, [len(v) for v in vals])
        for (err, dig), data, sh in zip(res, vals, objs):
            assert err is None and dig == hashlib.sha256(data).digest()
            ref = rs_oracle.split(k, m, data)
            assert rs_oracle.encode(k, m, ref) == 0
            assert [bytes(s) for s in sh] == [bytes(s) for s in ref]
        # a value_len past the k data shards is rejected, nothing written
        sh = svc.Split(b"abc" * 100)
        with pytest.raises(ECError):
            svc.EncodeHash(sh, k * len(sh[0]) + 1)
    finally:
        svc.close()


@pytest.mark.parametrize("k,m", [(4, 2), (10, 4), (17, 3)])
def test_async_submit_reap_matches_oracle(gpu, k, m):
    """rs_co_submit_encode / rs_co_submit_reconstruct / rs_co_reap: many calls in
    flight from few threads (how an event loop or the Go runtime multiplexes
    request goroutines), every output checked against the oracle once reaped;
    RS_ERR_BUSY when all staging batches hold unreaped calls, after which reaping
    and resubmitting goes on; rejected calls are never reaped."""
    import ctypes

    from replication_erasurecoding_object_store_amd import _lib
    from replication_erasurecoding_object_store_amd.ec import _shard_array

    L = _lib.lib()
    svc = CoalescingService(k, m, max_batch=32, inflight=3)
    try:
        t = k + m
        rng = np.random.default_rng(k * 100 + m)
        pending = {}  # tag -> (kind, shards, expected, keepalive)
        done = 0
        busy = 0
        tags = (ctypes.c_uint64 * 64)()
        rcs = (ctypes.c_int * 64)()

        def reap(timeout):
            nonlocal done
            n = L.rs_co_reap(svc._co, tags, rcs, 64, timeout)
            assert n >= 0
            for i in range(n):
                kind, sh, exp, keep = pending.pop(tags[i])
                assert rcs[i] == _lib.RS_OK
                assert [bytes(x) for x in sh] == exp, (kind, tags[i])
                done += 1
            return n

        for tag in range(400):
            length = [4096, 1000, 65536 + 5, 3][tag % 4]
            data = xoshiro_bytes(9000 + tag, length)
            ref = rs_oracle.split(k, m, data)
            assert rs_oracle.encode(k, m, ref) == 0
            exp = [bytes(x) for x in ref]
            sh = svc.Split(data)
            lost = []
            if tag % 2 == 0:
                kind = "encode"
                for j in range(k, t):
                    sh[j][:] = b"\x5a" * len(sh[j])
            else:
                kind = "reconstruct"
                sh = [bytearray(x) for x in ref]
                lost = [int(j) for j in rng.choice(t, size=int(rng.integers(1, m + 1)), replace=False)]
                for j in lost:
                    sh[j][:] = b"\x00" * len(sh[j])  # storage stays; len 0 marks it missing
            S = len(sh[0])
            ptrs, lens, keep = _shard_array(sh, S, fill_missing=False)
            for j in lost:
                lens[j] = 0
            fn = L.rs_co_submit_encode if kind == "encode" else L.rs_co_submit_reconstruct
            while True:
                rc = fn(svc._co, ptrs, lens, tag)
                if rc != _lib.RS_ERR_BUSY:
                    break
                busy += 1
                reap(-1)
            assert rc == _lib.RS_OK, rc
            pending[tag] = (kind, sh, exp, (ptrs, lens, keep))
        while pending:
            reap(-1)
        assert done > 300 and busy > 0, (done, busy)
        # a rejected call (shard sizes differ) returns its code and is never reaped
        sh = svc.Split(b"x" * 100)
        sh[1] = bytearray(len(sh[1]) + 1)
        ptrs, lens, keep = _shard_array(sh, 0, fill_missing=False)
        assert L.rs_co_submit_encode(svc._co, ptrs, lens, 7) == _lib.RS_ERR_SHARD_SIZE
        assert L.rs_co_reap(svc._co, tags, rcs, 64, 0) == 0
    finally:
        svc.close()


@pytest.mark.parametrize("k,m,S,mem", [(4, 2, 100000, "register"), (10, 4, 6554, "register"), (4, 2, 1001, "register"),
                                       (8, 4, 384000, "register"), (6, 3, 777, "register"),
                                       (4, 2, 100000, "alloc"), (10, 4, 6554, "alloc"),
                                       # tiny shards: partial first column, byte-exact stores
                                       (4, 2, 1, "alloc"), (4, 2, 3, "alloc"), (10, 4, 17, "register")])
def test_owned_buffers_run_in_place_registered_staged(gpu, k, m, S, mem):
    """mem="alloc": objects whose shards lie in context-owned page-locked memory
    (rs_host_alloc: request bodies and storage-node reads in an arena, SURVEY.md §8f
    rank 4) are encoded and reconstructed by the coalescer in place -- the
    pointer-table kernel reads and writes the caller's buffers, nothing is staged --
    with the oracle's bytes and no byte outside [0, S) of any shard written; pageable
    objects join the same batches (staged).  Asynchronous calls run in place too
    (nothing left to copy at reap).  mem="register": the same calls on
    rs_host_register'ed memory are staged (round 4: no kernel touches caller pages
    in place), same bytes, same guard bytes."""
    import ctypes
    import mmap

    from replication_erasurecoding_object_store_amd import _lib

    L = _lib.lib()
    t = k + m
    n_obj = 24
    P = (S + 15) // 16 * 16 + 48  # 16-B aligned shards, guard bytes between them
    nbytes = n_obj * t * P + 4096
    svc = CoalescingService(k, m, max_wait_us=3000)
    if mem == "alloc":
        p = ctypes.c_void_p()
        assert L.rs_host_alloc(svc._ctx, nbytes, ctypes.byref(p)) == 0
        base = p.value
        arr = np.ctypeslib.as_array((ctypes.c_uint8 * nbytes).from_address(base))
    else:
        region = mmap.mmap(-1, nbytes)
        arr = np.frombuffer(region, np.uint8)
        base = ctypes.addressof(ctypes.c_uint8.from_buffer(region))
    arr[:] = 0xA5
    rng = np.random.default_rng(k * 1000 + S)
    data = rng.integers(0, 256, (n_obj, k, S), dtype=np.uint8)
    want = np.zeros((n_obj, t, S), np.uint8)
    for i in range(n_obj):
        sh = [bytearray(data[i, c].tobytes()) for c in range(k)] + [bytearray(S) for _ in range(m)]
        assert rs_oracle.encode(k, m, sh) == 0
        want[i] = np.frombuffer(b"".join(sh), np.uint8).reshape(t, S)

    def view(i, s):
        return arr[(i * t + s) * P:(i * t + s) * P + S]

    def ptrs(i):
        return (_lib._u8p * t)(*[ctypes.cast(base + (i * t + s) * P, _lib._u8p) for s in range(t)])

    registered = False
    try:
        if mem == "register":
            assert L.rs_host_register(svc._ctx, base, nbytes) == 0
            registered = True
        for i in range(n_obj):
            for c in range(k):
                view(i, c)[:] = data[i, c]
        # encode: 24 registered objects and 8 pageable ones from 32 threads (batches mix both)
        pageable = [[bytearray(data[i, c].tobytes()) for c in range(k)] + [bytearray(S) for _ in range(m)]
                    for i in range(8)]

        def enc(tid):
            if tid < n_obj:
                lens = (ctypes.c_size_t * t)(*([S] * t))
                assert L.rs_co_encode(svc._co, ptrs(tid), lens) == _lib.RS_OK
            else:
                svc.Encode(pageable[tid - n_obj])

        _run_threads(n_obj + 8, enc)
        for i in range(n_obj):
            for s in range(t):
                assert np.array_equal(view(i, s), want[i, s]), ("encode", i, s)
        for i in range(8):
            assert [bytes(x) for x in pageable[i]] == [want[i, s].tobytes() for s in range(t)]
        # reconstruct: 1..m erased per object, their buffers scribbled; odd objects
        # blocking from threads, even ones asynchronous from this thread
        lost = [sorted(rng.choice(t, size=int(rng.integers(1, m + 1)), replace=False).tolist()) for _ in range(n_obj)]
        for i in range(n_obj):
            for s in lost[i]:
                view(i, s)[:] = 0x3C
        keep = []
        for i in range(0, n_obj, 2):
            p, lens = ptrs(i), (ctypes.c_size_t * t)(*[0 if s in lost[i] else S for s in range(t)])
            keep.append((p, lens))
            assert L.rs_co_submit_reconstruct(svc._co, p, lens, i) == _lib.RS_OK

        def rec(tid):
            i = 2 * tid + 1
            lens = (ctypes.c_size_t * t)(*[0 if s in lost[i] else S for s in range(t)])
            assert L.rs_co_reconstruct(svc._co, ptrs(i), lens) == _lib.RS_OK
            assert all(lens[s] == S for s in range(t))

        _run_threads(n_obj // 2, rec)
        tags = (ctypes.c_uint64 * 64)()
        rcs = (ctypes.c_int * 64)()
        reaped = set()
        while len(reaped) < n_obj // 2:
            n = L.rs_co_reap(svc._co, tags, rcs, 64, 1000000)
            assert n > 0
            for j in range(n):
                assert rcs[j] == _lib.RS_OK
                reaped.add(tags[j])
        assert reaped == set(range(0, n_obj, 2))
        assert ("apply_ptr_kernel" in L.rs_last_kernel(svc._ctx).decode()) == (mem == "alloc")
        for i in range(n_obj):
            for s in range(t):
                assert np.array_equal(view(i, s), want[i, s]), ("reconstruct", i, s, lost[i])
        # nothing outside the shards was written
        for i in range(n_obj * t):
            assert (arr[i * P + S:(i + 1) * P] == 0xA5).all(), ("guard", i)
        assert (arr[n_obj * t * P:] == 0xA5).all()
        if mem == "alloc":
            assert L.rs_host_unregister(svc._ctx, base) == _lib.RS_ERR_INVALID_ARG  # rs_host_free's
            assert L.rs_host_free(svc._ctx, base + 16) == _lib.RS_ERR_INVALID_ARG  # not an allocation
            assert L.rs_host_free(svc._ctx, base) == 0
            return
        # unregistered: the same memory is staged, same bytes
        assert L.rs_host_unregister(svc._ctx, base) == 0
        registered = False
        for s in range(m):
            view(0, k + s)[:] = 0
        lens = (ctypes.c_size_t * t)(*([S] * t))
        assert L.rs_co_encode(svc._co, ptrs(0), lens) == _lib.RS_OK
        assert "apply_ptr_kernel" not in L.rs_last_kernel(svc._ctx).decode()
        for s in range(t):
            assert np.array_equal(view(0, s), want[0, s])
    finally:
        if registered:
            L.rs_host_unregister(svc._ctx, base)
        svc.close()


@pytest.mark.parametrize("k,m,S", [(4, 2, 25600), (10, 4, 1024)])
def test_in_place_calls_share_batches_with_staged_many_forms(gpu, k, m, S):
    """In-place objects (context-owned pinned memory, each object's K+M shards
    contiguous as Split carves them from one body) and staged objects of the same
    shard length in the same device batches: rs_co_encode_hash (in place, cold_hash
    read where the value lies) and rs_co_encode_hash_many / rs_co_encode_many on
    pageable objects from concurrent threads.  Every staged slot of a batch that runs
    the pointer-table kernel must carry its own pointer row; parity = the oracle's,
    digests = hashlib's, for every object."""
    import ctypes
    import hashlib

    from replication_erasurecoding_object_store_amd import _lib

    L = _lib.lib()
    t = k + m
    n_obj = 48
    svc = CoalescingService(k, m, max_wait_us=2000)
    p = ctypes.c_void_p()
    assert L.rs_host_alloc(svc._ctx, n_obj * t * S, ctypes.byref(p)) == 0
    base = p.value
    arena = np.ctypeslib.as_array((ctypes.c_uint8 * (n_obj * t * S)).from_address(base))
    try:
        rng = np.random.default_rng(k * 7 + S)
        vlen = [int(rng.integers(1, k * S + 1)) for _ in range(n_obj)]
        values = [rng.integers(0, 256, v, dtype=np.uint8).tobytes() for v in vlen]
        want = []
        for i in range(n_obj):  # Split into the arena: body = object i's region
            body = arena[i * t * S:(i + 1) * t * S]
            body[:] = 0
            body[:vlen[i]] = np.frombuffer(values[i], np.uint8)
            sh = [bytearray(body[c * S:(c + 1) * S].tobytes()) for c in range(k)] + [bytearray(S) for _ in range(m)]
            assert rs_oracle.encode(k, m, sh) == 0
            want.append([bytes(x) for x in sh])

        def ptrs(i):
            return (_lib._u8p * t)(*[ctypes.cast(base + (i * t + s) * S, _lib._u8p) for s in range(t)])

        lens = (ctypes.c_size_t * t)(*([S] * t))

        def in_place(tid):
            for i in range(tid, n_obj, 16):
                dig = (ctypes.c_uint8 * 32)()
                assert L.rs_co_encode_hash(svc._co, ptrs(i), lens, vlen[i], dig) == 0
                assert bytes(dig) == hashlib.sha256(values[i]).digest(), ("in place digest", i)

        def staged_many(tid):
            objs = [[bytearray(want[i][c]) if c < k else bytearray(S) for c in range(t)]
                    for i in range(tid, n_obj, 4)]
            idx = list(range(tid, n_obj, 4))
            keep = [(ctypes.c_uint8 * S).from_buffer(b) for o in objs for b in o]
            sp = (_lib._u8p * (len(objs) * t))(*[ctypes.cast(x, _lib._u8p) for x in keep])
            ls = (ctypes.c_size_t * (len(objs) * t))(*([S] * (len(objs) * t)))
            rcs = (ctypes.c_int * len(objs))()
            if tid % 2:
                assert L.rs_co_encode_many(svc._co, len(objs), sp, ls, rcs) == 0
            else:
                vl = (ctypes.c_size_t * len(objs))(*[vlen[i] for i in idx])
                digs = (ctypes.c_uint8 * (32 * len(objs)))()
                assert L.rs_co_encode_hash_many(svc._co, len(objs), sp, ls, vl, digs, rcs) == 0
                for j, i in enumerate(idx):
                    assert bytes(digs[32 * j:32 * j + 32]) == hashlib.sha256(values[i]).digest(), ("many digest", i)
            assert list(rcs) == [0] * len(objs)
            for j, i in enumerate(idx):
                assert [bytes(x) for x in objs[j]] == want[i], ("staged many parity", i)

        _run_threads(20, lambda tid: in_place(tid) if tid < 16 else staged_many(tid - 16))
        for i in range(n_obj):
            for s in range(t):
                got = arena[(i * t + s) * S:(i * t + s + 1) * S].tobytes()
                assert got == want[i][s], ("in place parity", i, s)
        # the in-place forms of the _many calls too: every object in the arena
        for i in range(n_obj):
            arena[(i * t + k) * S:(i + 1) * t * S] = 0
        sp = (_lib._u8p * (n_obj * t))(*[ctypes.cast(base + j * S, _lib._u8p) for j in range(n_obj * t)])
        ls = (ctypes.c_size_t * (n_obj * t))(*([S] * (n_obj * t)))
        vl = (ctypes.c_size_t * n_obj)(*vlen)
        digs = (ctypes.c_uint8 * (32 * n_obj))()
        rcs = (ctypes.c_int * n_obj)()
        assert L.rs_co_encode_hash_many(svc._co, n_obj, sp, ls, vl, digs, rcs) == 0
        assert "apply_ptr_kernel" in L.rs_last_kernel(svc._ctx).decode()
        for i in range(n_obj):
            assert bytes(digs[32 * i:32 * i + 32]) == hashlib.sha256(values[i]).digest()
            for s in range(t):
                assert arena[(i * t + s) * S:(i * t + s + 1) * S].tobytes() == want[i][s]
        # a value whose data shards are not contiguous is hashed from the staging
        dig = (ctypes.c_uint8 * 32)()
        order = [1, 0] + list(range(2, t))  # (a ctypes pointer-array swap would alias)
        swapped = (_lib._u8p * t)(*[ctypes.cast(base + order[s] * S, _lib._u8p) for s in range(t)])
        v2 = arena[S:2 * S].tobytes() + arena[0:S].tobytes()
        assert L.rs_co_encode_hash(svc._co, swapped, lens, 2 * S, dig) == 0
        assert bytes(dig) == hashlib.sha256(v2).digest()
    finally:
        assert L.rs_host_free(svc._ctx, base) == 0
        svc.close()


def test_python_arena_encode_in_place(gpu):
    """The Python mirror's Arena (Service.NewArena, rs_host_alloc): Split's shards
    copied into arena views, Encode runs in place (pointer-table kernel), parity
    lands in the views; a degraded read with the survivors in the arena repairs the
    lost shards; oracle bytes throughout."""
    from replication_erasurecoding_object_store_amd import _lib

    k, m = 4, 2
    svc = CoalescingService(k, m, max_wait_us=200)
    arena = svc.NewArena(8 << 20)
    try:
        for n in (4096, 102400, 1001):
            arena.Reset()
            value = xoshiro_bytes(n, n)
            ref = rs_oracle.split(k, m, value)
            assert rs_oracle.encode(k, m, ref) == 0
            S = len(ref[0])
            views = [arena.Alloc(S) for _ in range(k + m)]
            for i in range(k):
                views[i][:] = ref[i]
            svc.Encode(views)
            # every view starts 16-B aligned: in place whatever S is (S = 251 for 1001 B)
            assert "apply_ptr_kernel" in _lib.lib().rs_last_kernel(svc.ctx).decode()
            assert [bytes(v) for v in views] == [bytes(r) for r in ref]
            got = list(views)
            got[1] = None
            got[5] = None
            svc.Reconstruct(got)
            assert [bytes(g) for g in got] == [bytes(r) for r in ref]
        assert arena.Alloc(16 << 20) is None
        with pytest.raises(TypeError):
            svc.Encode([bytes(8)] * (k + m))  # read-only buffers are refused
        # closing the service frees the arena's memory: its views are released first,
        # so a stale view raises instead of touching freed memory
        svc2 = CoalescingService(k, m)
        a2 = svc2.NewArena(4096)
        v2 = a2.Alloc(64)
        v2[:] = bytes(range(64))
        svc2.close()
        with pytest.raises(ValueError):
            v2[0]
        assert a2.Alloc(16) is None
        a2.Close()  # nothing left to free
        # one root view per arena: Alloc keeps only the slices it handed out, and
        # Reset forgets them (a long-lived arena does not grow a list per call)
        a3 = svc.NewArena(1 << 20)
        for _ in range(100):
            a3.Alloc(64)
        assert len(a3._views) == 100
        a3.Reset()
        assert a3._views == [] and a3.Alloc(1 << 20) is not None
        a3.Close()
    finally:
        arena.Close()
        svc.close()
