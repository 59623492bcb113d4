"""Several engines in one process, and per-stream state.

The reference builds ONE codec per process and shares it across every request
goroutine (cmd/api/main.go:206) and the healer's workers (cmd/healer/main.go:42,
poller.go:49), so the drop-in must serve several GPUs from one context and stay
correct when contexts and streams are used concurrently.  On a one-GPU box a
context over devices [0, 0] runs the multi-engine paths (fan-out of host batches,
least-busy dispatch, coalescer batches bound to engines) on two engines of the
same GPU.
"""
import threading

import numpy as np
import pytest

from oracle import rs_oracle
from replication_erasurecoding_object_store_amd.batch import BatchEngine, shard_pitch_for
from replication_erasurecoding_object_store_amd.coalescer import CoalescingService
from replication_erasurecoding_object_store_amd.ec import ECError, NewService
from replication_erasurecoding_object_store_amd.xoshiro import xoshiro_bytes

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(300)]


def _run_threads(n, fn):
    errs = []

    def wrap(i):
        try:
            fn(i)
        except Exception as e:  # surfaced below
            errs.append(e)

    ts = [threading.Thread(target=wrap, args=(i,)) for i in range(n)]
    for x in ts:
        x.start()
    for x in ts:
        x.join()
    if errs:
        raise errs[0]


def _oracle_parity(k, m, data_np, S):
    n = data_np.shape[0]
    buf = np.zeros((n, k + m, S), np.uint8)
    buf[:, :k] = data_np[:, :, :S]
    rs_oracle.encode_batch_scalar(k, m, buf.reshape(-1), (k + m) * S, S, S, n)
    return buf[:, k:]


def test_two_contexts_one_process_concurrent(gpu):
    """Two independent contexts (different codes) driven at once from two threads,
    each on its own torch stream, device batches and per-object calls mixed."""
    import torch

    engs = {(4, 2): BatchEngine(4, 2, 0), (10, 4): BatchEngine(10, 4, 0)}
    try:
        def work(i):
            k, m = list(engs)[i]
            eng = engs[(k, m)]
            S, N = 1000 + 554 * i, 3000
            P = shard_pitch_for(S)
            s = torch.cuda.Stream()
            g = torch.Generator(device="cuda").manual_seed(i)
            with torch.cuda.stream(s):
                data = torch.randint(0, 256, (N, k, P), dtype=torch.uint8, device="cuda", generator=g)
                parity = torch.empty((N, m, P), dtype=torch.uint8, device="cuda")
                for _ in range(3):
                    eng.encode(data, parity, S, N, stream=s)
            s.synchronize()
            assert np.array_equal(parity[:, :, :S].cpu().numpy(), _oracle_parity(k, m, data.cpu().numpy(), S))
            for j in range(20):
                obj = xoshiro_bytes(100 * i + j, 4096 + 37 * j)
                sh = eng.Split(obj)
                eng.Encode(sh)
                ref = rs_oracle.split(k, m, obj)
                rs_oracle.encode(k, m, ref)
                assert [bytes(x) for x in sh] == [bytes(x) for x in ref]

        _run_threads(2, work)
    finally:
        for e in engs.values():
            e.close()


def test_multi_engine_context_batches_and_objects(gpu):
    """rs_create_devices([0, 0]): host batches fan out over both engines (stripe
    ranges), per-object calls spread, results identical to the oracle."""
    import torch

    k, m, S, N = 4, 2, 1024, 40000  # 160 MB of user data: split over both engines
    eng = BatchEngine(k, m, [0, 0])
    try:
        assert eng.devices() == [0, 0]
        assert "x2" in eng.backend()
        P = shard_pitch_for(S)
        g = torch.Generator(device="cuda").manual_seed(9)
        src = torch.randint(0, 256, (N, k, P), dtype=torch.uint8, device="cuda", generator=g).cpu().numpy()
        for zc in (True, False):
            eng.set_host_zero_copy(zc)
            # zero-copy runs on the context's own page-locked memory (rs_host_alloc);
            # pageable memory is staged
            if zc:
                data = eng.host_alloc(N * k * P).reshape(N, k, P)
                parity = eng.host_alloc(N * m * P).reshape(N, m, P)
            else:
                data, parity = np.empty((N, k, P), np.uint8), np.empty((N, m, P), np.uint8)
            data[:] = src
            try:
                parity[:] = 0
                eng.encode_host(data, parity, S, N)
                assert eng.last_host_path() == ("zero-copy" if zc else "staged")
                sample = np.r_[0:64, N // 2 - 32:N // 2 + 32, N - 64:N]  # both engines' shares
                assert np.array_equal(parity[sample, :, :S], _oracle_parity(k, m, data[sample], S))
                # per-stripe repair masks across the whole batch
                rng = np.random.default_rng(zc)
                lost = rng.integers(0, k + m, N)
                masks = (((1 << (k + m)) - 1) & ~(1 << lost)).astype(np.uint32)
                d0, p0 = data.copy(), parity.copy()
                for i in range(N):
                    (data if lost[i] < k else parity)[i, lost[i] % k if lost[i] < k else lost[i] - k, :S] = 0
                eng.reconstruct_host(data, parity, S, N, masks)
                assert np.array_equal(data[:, :, :S], d0[:, :, :S]) and np.array_equal(parity[:, :, :S], p0[:, :, :S])
                # scrub: a flipped byte in the second engine's share is found at its index
                assert not eng.verify_host(data, parity, S, N).any()
                parity[N - 5, 1, 7] ^= 0x21
                bad = eng.verify_host(data, parity, S, N)
                assert np.nonzero(bad)[0].tolist() == [N - 5] and bad[N - 5] == 2
                parity[N - 5, 1, 7] ^= 0x21
            finally:
                if zc:
                    eng.host_free(data)
                    eng.host_free(parity)
        eng.set_host_zero_copy(True)

        # per-object calls from many threads: least-busy dispatch over both engines
        def obj(t):
            for j in range(15):
                b = xoshiro_bytes(1000 * t + j, 777 + 1000 * j)
                sh = eng.Split(b)
                eng.Encode(sh)
                ref = rs_oracle.split(k, m, b)
                rs_oracle.encode(k, m, ref)
                assert [bytes(x) for x in sh] == [bytes(x) for x in ref]
                got = [None if q in (t % 6, (t + 1) % 6) else bytearray(x) for q, x in enumerate(sh)]
                eng.Reconstruct(got)
                assert [bytes(x) for x in got] == [bytes(x) for x in ref]

        _run_threads(8, obj)
    finally:
        eng.close()


def test_multi_engine_coalescer(gpu):
    """The batch coalescer over a two-engine context: staging batches bound to
    both engines, every concurrent call's result identical to the oracle."""
    svc = CoalescingService(4, 2, [0, 0], max_batch=32, inflight=4)
    try:
        def worker(t):
            rng = np.random.default_rng(t)
            for j in range(25):
                b = xoshiro_bytes(t * 77 + j, 4096)
                sh = svc.Split(b)
                svc.Encode(sh)
                ref = rs_oracle.split(4, 2, b)
                rs_oracle.encode(4, 2, ref)
                assert [bytes(x) for x in sh] == [bytes(x) for x in ref]
                lost = rng.choice(6, size=2, replace=False)
                got = [None if q in lost else bytearray(x) for q, x in enumerate(sh)]
                svc.Reconstruct(got)
                assert [bytes(x) for x in got] == [bytes(x) for x in ref]

        _run_threads(32, worker)
        st = svc.stats()
        assert st["calls"] == 32 * 25 * 2 and st["stripes"] == st["calls"]
    finally:
        svc.close()


def test_multi_device_all_visible(gpu):
    """rs_create_multi(mask 0): every visible gfx950 GPU, one engine each."""
    import torch

    svc = NewService(device="all")
    try:
        assert svc.devices() == list(range(torch.cuda.device_count()))
        b = xoshiro_bytes(5, 5000)
        sh = svc.Split(b)
        svc.Encode(sh)
        ref = rs_oracle.split(4, 2, b)
        rs_oracle.encode(4, 2, ref)
        assert [bytes(x) for x in sh] == [bytes(x) for x in ref]
    finally:
        svc.close()


def test_device_calls_leave_callers_device_alone(gpu):
    """Library calls restore the calling thread's current HIP device."""
    import torch

    eng = BatchEngine(4, 2, 0)
    try:
        before = torch.cuda.current_device()
        sh = eng.Split(b"x" * 4000)
        eng.Encode(sh)
        assert torch.cuda.current_device() == before
    finally:
        eng.close()


def test_deferred_errors_are_per_stream(gpu):
    """rs_sync(A) reports only A's invalid device mask; B's sync stays clean, and A's
    error is cleared once reported (one status word served every stream)."""
    import torch

    k, m, S, N = 4, 2, 256, 64
    P = shard_pitch_for(S)
    eng = BatchEngine(k, m, 0)
    try:
        sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
        with torch.cuda.stream(sa):
            da = torch.randint(0, 256, (N, k, P), dtype=torch.uint8, device="cuda")
            pa = torch.empty((N, m, P), dtype=torch.uint8, device="cuda")
            bad_masks = torch.full((N,), 0b111111, dtype=torch.int32, device="cuda")
            bad_masks[5] = 0b000011  # 2 present < k: invalid
        with torch.cuda.stream(sb):
            db = torch.randint(0, 256, (N, k, P), dtype=torch.uint8, device="cuda")
            pb = torch.empty((N, m, P), dtype=torch.uint8, device="cuda")
            ok_masks = torch.full((N,), 0b111110, dtype=torch.int32, device="cuda")
        sa.synchronize()
        sb.synchronize()
        eng.encode(da, pa, S, N, stream=sa)
        eng.encode(db, pb, S, N, stream=sb)
        eng.reconstruct_devmask(da, pa, S, N, bad_masks, stream=sa)
        eng.reconstruct_devmask(db, pb, S, N, ok_masks, stream=sb)
        eng.sync(stream=sb)  # must not see A's error
        with pytest.raises(ECError, match="too few shards given"):
            eng.sync(stream=sa)
        eng.sync(stream=sa)  # reported once, then clear
    finally:
        eng.close()


def _hip_streams(n):
    """n distinct raw HIP streams (torch.cuda.Stream() hands out a small pool of
    reused handles), as torch ExternalStreams, and a destroyer."""
    import ctypes
    import importlib.util
    import os

    import torch

    hip = ctypes.CDLL(os.path.join(os.path.dirname(importlib.util.find_spec("torch").origin), "lib",
                                   "libamdhip64.so"))
    handles = []
    for _ in range(n):
        h = ctypes.c_void_p()
        assert hip.hipStreamCreate(ctypes.byref(h)) == 0
        handles.append(h)

    def destroy():
        for h in handles:
            hip.hipStreamDestroy(h)

    return [torch.cuda.ExternalStream(h.value) for h in handles], destroy


def test_deferred_errors_per_stream_beyond_1024_streams(gpu):
    """More streams than one status chunk (1 024 words): every stream keeps its own
    deferred-error word (streams past the 1 023rd shared the last word),
    and a released stream's word comes back clean to whichever stream gets it next."""
    import torch

    k, m, S, N = 4, 2, 256, 8
    P = shard_pitch_for(S)
    eng = BatchEngine(k, m, 0)
    streams, destroy = _hip_streams(1100)
    fresh, destroy2 = [], None
    try:
        d = torch.randint(0, 256, (N, k, P), dtype=torch.uint8, device="cuda")
        p = torch.empty((N, m, P), dtype=torch.uint8, device="cuda")
        eng.encode(d, p, S, N)
        good = torch.full((N,), 0b111110, dtype=torch.int32, device="cuda")
        bad = good.clone()
        bad[3] = 0b000011
        torch.cuda.synchronize()
        assert len({s.cuda_stream for s in streams}) == 1100
        for i, s in enumerate(streams):  # every 7th stream gets an invalid mask
            eng.reconstruct_devmask(d, p, S, N, bad if i % 7 == 0 else good, stream=s)
        for i, s in enumerate(streams):
            if i % 7 == 0:
                with pytest.raises(ECError, match="too few shards given"):
                    eng.sync(stream=s)
            else:
                eng.sync(stream=s)
        # release half of them with an error pending: the words come back zeroed
        for s in streams[:550]:
            eng.reconstruct_devmask(d, p, S, N, bad, stream=s)
            with pytest.raises(ECError):
                eng.stream_release(stream=s)
        fresh, destroy2 = _hip_streams(550)  # their words are the released ones
        for s in fresh:
            eng.reconstruct_devmask(d, p, S, N, good, stream=s)
        for s in fresh:
            eng.sync(stream=s)
            eng.stream_release(stream=s)
        for s in streams[550:]:
            eng.stream_release(stream=s)
    finally:
        torch.cuda.synchronize()
        destroy()
        if destroy2:
            destroy2()
        eng.close()


def test_host_mask_uploads_survive_queued_kernels(gpu):
    """Per-stripe host masks for asynchronous device calls, many calls queued behind
    a long kernel on one stream and more on a second stream: every call must use
    its own masks (a mask slot was reusable before its kernel ran)."""
    import torch

    if not hasattr(torch.cuda, "_sleep"):
        pytest.skip("torch.cuda._sleep unavailable")
    k, m, S, N = 4, 2, 512, 2048
    t, P = k + m, shard_pitch_for(S)
    eng = BatchEngine(k, m, 0)
    try:
        data = torch.randint(0, 256, (N, k, P), dtype=torch.uint8, device="cuda")
        parity = torch.empty((N, m, P), dtype=torch.uint8, device="cuda")
        eng.encode(data, parity, S, N)
        torch.cuda.synchronize()
        full = torch.cat([data[:, :, :S], parity[:, :, :S]], dim=1)
        streams = [torch.cuda.Stream(), torch.cuda.Stream()]
        calls = []
        rng = np.random.default_rng(11)
        for j in range(24):
            s = streams[j % 2]
            if j < 2:
                with torch.cuda.stream(s):
                    torch.cuda._sleep(50_000_000)  # hold the stream while later calls upload
            lost = rng.integers(0, t, N)
            masks = (((1 << t) - 1) & ~(1 << lost)).astype(np.uint32)
            out = torch.full((N, m, P), 0xC3, dtype=torch.uint8, device="cuda")
            s.wait_stream(torch.cuda.current_stream())  # `out` is ready before the call reads it
            eng.reconstruct_out(data, parity, out, S, N, present_masks=masks, stream=s)
            del masks  # the engine must have copied them
            calls.append((lost, out))
        torch.cuda.synchronize()
        for lost, out in calls:
            want = full[torch.arange(N, device="cuda"), torch.from_numpy(lost).cuda()]
            assert torch.equal(out[:, 0, :S], want)
    finally:
        eng.close()
