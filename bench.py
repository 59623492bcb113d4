"""Benchmark: device-resident RS(4+2) encode + 2-erasure reconstruct on MI355X.

Metric (BASELINE.json): "GiB/s device-resident RS(4+2) encode + 2-erasure
reconstruct, batched stripes".  One *step* = one pass of the hot path over one
batch: encode the batch (configs[1]: 65 536 objects x 4 KiB stripe, RS(4+2),
S = 1 024) and then reconstruct two erased shards per stripe with a seeded random
pattern per stripe (configs[2], 2-missing case).  User data per step =
2 x N x K x S bytes; `value` = user-data GiB/s over all ranks.

Inputs are resident in HBM before the timed region; batches rotate over >= 2 GiB
so the 256 MiB Infinity Cache cannot serve them.  Multi-GPU: one process per GPU,
each with its own stripe batches (objects are independent: weak scaling, no
data-path collective); the only collectives are the timing barrier / max-reduce.

Roofline: the dominant kernel's algorithmic bytes per launch (encode N.S.(K+M),
reconstruct N.S.(K+e)) / its average launch time measured with HIP
events on the launch stream, against 8.0 TB/s (MI355X_MICROARCH.md).
cpu_baseline: oracle/rs_cpu_baseline.c (AVX-512 GFNI / AVX2 split-nibble C
restatement of klauspost's CPU kernels -- a port, not the Go reference, which is
absent) on the host cores of this box, same workload, bounded sample.
"""
from __future__ import annotations

import argparse
import glob
import itertools
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

GiB = float(1 << 30)
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=30)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--stripes", type=int, default=65536)
    p.add_argument("--stripe-kib", type=int, default=4)
    p.add_argument("--k", type=int, default=4)
    p.add_argument("--m", type=int, default=2)
    p.add_argument("--rotate-gib", type=float, default=2.0)
    p.add_argument("--no-extras", action="store_true")
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=10.0)
    p.add_argument("--json-out", default="")
    return p.parse_args()


def two_erasure_masks(rng, n, t):
    pairs = np.array(list(itertools.combinations(range(t), 2)))
    ch = pairs[rng.integers(0, len(pairs), n)]
    full = (1 << t) - 1
    return (full & ~((1 << ch[:, 0]) | (1 << ch[:, 1]))).astype(np.uint32)


def make_batches(torch, n_batches, N, k, m, P, seed):
    """Split layout (the fast device layout): data [N, K, P] + parity [N, M, P]."""
    g = torch.Generator(device="cuda").manual_seed(seed)
    out = []
    for _ in range(n_batches):
        d = torch.randint(0, 256, (N, k, P), dtype=torch.uint8, device="cuda", generator=g)
        p = torch.empty((N, m, P), dtype=torch.uint8, device="cuda")
        out.append((d, p))
    return out


def measure_rs(torch, eng, k, m, S, N, steps, warmup, rotate_bytes, seed, roofline_reps=20, barrier=lambda: None):
    """Step = encode the batch + reconstruct 2 erased shards per stripe (seeded
    per-stripe pattern, device-resident masks).  Returns the step time, and each
    kernel's average launch duration from `roofline_reps` back-to-back launches
    bracketed by one HIP event pair on the launch stream (torch's current stream,
    which the engine launches on)."""
    from replication_erasurecoding_object_store_amd.batch import shard_pitch_for

    t = k + m
    P = shard_pitch_for(S)
    batch_bytes = N * t * P
    nb = max(2, int(np.ceil(rotate_bytes / batch_bytes)))
    bufs = make_batches(torch, nb, N, k, m, P, seed)
    # reconstruct writes the 2 missing shards of every stripe to a separate output
    # buffer: the reference's semantics (Reconstruct gives missing entries NEW
    # slices; the healer writes back only those) and include/rsgpu.h's
    # rs_reconstruct_batch_out
    # (device masks: the engine cannot bound #missing on the host, so it requires
    # room for m outputs per stripe; only the first 2 are written here)
    outs = [torch.empty((N, m, P), dtype=torch.uint8, device="cuda") for _ in range(nb)]
    rng = np.random.default_rng(0x5EED0003)
    masks = [torch.from_numpy(two_erasure_masks(rng, N, t).view(np.int32)).cuda() for _ in range(nb)]
    for d, p in bufs:  # make every batch a codeword before timing
        eng.encode(d, p, S, N)

    def enc(i):
        d, p = bufs[i % nb]
        eng.encode(d, p, S, N)

    def rec(i):
        d, p = bufs[i % nb]
        eng.reconstruct_out(d, p, outs[i % nb], S, N, masks_dev=masks[i % nb])

    for i in range(warmup):
        enc(i)
        rec(i)
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        enc(i)
        rec(i)
    torch.cuda.synchronize()
    barrier()
    dt = time.perf_counter() - t0
    eng.sync()
    kernel_ms = {}
    kernel_names = {}
    for name, fn in (("encode", enc), ("reconstruct", rec)):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(roofline_reps):
            fn(i)
        e1.record()
        torch.cuda.synchronize()
        kernel_ms[name] = e0.elapsed_time(e1) / roofline_reps
        kernel_names[name] = eng.last_kernel()
    eng.sync()
    # full-size property check on every stripe of two batches: the reconstructed
    # shards equal the erased originals (encode -> erase 2 -> reconstruct round trip)
    ok = True
    for i in range(min(nb, 2)):
        d, p = bufs[i]
        full = torch.cat([d[:, :, :S], p[:, :, :S]], dim=1)
        mk = masks[i].cpu().numpy().view(np.uint32)
        lost = torch.from_numpy((((mk[:, None] >> np.arange(t)[None, :]) & 1) == 0)).cuda()
        want = full[lost].view(N, 2, S)  # missing shards in index order
        ok &= bool(torch.equal(outs[i][:, :2, :S], want))
    del bufs, masks, outs
    torch.cuda.empty_cache()
    return {"dt": dt, "steps": steps, "kernel_ms": kernel_ms, "batch_bytes": batch_bytes, "n_batches": nb, "ok": ok,
            "kernels": kernel_names}


def cpu_baseline(k, m, S, N_sample, seconds):
    from oracle import rs_oracle

    t = k + m
    P = S  # host layout: contiguous shards
    buf = np.random.default_rng(1).integers(0, 256, N_sample * t * P, dtype=np.uint8)
    try:
        threads = len(os.sched_getaffinity(0))
    except AttributeError:
        threads = os.cpu_count() or 1
    threads = max(1, min(threads, int(os.environ.get("OMP_NUM_THREADS", threads))))
    mat = rs_oracle.build_matrix(k, m)
    surv, miss, rows = rs_oracle.decode_rows(k, m, [0, 0] + [1] * (t - 2))
    level = 0
    done = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        level = rs_oracle.baseline_apply_batch(k, mat[k:], list(range(k)), list(range(k, t)), buf, t * P, P, S,
                                               N_sample, threads)
        rs_oracle.baseline_apply_batch(k, rows, surv, miss, buf, t * P, P, S, N_sample, threads)
        done += 1
    dt = time.perf_counter() - t0
    gibs = done * 2 * N_sample * k * S / dt / GiB
    simd = {0: "scalar", 2: "avx2-vpshufb", 3: "avx512-gfni"}.get(level, str(level))
    return {
        "value": round(gibs, 3),
        "unit": "GiB/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{done} passes x (encode + 2-erasure reconstruct) of {N_sample} x {k * S // 1024} KiB "
                  f"RS({k}+{m}) stripes, {simd}, one stripe per task, {threads} threads "
                  f"(C restatement of klauspost's CPU kernels; Go reference absent)",
    }


def copy_peak(torch, eng, nbytes=1 << 30, iters=20):
    a = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    b = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    a.fill_(1)
    for _ in range(3):
        eng.device_copy(b, a)
    torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        eng.device_copy(b, a)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / iters
    del a, b
    torch.cuda.empty_cache()
    return 2 * nbytes / (ms * 1e-3) / 1e9


def link_peak(torch, nbytes=256 << 20):
    """Pinned host <-> HBM copy rates (the PCIe ceiling the host path works under)."""
    h = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    d = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    out = {}
    for name, fn in (("h2d", lambda: d.copy_(h, non_blocking=True)), ("d2h", lambda: h.copy_(d, non_blocking=True))):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(4):
            fn()
        torch.cuda.synchronize()
        out[name + "_GBps"] = round(4 * nbytes / (time.perf_counter() - t0) / 1e9, 1)
    return out


def host_e2e(torch, eng, k, m, S, N):
    """Pinned host -> H2D -> kernel -> D2H (split layout, shards back to back as
    Split produces them): encode, then 1-erasure reconstruct.  Rates are user data
    bytes (N*K*S) per second; the link moves K+M (encode: K in, M out) shards."""
    data = np.random.default_rng(2).integers(0, 256, (N, k, S), dtype=np.uint8)
    parity = np.zeros((N, m, S), np.uint8)
    eng.host_register(data)
    eng.host_register(parity)
    out = {"bytes_user": N * k * S}
    try:
        for zc in (True, False):
            eng.set_host_zero_copy(zc)
            eng.encode_host(data, parity, S, N)  # pipeline state + first touch of the pinned pages
            path = eng.last_host_path()
            t0 = time.perf_counter()
            eng.encode_host(data, parity, S, N)
            t_enc = time.perf_counter() - t0
            mask = ((1 << (k + m)) - 1) & ~1
            t0 = time.perf_counter()
            eng.reconstruct_host(data, parity, S, N, mask)
            t_rec = time.perf_counter() - t0
            out[path] = {"encode_GiBps": round(N * k * S / t_enc / GiB, 2),
                         "reconstruct1_GiBps": round(N * k * S / t_rec / GiB, 2)}
    finally:
        eng.set_host_zero_copy(True)
        eng.host_unregister(data)
        eng.host_unregister(parity)
    out.update(link_peak(torch))
    return out


def healer_mix(torch, eng, k, m, S, N, seed=0x5EED0005):
    """N objects, each either encoded (parity missing) or
    repaired from one erasure (index uniform in [0, k+m)), 50/50 by a seeded draw,
    in ONE batched call with a present-mask per stripe.  e2e: shards in pinned host
    memory, H2D + kernel + D2H inside the timed region (rs_reconstruct_batch,
    RS_MEM_HOST).  device: the same masks on HBM-resident shards."""
    t = k + m
    full = (1 << t) - 1
    rng = np.random.default_rng(seed)
    is_rec = rng.random(N) < 0.5
    lost = rng.integers(0, t, N)
    masks = np.where(is_rec, full & ~(1 << lost), (1 << k) - 1).astype(np.uint32)
    data = torch.empty((N, k, S), dtype=torch.uint8, pin_memory=True)
    parity = torch.empty((N, m, S), dtype=torch.uint8, pin_memory=True)
    g = torch.Generator(device="cuda").manual_seed(seed)
    step = 1 << 16
    for s0 in range(0, N, step):  # random data + its true parity, made on the GPU
        n = min(step, N - s0)
        dd = torch.randint(0, 256, (n, k, S), dtype=torch.uint8, device="cuda", generator=g)
        pp = torch.empty((n, m, S), dtype=torch.uint8, device="cuda")
        eng.encode(dd, pp, S, n)
        data[s0:s0 + n].copy_(dd)
        parity[s0:s0 + n].copy_(pp)
    torch.cuda.synchronize()
    dn, pn = data.numpy(), parity.numpy()
    sample = rng.choice(N, size=min(N, 4096), replace=False)
    ref_d, ref_p = dn[sample].copy(), pn[sample].copy()
    lost_d = (~masks[:, None] >> np.arange(k)[None, :]) & 1
    lost_p = (~masks[:, None] >> np.arange(k, t)[None, :]) & 1

    def erase():
        dn[lost_d.astype(bool)] = 0
        pn[lost_p.astype(bool)] = 0

    e2e, ok = {}, True
    for zc in (True, False):  # torch's pinned pages are GPU-mapped: zero-copy qualifies
        eng.set_host_zero_copy(zc)
        erase()
        eng.reconstruct_host(dn, pn, S, N, masks)  # warm: pipeline slabs, LUT
        times = []
        for _ in range(2):
            erase()
            t0 = time.perf_counter()
            eng.reconstruct_host(dn, pn, S, N, masks)
            times.append(time.perf_counter() - t0)
        ok = ok and bool(np.array_equal(dn[sample], ref_d) and np.array_equal(pn[sample], ref_p))
        e2e[eng.last_host_path()] = min(times)
    eng.set_host_zero_copy(True)
    # device-resident, same masks, in place
    dd = data.cuda()
    pd = parity.cuda()
    md = torch.from_numpy(masks.view(np.int32)).cuda()
    eng.reconstruct_devmask(dd, pd, S, N, md)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        eng.reconstruct_devmask(dd, pd, S, N, md)
    e1.record()
    torch.cuda.synchronize()
    t_dev = e0.elapsed_time(e1) / 5 * 1e-3
    eng.sync()
    del dd, pd, md, data, parity
    torch.cuda.empty_cache()
    user = N * k * S
    return {"objects": N, "shard_len": S, "encode_frac": round(float((~is_rec).mean()), 4),
            "e2e_GiBps": {p: round(user / t / GiB, 2) for p, t in e2e.items()},
            "e2e_objects_per_s": {p: round(N / t) for p, t in e2e.items()},
            "device_GiBps": round(user / t_dev / GiB, 1), "ok_sample": ok,
            "note": "zero-copy: kernel reads survivors / writes missing shards over PCIe in place; "
                    "staged: every k+m slot DMA'd each way"}


def scrub_rate(torch, eng, k, m, S, N, rotate_bytes, seed=0x5EED0006, reps=10):
    """Device-resident verify / bit-rot scrub (rs_verify_batch): re-encode and
    compare every stripe, K+M shards read per stripe, nothing written but the
    per-stripe mismatch words.  Checks clean batches verify clean and one flipped
    byte is found."""
    from replication_erasurecoding_object_store_amd.batch import shard_pitch_for

    P = shard_pitch_for(S)
    nb = max(2, int(np.ceil(rotate_bytes / (N * (k + m) * P))))
    bufs = make_batches(torch, nb, N, k, m, P, seed)
    for d, p in bufs:
        eng.encode(d, p, S, N)
    bad = torch.empty(N, dtype=torch.int32, device="cuda")
    for i in range(2):
        eng.verify(*bufs[i % nb], bad, S, N)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(reps):
        eng.verify(*bufs[i % nb], bad, S, N)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    d, p = bufs[0]
    eng.verify(d, p, bad, S, N)
    torch.cuda.synchronize()
    clean = int(bad.count_nonzero()) == 0
    p[N // 3, m - 1, S - 1] ^= 0x40
    eng.verify(d, p, bad, S, N)
    torch.cuda.synchronize()
    hit = bad.nonzero().flatten().tolist() == [N // 3] and int(bad[N // 3]) == 1 << (m - 1)
    kname = eng.last_kernel()
    del bufs
    torch.cuda.empty_cache()
    return {"kernel": kname, "shard_len": S, "stripes": N, "ms": round(ms, 5),
            "user_GiBps": round(N * k * S / (ms * 1e-3) / GiB, 1),
            "hbm_frac": round(N * S * (k + m) / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4), "ok": clean and hit}


def layout_and_patterns(torch, eng, k, m, S, N, rotate_bytes, reps=10):
    """Config 2's SoA layout variant and config 3's named erasure patterns, each as
    kernel time per launch (HIP events, rotating >= 2 GiB).  Rates: user data
    K*S*N per second and HBM fraction of the algorithmic bytes."""
    from replication_erasurecoding_object_store_amd.batch import shard_pitch_for

    t = k + m
    P = shard_pitch_for(S)
    nb = max(2, int(np.ceil(rotate_bytes / (N * t * P))))
    g = torch.Generator(device="cuda").manual_seed(0x5EED0003)
    split = [(torch.randint(0, 256, (N, k, P), dtype=torch.uint8, device="cuda", generator=g),
              torch.empty((N, m, P), dtype=torch.uint8, device="cuda"), torch.empty((N, m, P), dtype=torch.uint8,
                                                                                     device="cuda"))
             for _ in range(nb)]
    for d, p, _ in split:
        eng.encode(d, p, S, N)
    rng = np.random.default_rng(0x5EED0003)
    one = ((1 << t) - 1) & ~(1 << rng.integers(0, t, N))
    full = (1 << t) - 1
    dev_one = torch.from_numpy(one.astype(np.uint32).view(np.int32)).cuda()

    def timed(fn):
        for i in range(2):
            fn(i)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(reps):
            fn(i)
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps * 1e-3

    res = {}

    def put(name, sec, e):
        res[name] = {"user_GiBps": round(N * k * S / sec / GiB, 1),
                     "hbm_frac": round(N * S * (k + e) / sec / 1e9 / HBM_PEAK_GBS, 4)}

    put("rec1_per_stripe_out", timed(lambda i: eng.reconstruct_out(split[i % nb][0], split[i % nb][1],
                                                                      split[i % nb][2], S, N, masks_dev=dev_one)), 1)
    for name, pat in (("rec_0_1_uniform_out", (0, 1)), ("rec_0_4_uniform_out", (0, 4)),
                      ("rec_4_5_uniform_out", (4, 5))):
        mask = full & ~sum(1 << j for j in pat)
        put(name, timed(lambda i: eng.reconstruct_out(split[i % nb][0], split[i % nb][1], split[i % nb][2], S, N,
                                                      present_masks=mask)), 2)
    del split
    torch.cuda.empty_cache()
    # SoA: shard s of every stripe in one plane
    soa = [(torch.randint(0, 256, (k, N, P), dtype=torch.uint8, device="cuda", generator=g),
            torch.empty((m, N, P), dtype=torch.uint8, device="cuda")) for _ in range(nb)]
    put("soa_encode", timed(lambda i: eng.encode(soa[i % nb][0], soa[i % nb][1], S, N, shard_pitch=N * P,
                                                 data_stripe_pitch=P, parity_stripe_pitch=P)), m)
    del soa
    torch.cuda.empty_cache()
    return res


def sha256_rate(torch, eng, N=65536, length=4096, reps=5, cpu_seconds=3.0):
    """Batched SHA-256 of N device-resident objects (the reference's cold_hash,
    writeservice.go:51-54) vs hashlib (OpenSSL) on the host cores."""
    import hashlib

    g = torch.Generator(device="cuda").manual_seed(0x5EED0007)
    bufs = [torch.randint(0, 256, (N, length), dtype=torch.uint8, device="cuda", generator=g) for _ in range(2)]
    out = torch.empty((N, 32), dtype=torch.uint8, device="cuda")
    eng.sha256(bufs[0], length, N, digests=out)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(reps):
        eng.sha256(bufs[i % 2], length, N, digests=out)
    e1.record()
    torch.cuda.synchronize()
    sec = e0.elapsed_time(e1) / reps * 1e-3
    host = bufs[(reps - 1) % 2][:256].cpu().numpy()
    ok = all(out[i].cpu().numpy().tobytes() == hashlib.sha256(host[i].tobytes()).digest() for i in range(0, 256, 17))
    # host baseline: SHA-NI (the class of Go crypto/sha256's amd64 code) on all
    # host threads, over a sample of the same objects, timed to ~cpu_seconds
    sys.path.insert(0, ROOT)
    from oracle import rs_oracle

    threads = min(len(os.sched_getaffinity(0)), int(os.environ.get("OMP_NUM_THREADS", "16") or 16))
    sample = bufs[0][:8192].cpu().numpy()
    ns, t_cpu, ni = 0, 0.0, False
    while t_cpu < cpu_seconds:
        t0 = time.perf_counter()
        _, ni = rs_oracle.baseline_sha256_batch(sample, length, length, sample.shape[0], threads)
        t_cpu += time.perf_counter() - t0
        ns += sample.shape[0]
    cpu_rate = ns * length / t_cpu / GiB
    del bufs
    torch.cuda.empty_cache()
    return {"objects": N, "object_bytes": length, "ms": round(sec * 1e3, 4), "GiBps": round(N * length / sec / GiB, 1),
            "objects_per_s": round(N / sec), "ok": ok,
            "cpu_baseline_GiBps": round(cpu_rate, 2), "cpu_threads": threads,
            "cpu_kind": "port (oracle/sha256_cpu_baseline.c, " + ("SHA-NI" if ni else "scalar") + ")"}


def pmc_traffic(workload):
    """Per-launch HBM bytes from the newest committed rocprofv3 PMC summary of this
    workload (profiles/<tag>_pmc.json written by tools/prof_summary.py), if any."""
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc*.json")), reverse=True):
        try:
            with open(path) as f:
                doc = json.load(f)
        except Exception:
            continue
        if doc.get("workload") == workload:
            return doc
    return None


def main():
    args = parse()
    import torch

    from replication_erasurecoding_object_store_amd import dist as rdist
    from replication_erasurecoding_object_store_amd.batch import BatchEngine

    rank, local, world = rdist.world()
    if world > 1:
        # RCCL; control collectives only (barrier, max time).  RSGPU_BENCH_BACKEND=gloo
        # runs them on the CPU instead, so the N>1 path can be rehearsed with several
        # ranks sharing one GPU (the driver's multi-GPU runs use the default).
        backend = os.environ.get("RSGPU_BENCH_BACKEND", "nccl")
        if backend == "gloo":
            torch.cuda.set_device(local % torch.cuda.device_count())
        rdist.init(backend)
    else:
        torch.cuda.set_device(0)

    k, m = args.k, args.m
    S = args.stripe_kib * 1024 // k
    N = args.stripes
    eng = BatchEngine(k, m, torch.cuda.current_device())
    rotate = int(args.rotate_gib * GiB)

    # weak scaling: every rank owns its own N-stripe batches (independent objects)
    res = measure_rs(torch, eng, k, m, S, N, args.steps, args.warmup, rotate, seed=0x5EED0002 + rank,
                     barrier=rdist.barrier)
    dt = rdist.max_over_ranks(res["dt"])
    res["ok"] = rdist.all_true(res["ok"])
    user_bytes_per_step = 2 * N * k * S
    value = world * args.steps * user_bytes_per_step / dt / GiB
    ms_step = dt / args.steps * 1e3

    km = res["kernel_ms"]
    alg = {"encode": N * S * (k + m), "reconstruct": N * S * (k + 2)}
    dom = max(km, key=km.get) if km else "reconstruct"
    achieved = alg[dom] / (km.get(dom, float("nan")) * 1e-3) / 1e9 if km else None
    traffic = None
    pmc = pmc_traffic(f"rs{k}{m}_{args.stripe_kib}KiB_N{N}_split")
    if pmc:
        traffic = pmc.get("hbm_bytes_per_launch", {}).get(dom)

    out = {
        "metric": "GiB/s device-resident RS(4+2) encode + 2-erasure reconstruct, batched stripes",
        "value": round(value, 3),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic: uniform random bytes (torch on-device RNG), seeded per-stripe 2-erasure patterns "
                "(seed 0x5EED0003)",
        "config": {
            "workload": f"RS({k}+{m}) encode + 2-erasure reconstruct, {N} objects x {args.stripe_kib} KiB stripe "
                        f"(S={S}) per GPU, device-resident, {res['n_batches']} rotating batches "
                        f"({res['n_batches'] * res['batch_bytes'] / GiB:.2f} GiB)",
            "k": k, "m": m, "shard_len": S, "stripes_per_gpu": N,
            "parallelism": f"dp{world} (independent stripes per GPU, no collective)",
        },
        "roofline": {
            "bound": "hbm",
            "kernel": f"{res['kernels'].get(dom)} ({dom}; rocprof name rs::apply_kernel<{k}, {m}, 2, "
                      f"{'true' if dom == 'reconstruct' else 'false'}>)",
            "timing": "HIP events around 20 back-to-back launches on the launch stream",
            "achieved": round(achieved, 1) if achieved else None,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4) if achieved else None,
            "traffic": traffic,
            "kernel_ms": {kk: round(v, 5) for kk, v in km.items()},
            "alg_bytes_per_launch": alg,
        },
        "parity_check_full_size": res["ok"],
    }
    if rank == 0 and world == 1 and not args.no_cpu:
        out["cpu_baseline"] = cpu_baseline(k, m, S, 16384, args.cpu_seconds)
    if rank == 0 and world == 1 and not args.no_extras:
        extras = {"copy_kernel_peak_GBps": round(copy_peak(torch, eng), 1)}
        sweep = {}
        for kk, mm in [(4, 2), (8, 4), (10, 4)]:
            e2 = BatchEngine(kk, mm, 0)
            SS = -(-65536 // kk)
            NN = 16384
            r = measure_rs(torch, e2, kk, mm, SS, NN, 5, 2, rotate, seed=0x5EED0004, roofline_reps=10)
            kms = r["kernel_ms"]
            sweep[f"rs{kk}{mm}_64KiB"] = {
                "shard_len": SS, "stripes": NN,
                "encode_GiBps": round(NN * kk * SS / (kms["encode"] * 1e-3) / GiB, 1),
                "reconstruct2_GiBps": round(NN * kk * SS / (kms["reconstruct"] * 1e-3) / GiB, 1),
                "encode_hbm_frac": round(NN * SS * (kk + mm) / (kms["encode"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                "reconstruct2_hbm_frac": round(NN * SS * (kk + 2) / (kms["reconstruct"] * 1e-3) / 1e9 / HBM_PEAK_GBS,
                                               4),
                "ok": r["ok"],
            }
            e2.close()
        extras["kmsweep_64KiB_device"] = sweep
        extras["config3_patterns_and_soa_rs42_4KiB"] = layout_and_patterns(torch, eng, k, m, S, N, rotate)
        extras["scrub_verify_device"] = {"rs42_4KiB": scrub_rate(torch, eng, k, m, S, N, rotate)}
        e2 = BatchEngine(10, 4, 0)
        extras["scrub_verify_device"]["rs104_64KiB"] = scrub_rate(torch, e2, 10, 4, 6554, 16384, rotate)
        e2.close()
        extras["host_e2e_pinned_rs42_4KiB"] = host_e2e(torch, eng, k, m, S, 1 << 18)
        extras["healer_mix_config5"] = healer_mix(torch, eng, k, m, S, 1 << 20)
        extras["sha256_cold_hash_4KiB"] = sha256_rate(torch, eng)
        out["extras"] = extras
    if rank == 0:
        line = json.dumps(out)
        print(line, flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                f.write(line + "\n")
    eng.close()
    rdist.shutdown()


if __name__ == "__main__":
    main()
