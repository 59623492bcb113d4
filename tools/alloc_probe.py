"""Does the way batch memory is allocated move the RS kernels' HBM rate?  (tools/, not product)

The same leg reads 69-77 % of 8 TB/s from process to process and box to box (DESIGN.md
§9, §10), while buffer placement inside one allocation does not matter
(tools/placement_probe.py).  This probe times a few kmsweep legs, in one process and
interleaved rounds, over rotating batch sets allocated five ways:
  torch    torch's caching allocator (what bench.py and the tests use)
  malloc   one hipMalloc per buffer
  contig   hipExtMallocWithFlags(hipDeviceMallocContiguous) per buffer
  frag     hipMalloc per buffer after 4 GiB of 2 MiB holes were punched into VRAM
           (every other one of 2 MiB allocations freed), so the batches land in holes
  arena    one hipExtMallocWithFlags(contiguous) arena per batch set, carved
Prints GB/s (algorithmic bytes / event-timed kernel time), one line per (leg, mode).

Usage: python tools/alloc_probe.py [--rounds 3] [--min-ms 100] [--legs a,b]
"""
import argparse
import ctypes
import itertools
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

LEGS = {
    # name: (k, m, S, N, mode)
    "rs42_4K_rec2p_out": (4, 2, 1024, 65536, "rec2p_out"),
    "rs42_4K_enc": (4, 2, 1024, 65536, "enc"),
    "rs104_64K_rec1pb_out": (10, 4, 6554, 16384, "rec1pb_out"),
    "rs104_64K_enc": (10, 4, 6554, 16384, "enc"),
    "rs84_64K_enc": (8, 4, 8192, 16384, "enc"),
    "rs84_64K_rec1pb_out": (8, 4, 8192, 16384, "rec1pb_out"),
}
MODES = ("torch", "malloc", "contig", "frag", "arena")
HIP_DEVICE_MALLOC_CONTIGUOUS = 0x4
HIP_MEMCPY_D2D = 3


class DevBuf:
    """A raw device allocation with the attributes BatchEngine reads from a tensor."""

    def __init__(self, ptr, shape):
        self.ptr, self.shape = ptr, shape

    def data_ptr(self):
        return self.ptr

    def dim(self):
        return len(self.shape)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--min-ms", type=float, default=100.0)
    ap.add_argument("--legs", default="all")
    ap.add_argument("--modes", default=",".join(MODES))
    args = ap.parse_args()
    import torch

    from replication_erasurecoding_object_store_amd.batch import BatchEngine, shard_pitch_for

    torch.cuda.init()
    hip = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
    hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
    hip.hipExtMallocWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
    hip.hipFree.argtypes = [ctypes.c_void_p]
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    hip.hipDeviceSynchronize.argtypes = []

    def hmalloc(nbytes, flags=None):
        p = ctypes.c_void_p()
        rc = hip.hipMalloc(ctypes.byref(p), nbytes) if flags is None else \
            hip.hipExtMallocWithFlags(ctypes.byref(p), nbytes, flags)
        if rc != 0:
            raise MemoryError(f"hip alloc of {nbytes} B flags {flags}: error {rc}")
        return p.value

    raw = []  # every hip allocation, freed at the end

    legs = LEGS if args.legs == "all" else {n: LEGS[n] for n in args.legs.split(",")}
    modes = args.modes.split(",")
    GiB = 1 << 30
    holes = []
    if "frag" in modes:
        # punch 2 MiB holes: allocate 2 MiB pieces, free every other one
        pieces = [hmalloc(2 << 20) for _ in range(4096)]
        for i, p in enumerate(pieces):
            if i % 2:
                hip.hipFree(ctypes.c_void_p(p))
            else:
                holes.append(p)
    results = {}
    for name, (k, m, S, N, mode) in legs.items():
        eng = BatchEngine(k, m, 0)
        t = k + m
        P = shard_pitch_for(S)
        nb = max(2, int(np.ceil(2.2 * GiB / (N * t * P))))
        g = torch.Generator(device="cuda").manual_seed(1)
        src = torch.randint(0, 256, (N, k, P), dtype=torch.uint8, device="cuda", generator=g)
        rng = np.random.default_rng(3)
        pairs = np.array(list(itertools.combinations(range(t), 2)))
        ch = pairs[rng.integers(0, len(pairs), N)]
        m2 = torch.from_numpy((((1 << t) - 1) & ~((1 << ch[:, 0]) | (1 << ch[:, 1]))).astype(np.uint32)
                              .view(np.int32)).cuda()
        one = ((1 << t) - 1) & ~(1 << rng.integers(0, t, N))
        m1 = torch.from_numpy(one.astype(np.uint32).view(np.int32)).cuda()
        e = {"enc": m, "rec1pb_out": 1}.get(mode, 2)
        alg = N * S * (k + e)
        shapes = [(N, k, P), (N, m, P), (N, m, P)]
        sets = {}
        for md in modes:
            bs = []
            for _ in range(nb):
                sizes = [int(np.prod(s)) for s in shapes]
                if md == "torch":
                    ts = [torch.empty(s, dtype=torch.uint8, device="cuda") for s in shapes]
                    bufs = ts
                elif md == "arena":
                    base = hmalloc(sum(sizes), HIP_DEVICE_MALLOC_CONTIGUOUS)
                    raw.append(base)
                    offs = np.cumsum([0] + sizes[:-1])
                    bufs = [DevBuf(base + int(o), s) for o, s in zip(offs, shapes)]
                else:
                    ptrs = [hmalloc(sz, HIP_DEVICE_MALLOC_CONTIGUOUS if md == "contig" else None) for sz in sizes]
                    raw.extend(ptrs)
                    bufs = [DevBuf(p, s) for p, s in zip(ptrs, shapes)]
                d = bufs[0]
                if hip.hipMemcpy(ctypes.c_void_p(d.data_ptr()), ctypes.c_void_p(src.data_ptr()), sizes[0],
                                 HIP_MEMCPY_D2D) != 0:
                    raise RuntimeError("hipMemcpy")
                eng.encode(d, bufs[1], S, N)
                bs.append(bufs)
            sets[md] = bs
        torch.cuda.synchronize()

        def run(md, i):
            d, p, o = sets[md][i % nb]
            if mode == "enc":
                eng.encode(d, p, S, N)
            elif mode == "rec1pb_out":
                eng.reconstruct_out(d, p, o, S, N, masks_dev=m1, max_missing=1)
            else:
                eng.reconstruct_out(d, p, o, S, N, masks_dev=m2)

        for rnd in range(args.rounds):
            for md in modes:
                for i in range(2):
                    run(md, i)
                iters = 10
                for rep in range(2):
                    e0 = torch.cuda.Event(enable_timing=True)
                    e1 = torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for i in range(iters):
                        run(md, i)
                    e1.record()
                    torch.cuda.synchronize()
                    ms = e0.elapsed_time(e1) / iters
                    iters = max(10, int(np.ceil(args.min_ms / max(ms, 1e-3))))
                results.setdefault((name, md), []).append(alg / (ms * 1e-3) / 1e9)
        # outputs agree across allocation modes (same inputs, same masks)
        ref = None
        for md in modes:
            run(md, 0)
            torch.cuda.synchronize()
            d, p, o = sets[md][0]
            buf = o if mode != "enc" else p
            host = np.empty(int(np.prod(buf.shape)), np.uint8)
            hip.hipMemcpy(ctypes.c_void_p(host.ctypes.data), ctypes.c_void_p(buf.data_ptr()), host.size, 2)
            host = host.reshape(N, m, P)[:, :e, :S]  # padding is never written
            h = hash(host.tobytes())
            ref = h if ref is None else ref
            if h != ref:
                print(f"{name}: outputs differ in mode {md}", flush=True)
        for md in modes:
            r = results[(name, md)]
            print(f"{name:22s} {md:7s} median {np.median(r):7.1f} GB/s ({np.median(r) / 80:5.1f} %)  "
                  f"rounds {' '.join(f'{x / 80:5.1f}' for x in r)}  {eng.last_kernel()}", flush=True)
        del sets
        for p in raw:
            hip.hipFree(ctypes.c_void_p(p))
        raw.clear()
        torch.cuda.empty_cache()
    for p in holes:
        hip.hipFree(ctypes.c_void_p(p))


if __name__ == "__main__":
    main()
