"""Same-process A/B of librsgpu variants (abx/<name>.so from tools/build_ab.sh).

tools/run_ab.sh runs each variant in its own process, and an allocation's physical
pages move a leg by up to 2 points from process to process (`HISTORY.md` §A.5: the
spread is fixed per allocation).  Here every variant library is loaded into ONE
process (ctypes, RTLD_LOCAL: each keeps its own kernels and context) and they
take turns on the SAME device buffers, in an order that rotates every round, each
timed over >= min_ms of back-to-back launches.  Reported per variant: the median
fraction of 8 TB/s and the median of its per-round difference to the first
variant (paired, so a drift of the chip's state cancels).

Usage: python tools/ab_same.py --variants base,seg,pat@3 --workloads rs104_64K_rec1pb_out,... [--rounds 5]
Workload names and modes: tools/ab_bench.py (device-resident modes only).
"""
import argparse
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

from ab_bench import WORKLOADS, alg_bytes  # noqa: E402

_vp, _sz, _i = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
SIGS = {
    "rs_create": (_i, [_i, _i, _i, _i, ctypes.POINTER(_vp)]),
    "rs_destroy": (None, [_vp]),
    "rs_encode_batch": (_i, [_vp, _vp, _sz, _vp, _sz, _sz, _sz, _sz, _i, _vp]),
    "rs_reconstruct_batch_out": (_i, [_vp, _vp, _sz, _vp, _sz, _sz, _sz, _sz, _vp, _sz, _i, _vp, _sz, _vp]),
    "rs_reconstruct_batch": (_i, [_vp, _vp, _sz, _vp, _sz, _sz, _sz, _sz, _vp, _sz, _i, _vp]),
    "rs_reconstruct_batch_devmask": (_i, [_vp, _vp, _sz, _vp, _sz, _sz, _sz, _sz, _vp, _vp]),
    "rs_verify_batch": (_i, [_vp, _vp, _sz, _vp, _sz, _sz, _sz, _sz, _vp, _i, _vp]),
    "rs_reconstruct_batch_out_devmask": (_i, [_vp, _vp, _sz, _vp, _sz, _sz, _sz, _sz, _vp, _i, _vp, _sz, _vp]),
    "rs_reconstruct_batch_out_packed": (_i, [_vp, _vp, _sz, _vp, _sz, _sz, _sz, _sz, _vp, _i, _vp, _vp, _vp]),
    "rs_last_kernel": (ctypes.c_char_p, [_vp]),
    "rs_set_out_pad_writes": (_i, [_vp, _i]),
    "rs_set_occupancy_cap": (_i, [_vp, _i]),
    "rs_sync": (_i, [_vp, _vp]),
}


class Variant:
    def __init__(self, name, path, occ_cap=None, env=None):
        self.name = name
        self.occ_cap = occ_cap
        self.env = env or {}  # set around this variant's rs_create (engine-creation knobs)
        self.lib = ctypes.CDLL(path, mode=os.RTLD_LOCAL | os.RTLD_NOW)
        for fn, (res, args) in SIGS.items():
            if fn == "rs_reconstruct_batch_out_packed" and not hasattr(self.lib, fn):
                continue  # variants built before the packed entry point
            f = getattr(self.lib, fn)
            f.restype, f.argtypes = res, args
        self.packed = False  # "+packed": the mixed scans through rs_reconstruct_batch_out_packed
        self.ctx = {}

    def ctx_for(self, k, m):
        if (k, m) not in self.ctx:
            c = _vp()
            saved = {key: os.environ.get(key) for key in self.env}
            os.environ.update(self.env)
            try:
                rc = self.lib.rs_create(k, m, 0, 0, ctypes.byref(c))
            finally:
                for key, v in saved.items():
                    if v is None:
                        os.environ.pop(key, None)
                    else:
                        os.environ[key] = v
            assert rc == 0, f"{self.name}: rs_create {rc}"
            if self.occ_cap is not None:
                assert self.lib.rs_set_occupancy_cap(c, self.occ_cap) == 0
            self.ctx[(k, m)] = c
        return self.ctx[(k, m)]

    def close(self):
        for c in self.ctx.values():
            self.lib.rs_destroy(c)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", required=True, help="comma-separated abx/<name>.so (the first is the reference)")
    ap.add_argument("--workloads", required=True)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--min-ms", type=float, default=100.0)
    ap.add_argument("--out-pad", action="store_true", help="rs_set_out_pad_writes(1) on every variant")
    args = ap.parse_args()
    import torch

    GiB = 1 << 30
    names = args.variants.split(",")
    # "name@c": abx/name.so with rs_set_occupancy_cap(c) (e.g. a compute-free twin at the
    # occupancy its real kernel's registers allow); "shipped": the in-tree library;
    # "name+packed": the mixed scans (recmix_out / recmixh_out) with packed output rows,
    # so "shipped,shipped+packed" pairs the two layouts (their digests differ by layout)
    def variant(n):
        lib, _, cap = n.partition("@")
        lib, _, opt = lib.partition("+")
        path = (os.path.join(ROOT, "replication_erasurecoding_object_store_amd", "librsgpu.so") if lib == "shipped"
                else os.path.join(ROOT, "abx", lib + ".so"))
        v = Variant(n, path, int(cap) if cap else None)
        v.packed = opt == "packed"
        return v

    vs = [variant(n) for n in names]
    print(f"variants (one process): {names}; rounds {args.rounds}; >= {args.min_ms} ms per point", flush=True)
    for wl in args.workloads.split(","):
        # "<workload>@dense": bounded calls write `bound` rows per stripe back to back;
        # "@densepad": the same with the out stripe pitch 256 B longer; default: m-row slots;
        # "@spad" / "@densespad": the input stripe pitches 256 B longer (below)
        wl, _, layout = wl.partition("@")
        k, m, S, N, mode = WORKLOADS[wl]
        t = k + m
        P = (S + 255) // 256 * 256
        nb = max(2, int(np.ceil(2.2 * GiB / (N * t * P))))
        g = torch.Generator(device="cuda").manual_seed(1)
        # "@spad": 256 B more between stripes in the data and parity regions (stripe
        # pitches k*P + 256 / m*P + 256), other layouts the packed k*P / m*P
        spad = 256 if layout.endswith("spad") else 0
        DSP, PSP = k * P + spad, m * P + spad
        bufs = [(torch.randint(0, 256, (N, DSP), dtype=torch.uint8, device="cuda", generator=g),
                 torch.empty((N, PSP), dtype=torch.uint8, device="cuda")) for _ in range(nb)]
        out_rows = ({"rec1pb_out": 1, "rec2pb_out": 2, "rec2sb_out": 2}.get(mode, m)
                    if layout in ("dense", "densepad", "densespad") else m)
        osp = out_rows * P + (256 if layout == "densepad" else 0)
        outs = [torch.empty((N, osp), dtype=torch.uint8, device="cuda") for _ in range(nb)]
        rng = np.random.default_rng(3)
        full = (1 << t) - 1
        if mode in ("rec1pb_out", "rec1p_out"):
            mk = full & ~(1 << rng.integers(0, t, N))
            bound = 1 if mode == "rec1pb_out" else 0
        elif mode in ("rec2u", "rec2u_out"):  # one host pattern for the batch: data 0 and 1 lost
            mk = np.array([full & ~0b11])
            bound = 0
        elif mode == "ver":
            mk, bound = None, 0
        elif mode == "rec2sb_out":  # one pattern on every stripe, per-stripe device masks, bound 2
            mk = np.full(N, full & ~0b11)
            bound = 2
        elif mode in ("rec2pb_out", "rec2p_out", "rec2p"):
            import itertools

            pairs = np.array(list(itertools.combinations(range(t), 2)))
            ch = pairs[rng.integers(0, len(pairs), N)]
            mk = full & ~((1 << ch[:, 0]) | (1 << ch[:, 1]))
            bound = 2 if mode == "rec2pb_out" else 0
        elif mode == "rec4p_out":
            mk = np.array([full & ~sum(1 << int(j) for j in rng.choice(t, size=min(4, m), replace=False))
                           for _ in range(N)])
            bound = 0
        elif mode in ("recmix_out", "recmix1_out", "recmixh_out", "recmixp_out", "recmixph_out"):
            lo = 1 if mode == "recmix1_out" else 0
            mk = np.full(N, full)
            for i, ne in enumerate(rng.integers(lo, m + 1, N)):
                for j in rng.choice(t, size=int(ne), replace=False):
                    mk[i] &= ~(1 << int(j))
            bound = 0
        elif mode == "enc":
            mk, bound = None, 0
        else:
            raise SystemExit(f"{wl}: mode {mode} not supported here")
        bad = torch.zeros(N, dtype=torch.int32, device="cuda")
        roffs = torch.zeros(N + 1, dtype=torch.int32, device="cuda")  # packed modes' row offsets
        alg = alg_bytes(wl)
        if mk is not None:
            mk = mk.astype(np.uint32)
            if mode in ("recmix_out", "recmix1_out", "recmixh_out", "recmixp_out", "recmixph_out"):
                nmiss = np.array([bin(int(x) ^ full).count("1") for x in mk])
                alg = int(S * (k * np.count_nonzero(nmiss) + nmiss.sum()))
            md = torch.from_numpy(mk.view(np.int32)).cuda()
            mh = np.ascontiguousarray(mk)  # host masks (recmixh_out): the engine uploads them
        for v in vs:
            v.lib.rs_set_out_pad_writes(v.ctx_for(k, m), 1 if args.out_pad else 0)

        def run(v, i):
            c = v.ctx_for(k, m)
            d, p = bufs[i % nb]
            if mode == "enc":
                rc = v.lib.rs_encode_batch(c, d.data_ptr(), DSP, p.data_ptr(), PSP, P, S, N, 0, None)
            elif mode == "ver":
                rc = v.lib.rs_verify_batch(c, d.data_ptr(), DSP, p.data_ptr(), PSP, P, S, N, bad.data_ptr(), 0,
                                           None)
            elif mode == "rec2u":  # in place: rewrites the lost shards with their own bytes
                rc = v.lib.rs_reconstruct_batch(c, d.data_ptr(), DSP, p.data_ptr(), PSP, P, S, N, mh.ctypes.data,
                                                1, 0, None)
            elif mode == "rec2u_out":
                rc = v.lib.rs_reconstruct_batch_out(c, d.data_ptr(), DSP, p.data_ptr(), PSP, P, S, N,
                                                    mh.ctypes.data, 1, 0, outs[i % nb].data_ptr(), m * P, None)
            elif mode == "rec2p":  # in place, per-stripe device masks
                rc = v.lib.rs_reconstruct_batch_devmask(c, d.data_ptr(), DSP, p.data_ptr(), PSP, P, S, N,
                                                        md.data_ptr(), None)
            elif bound:
                rc = v.lib.rs_reconstruct_batch_out_devmask(c, d.data_ptr(), DSP, p.data_ptr(), PSP, P, S, N,
                                                            md.data_ptr(), bound, outs[i % nb].data_ptr(), osp,
                                                            None)
            elif mode in ("recmixp_out", "recmixph_out") or (v.packed and mode in ("recmix_out", "recmixh_out")):
                dev = mode in ("recmixp_out", "recmix_out")  # packed rows (rs_reconstruct_batch_out_packed)
                rc = v.lib.rs_reconstruct_batch_out_packed(c, d.data_ptr(), DSP, p.data_ptr(), PSP, P, S, N,
                                                           md.data_ptr() if dev else mh.ctypes.data, 1 if dev else 0,
                                                           outs[i % nb].data_ptr(), roffs.data_ptr(), None)
            elif mode == "recmixh_out":
                rc = v.lib.rs_reconstruct_batch_out(c, d.data_ptr(), DSP, p.data_ptr(), PSP, P, S, N,
                                                    mh.ctypes.data, N, 0, outs[i % nb].data_ptr(), m * P, None)
            else:
                rc = v.lib.rs_reconstruct_batch_out(c, d.data_ptr(), DSP, p.data_ptr(), PSP, P, S, N,
                                                    md.data_ptr(), N, 1, outs[i % nb].data_ptr(), m * P, None)
            assert rc == 0, (v.name, rc)

        for v in vs:  # every batch a codeword; warm each variant's kernels
            for d, p in bufs:
                v.lib.rs_encode_batch(v.ctx_for(k, m), d.data_ptr(), DSP, p.data_ptr(), PSP, P, S, N, 0, None)
            run(v, 0)
        torch.cuda.synchronize()
        res = {v.name: [] for v in vs}
        digests = {}
        for r in range(args.rounds):
            order = vs[r % len(vs):] + vs[:r % len(vs)]
            for v in order:
                run(v, 0)
                run(v, 1)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                iters = 10
                for rep in range(2):  # the first pass sizes the second
                    e0.record()
                    for i in range(iters):
                        run(v, i)
                    e1.record()
                    torch.cuda.synchronize()
                    ms = e0.elapsed_time(e1) / iters
                    iters = max(10, int(np.ceil(args.min_ms / max(ms, 1e-3))))
                res[v.name].append(alg / (ms * 1e-3) / 1e9 / 8000)
        for v in vs:
            run(v, 0)
            torch.cuda.synchronize()
            o = (bufs[0][1] if mode == "enc" else bad if mode == "ver" else
                 bufs[0][0] if mode in ("rec2u", "rec2p") else outs[0]).cpu().numpy()
            digests[v.name] = hash(o.tobytes())
            kname = v.lib.rs_last_kernel(v.ctx_for(k, m)).decode()
            base = np.array(res[vs[0].name])
            mine = np.array(res[v.name])
            print(f"{wl + ('@' + layout if layout else ''):24s} {v.name:10s} median {np.median(mine) * 100:5.1f}%  min {mine.min() * 100:5.1f}  "
                  f"max {mine.max() * 100:5.1f}  paired diff vs {vs[0].name}: {np.median(mine - base) * 100:+5.2f} "
                  f"points  {kname}", flush=True)
        agree = len(set(digests.values())) == 1
        print(f"{wl:24s} outputs agree across variants: {agree}", flush=True)
        del bufs, outs
        torch.cuda.empty_cache()
    for v in vs:
        v.close()


if __name__ == "__main__":
    main()
