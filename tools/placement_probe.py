"""Does buffer placement move the out-of-place reconstruct rate?  The same
RS(10+4) 64 KiB bounded 1-erasure launch (apply_flat_ps_kernel<10,4,1>) read
72.7 % and 77.4 % of 8 TB/s in two processes on one box
(profiles/r03z_ab_dense_out_rejected.log).  Here one process carves the data,
parity and out regions out of one allocation at chosen byte offsets from each
other and times the launch over >= 100 ms per placement, twice in alternating
order, so placement effects separate from process-to-process state.

Usage: python tools/placement_probe.py [k m S N]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from replication_erasurecoding_object_store_amd.batch import BatchEngine, shard_pitch_for

    k, m, S, N = (int(x) for x in sys.argv[1:5]) if len(sys.argv) > 4 else (10, 4, 6554, 16384)
    t = k + m
    P = shard_pitch_for(S)
    eng = BatchEngine(k, m, 0)
    dbytes, pbytes, obytes = N * k * P, N * m * P, N * P
    slack = 8 << 20
    nb = 3  # rotate 3 placements' worth of batches: > the 256 MiB Infinity Cache
    rng = np.random.default_rng(3)
    one = ((1 << t) - 1) & ~(1 << rng.integers(0, t, N))
    masks1 = torch.from_numpy(one.astype(np.uint32).view(np.int32)).cuda()
    # (data->parity gap, parity->out gap) in bytes past the previous region's end
    gaps = [(0, 0), (4096, 4096), (65536, 65536), (1 << 20, 1 << 20), (2 << 20, 3 << 20),
            (256, 768), (4 << 20, 4096), (12288, 2 << 20)]
    bufs = []
    for _ in range(nb):
        whole = torch.empty(dbytes + pbytes + obytes + 2 * slack + 4096, dtype=torch.uint8, device="cuda")
        whole[:dbytes].random_(0, 256)
        bufs.append(whole)
    alg = N * S * (k + 1)
    res = {}
    for rnd in range(2):
        order = gaps if rnd == 0 else gaps[::-1]
        for g in order:
            views = []
            for whole in bufs:
                d = whole[:dbytes].view(N, k, P)
                po = dbytes + g[0]
                p = whole[po:po + pbytes].view(N, m, P)
                oo = po + pbytes + g[1]
                o = whole[oo:oo + obytes].view(N, 1, P)
                views.append((d, p, o))
            for d, p, _ in views:
                eng.encode(d, p, S, N)

            def run(i):
                d, p, o = views[i % nb]
                eng.reconstruct_out(d, p, o, S, N, masks_dev=masks1, max_missing=1)

            for i in range(3):
                run(i)
            iters = 10
            for rep in range(2):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                e0.record()
                for i in range(iters):
                    run(i)
                e1.record()
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / iters
                iters = max(10, int(np.ceil(100.0 / ms)))
            res.setdefault(g, []).append(alg / (ms * 1e-3) / 8e12 * 100)
            print(f"round {rnd} gaps data->parity {g[0]:>8d} parity->out {g[1]:>8d}: "
                  f"{res[g][-1]:5.1f} % of 8 TB/s  {eng.last_kernel()}", flush=True)
    print("summary (both rounds):")
    for g in gaps:
        print(f"  {g[0]:>8d} {g[1]:>8d}: " + " / ".join(f"{x:5.1f}" for x in res[g]))


if __name__ == "__main__":
    main()
