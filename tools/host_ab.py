"""Host-resident batch paths: zero-copy vs staged, and workgroups/CU for the
zero-copy kernel (PCIe latency wants more requests in flight than HBM does).
Usage: python tools/host_ab.py [--n 262144]"""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
GiB = 1 << 30


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 18)
    ap.add_argument("--bpc", default="0,2,4,8,16")
    args = ap.parse_args()
    import torch

    from replication_erasurecoding_object_store_amd.batch import BatchEngine

    k, m, S, N = 4, 2, 1024, args.n
    eng = BatchEngine(k, m, 0)
    data = torch.randint(0, 256, (N, k, S), dtype=torch.uint8).pin_memory().numpy()
    parity = torch.zeros((N, m, S), dtype=torch.uint8).pin_memory().numpy()
    rng = np.random.default_rng(5)
    masks = np.where(rng.random(N) < 0.5, 0b111111 & ~(1 << rng.integers(0, 6, N)), 0b001111).astype(np.uint32)
    for zc in (True, False):
        eng.set_host_zero_copy(zc)
        for bpc in [int(b) for b in args.bpc.split(",")] if zc else [0]:
            eng.set_blocks_per_cu(bpc)
            res = {}
            for name, fn in (("encode", lambda: eng.encode_host(data, parity, S, N)),
                             ("rec1", lambda: eng.reconstruct_host(data, parity, S, N, 0b111110)),
                             ("mix", lambda: eng.reconstruct_host(data, parity, S, N, masks)),
                             ("verify", lambda: eng.verify_host(data, parity, S, N))):
                fn()
                ts = []
                for _ in range(3):
                    t0 = time.perf_counter()
                    fn()
                    ts.append(time.perf_counter() - t0)
                res[name] = round(N * k * S / min(ts) / GiB, 2)
            print(f"{eng.last_host_path():9s} bpc={bpc:2d}  GiB/s of user data: {res}", flush=True)
    eng.set_blocks_per_cu(0)
    eng.set_host_zero_copy(True)


if __name__ == "__main__":
    main()
