"""Zero-copy host-batch reconstruct diagnostic (tests/test_gpu_parity.py::
test_split_layout_host[1024-True] failed once on r03y): repeats the test's steps and
reports where the in-place host result differs from the expected bytes, and whether a
second look after a pause still differs (late-landing writes vs wrong writes)."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from oracle import rs_oracle
from replication_erasurecoding_object_store_amd.batch import BatchEngine


def describe(got, want, N, k, P):
    bad = np.nonzero(got.reshape(-1) != want.reshape(-1))[0]
    if bad.size == 0:
        return None
    st = bad // (k * P)
    sh = (bad // P) % k
    off = bad % P
    first = [dict(stripe=int(st[i]), shard=int(sh[i]), off=int(off[i]), got=int(got.reshape(-1)[bad[i]]),
                  want=int(want.reshape(-1)[bad[i]])) for i in range(min(8, bad.size))]
    return dict(n=int(bad.size), stripes=int(np.unique(st).size), shards=sorted(set(sh.tolist())),
                zeros=int((got.reshape(-1)[bad] == 0).sum()), off_min=int(off.min()), off_max=int(off.max()),
                first=first)


def main():
    trials = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    k, m, S, N = 4, 2, 1024, 3000
    eng = BatchEngine(k, m, 0)
    out = []
    for t in range(trials):
        rng = np.random.default_rng(1024 + t)
        data = rng.integers(0, 256, (N, k, S), dtype=np.uint8)
        parity = np.zeros((N, m, S), np.uint8)
        eng.host_register(data)
        eng.host_register(parity)
        try:
            eng.encode_host(data, parity, S, N)
            path = eng.last_host_path()
            uni = np.concatenate([data, np.zeros_like(parity)], axis=1).copy()
            rs_oracle.encode_batch_scalar(k, m, uni.reshape(-1), (k + m) * S, S, S, N)
            enc = describe(parity, uni[:, k:], N, m, S)
            d0, p0 = data.copy(), parity.copy()
            data[:, 1] = 0
            parity[:, 0] = 0
            eng.reconstruct_host(data, parity, S, N, 0b101101)
            r_d, r_p = describe(data, d0, N, k, S), describe(parity, p0, N, m, S)
            late = None
            if r_d or r_p:
                time.sleep(0.05)
                late = dict(data=describe(data, d0, N, k, S), parity=describe(parity, p0, N, m, S))
            rec = dict(trial=t, path=path, kernel=eng.last_kernel(), enc=enc, rec_data=r_d, rec_parity=r_p,
                       after_50ms=late)
            print(json.dumps(rec), flush=True)
            out.append(rec)
        finally:
            eng.host_unregister(data)
            eng.host_unregister(parity)
    eng.close()
    fails = sum(1 for r in out if r["enc"] or r["rec_data"] or r["rec_parity"])
    print(json.dumps(dict(trials=trials, failing=fails)))


if __name__ == "__main__":
    main()
