"""Debug: out-of-place per-stripe reconstruct for (K, M, S) with 0..B erasures per
stripe: host masks (E = the masks' maximum) and device masks with max_missing = B.
Counts mismatching (stripe, row) pairs over several trials; prints the first few."""
import sys
import numpy as np
import torch
sys.path.insert(0, ".")
from replication_erasurecoding_object_store_amd.batch import BatchEngine, shard_pitch_for

k, m, S, B = (int(x) for x in sys.argv[1:5])
trials = int(sys.argv[5]) if len(sys.argv) > 5 else 3
eng = BatchEngine(k, m, 0)
N, t = 2049, k + m
P = shard_pitch_for(S)
g = torch.Generator(device="cuda").manual_seed(k * 1000 + S)
data = torch.randint(0, 256, (N, k, P), dtype=torch.uint8, device="cuda", generator=g)
parity = torch.empty((N, m, P), dtype=torch.uint8, device="cuda")
eng.encode(data, parity, S, N)
ref = torch.cat([data, parity], dim=1).cpu().numpy()
total = 0
for trial in range(trials):
    rng = np.random.default_rng(S + k + 17 * trial + B)
    masks = np.full(N, (1 << t) - 1, np.uint32)
    for i in range(N):
        for j in rng.choice(t, size=rng.integers(0, B + 1), replace=False):
            masks[i] &= ~np.uint32(1 << int(j))
    for mode in ("host", "dev"):
        out = torch.full((N, m, P), 0xC3, dtype=torch.uint8, device="cuda")
        if mode == "host":
            eng.reconstruct_out(data, parity, out, S, N, present_masks=masks)
        else:
            eng.reconstruct_out(data, parity, out, S, N, masks_dev=torch.from_numpy(masks.view(np.int32)).cuda(),
                                max_missing=B)
            eng.sync()
        torch.cuda.synchronize()
        got = out.cpu().numpy()
        nbad = 0
        for i in range(N):
            missing = [j for j in range(t) if not (masks[i] >> j) & 1]
            for r, j in enumerate(missing):
                d = np.nonzero(got[i, r, :S] != ref[i, j, :S])[0]
                if len(d):
                    nbad += 1
                    if nbad <= 3:
                        print(f"  {mode} stripe {i} row {r} shard {j} bad bytes {len(d)} [{d.min()}..{d.max()}]")
            if (got[i, len(missing):] != 0xC3).any():
                nbad += 1
        total += nbad
        print(f"K={k} M={m} S={S} B={B} trial {trial} {mode}: {nbad} bad, kernel {eng.last_kernel()}", flush=True)
print(f"TOTAL K={k} M={m} S={S} B={B}: {total} bad")
