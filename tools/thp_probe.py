"""Host-memory facts behind the zero-copy hypothesis in DESIGN.md §2: THP and NUMA
balancing settings of the box, and whether a numpy array registered with
rs_host_register is backed by transparent huge pages (AnonHugePages of its mapping)
before and after registration and a zero-copy kernel."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from replication_erasurecoding_object_store_amd.batch import BatchEngine


def read(path):
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError as e:
        return f"<{e.__class__.__name__}>"


def mapping_of(addr, nbytes):
    """Sum of the /proc/self/smaps fields over the mappings overlapping
    [addr, addr + nbytes) (numpy's madvise splits an array's mapping in several)."""
    with open("/proc/self/smaps") as f:
        lines = f.read().splitlines()
    out, cur = {"vmas": 0, "Rss": 0, "AnonHugePages": 0, "Locked": 0, "THPeligible": 0}, False
    for ln in lines:
        head = ln.split()
        if head and "-" in head[0] and all(c in "0123456789abcdef-" for c in head[0]):
            lo, hi = (int(x, 16) for x in head[0].split("-"))
            cur = lo < addr + nbytes and addr < hi
            out["vmas"] += int(cur)
        elif cur and ":" in ln:
            k, v = ln.split(":", 1)
            if k in out:
                out[k] += int(v.split()[0])
    return out  # kB, THPeligible = number of eligible mappings


def main():
    facts = {k: read(p) for k, p in {
        "thp_enabled": "/sys/kernel/mm/transparent_hugepage/enabled",
        "thp_defrag": "/sys/kernel/mm/transparent_hugepage/defrag",
        "khugepaged_defrag": "/sys/kernel/mm/transparent_hugepage/khugepaged/defrag",
        "khugepaged_scan_sleep_ms": "/sys/kernel/mm/transparent_hugepage/khugepaged/scan_sleep_millisecs",
        "numa_balancing": "/proc/sys/kernel/numa_balancing",
        "compact_unevictable_allowed": "/proc/sys/vm/compact_unevictable_allowed",
        "kernel": "/proc/sys/kernel/osrelease",
    }.items()}
    print(json.dumps(facts), flush=True)
    k, m, S, N = 4, 2, 1024, 3000
    data = np.random.default_rng(1).integers(0, 256, (N, k, S), dtype=np.uint8)
    parity = np.zeros((N, m, S), np.uint8)
    print(json.dumps({"stage": "allocated", "data": mapping_of(data.ctypes.data, data.nbytes),
                      "parity": mapping_of(parity.ctypes.data, parity.nbytes)}), flush=True)
    eng = BatchEngine(k, m, 0)
    eng.host_register(data)
    eng.host_register(parity)
    print(json.dumps({"stage": "registered", "data": mapping_of(data.ctypes.data, data.nbytes),
                      "parity": mapping_of(parity.ctypes.data, parity.nbytes)}), flush=True)
    eng.encode_host(data, parity, S, N)
    print(json.dumps({"stage": "after zero-copy encode", "path": eng.last_host_path(),
                      "data": mapping_of(data.ctypes.data, data.nbytes),
                      "parity": mapping_of(parity.ctypes.data, parity.nbytes)}), flush=True)
    eng.host_unregister(data)
    eng.host_unregister(parity)
    eng.close()


if __name__ == "__main__":
    main()
