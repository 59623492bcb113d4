"""Markdown table of tools/run_drop_in.sh output: per object size, user GiB/s (and
calls/s) of the CPU codec on 1 core and on the CPU quota, and of the coalesced GPU
drop-in with blocking callers and with asynchronous calls, staged (caller memory)
and in place (rs_host_alloc arena).

Usage: python tools/coalesce_table.py <run_drop_in log>
"""
import json
import sys
from collections import defaultdict


def main():
    rows = defaultdict(dict)
    cols = []
    for line in open(sys.argv[1]):
        if not line.startswith("{"):
            continue
        r = json.loads(line)
        mode = r["mode"]
        where = ", in place" if r.get("registered") == 2 else (", staged" if mode != "cpu" else "")
        if mode == "cpu":
            key = f"CPU codec, {r['threads']} thread{'s' if r['threads'] > 1 else ''}"
        elif mode == "coalesced":
            key = f"GPU coalesced, {r['threads']} blocking callers{where}"
        elif mode == "async":
            key = f"GPU async, {r['threads']} loops x {r['depth']} in flight{where}"
        elif mode == "hybrid":
            key = (f"hybrid, GPU limit {r['gpu_limit']}" + (f", GPU from {r['min_obj']} B" if r.get("min_obj") else "")
                   + where)
        else:
            key = f"{mode} {r['threads']}{where}"
        if key not in cols:
            cols.append(key)
        rows[r["obj_bytes"]][key] = (r["user_GiBps"], r["calls_per_s"], r.get("cpu_share"))
    print("| object | " + " | ".join(cols) + " |")
    print("|---|" + "---|" * len(cols))
    for obj in sorted(rows):
        cells = []
        for c in cols:
            v = rows[obj].get(c)
            share = f", {v[2] * 100:.0f} % on CPU" if v and v[2] is not None and "hybrid" in c else ""
            cells.append(f"{v[0]:.1f} GiB/s ({v[1] / 1e3:.0f} K/s{share})" if v else "")
        size = f"{obj // 1024} KiB" if obj % 1024 == 0 else f"{obj / 1024:.0f} KiB"
        print(f"| {size} | " + " | ".join(cells) + " |")


if __name__ == "__main__":
    main()
