"""Summarise a tools/profile_bench.sh run into profiles/<tag>_*.{md,json}.

Durations come from the kernel-trace pass; HBM bytes from the two separate PMC
passes, corrected as MI355X_MICROARCH.md §HBM prescribes for gfx950:
  FETCH_SIZE and WRITE_SIZE are in KiB (x 1024);
  FETCH_SIZE reports exactly half the bytes of a wide (16 B/lane) coalesced
  streaming read -> doubled;  WRITE_SIZE is exact for 16-B-per-lane stores.
Only the full-size dispatches of each kernel are summarised (the largest grid the
kernel was launched with), so bench.py's small verification launches are excluded.

Usage: python tools/prof_summary.py gpurun_out/prof_r01 r01 "<workload key>"
"""
from __future__ import annotations

import csv
import json
import os
import statistics
import sys
from collections import defaultdict


def rows(path):
    with open(path, newline="") as f:
        return list(csv.DictReader(f))


def short(name: str) -> str:
    return name.replace("void ", "").split("(")[0]


def full_size(vals):
    if not vals:
        return vals
    med = statistics.median(vals)
    return [v for v in vals if v >= 0.5 * med]


def main():
    src, tag = sys.argv[1], sys.argv[2]
    workload = sys.argv[3] if len(sys.argv) > 3 else ""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    trace = rows(os.path.join(src, "trace", "run_kernel_trace.csv"))
    by = defaultdict(list)
    for r in trace:
        by[r["Kernel_Name"]].append((int(r["Grid_Size_X"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"]),
                                     int(r["VGPR_Count"]), int(r["SGPR_Count"])))
    stats = rows(os.path.join(src, "trace", "run_kernel_stats.csv"))

    def pmc(sub, counter):
        out = defaultdict(list)
        p = os.path.join(src, sub, "run_counter_collection.csv")
        if not os.path.exists(p):
            return out
        for r in rows(p):
            if r["Counter_Name"] == counter:
                out[r["Kernel_Name"]].append((int(r["Grid_Size"]), float(r["Counter_Value"])))
        return out

    fetch = pmc("fetch", "FETCH_SIZE")
    write = pmc("write", "WRITE_SIZE")
    summary = {}
    for name, lst in by.items():
        if "rs::" not in name:
            continue
        gmax = max(g for g, *_ in lst)
        # the grid is capped (CUs x blocks/CU), so small launches can share it:
        # keep the dispatches near the median
        durs = full_size([d for g, d, *_ in lst if g == gmax])
        f = full_size([v for g, v in fetch.get(name, []) if g == gmax])
        w = full_size([v for g, v in write.get(name, []) if g == gmax])
        fetch_b = statistics.mean(f) * 1024 * 2 if f else None
        write_b = statistics.mean(w) * 1024 if w else None
        summary[short(name)] = {
            "grid": gmax,
            "dispatches": len(durs),
            "avg_ns": statistics.mean(durs),
            "median_ns": statistics.median(durs),
            "vgpr": lst[0][2],
            "sgpr": lst[0][3],
            "fetch_bytes_corrected": fetch_b,
            "write_bytes": write_b,
            "hbm_bytes": (fetch_b + write_b) if (fetch_b is not None and write_b is not None) else None,
        }
    # bench.py reads hbm_bytes_per_launch[{encode,reconstruct}]
    per_launch = {}
    for k, v in summary.items():
        role = "reconstruct" if k.endswith("true>") else "encode"
        if v["hbm_bytes"] is not None:
            per_launch[role] = v["hbm_bytes"]
    out = {"tag": tag, "workload": workload, "kernels": summary, "hbm_bytes_per_launch": per_launch,
           "correction": "FETCH_SIZE*1024*2 (gfx950 half-count on wide streaming reads) + WRITE_SIZE*1024"}
    os.makedirs(os.path.join(root, "profiles"), exist_ok=True)
    with open(os.path.join(root, "profiles", f"{tag}_pmc.json"), "w") as fjs:
        json.dump(out, fjs, indent=1)
    with open(os.path.join(root, "profiles", f"{tag}_kernel_stats.md"), "w") as fmd:
        fmd.write(f"# rocprofv3 summary {tag}\n\nworkload: `{workload}`\n\n")
        fmd.write("## rocprofv3 --kernel-trace --stats (kernel_stats.csv, all dispatches)\n\n")
        fmd.write("| kernel | calls | avg ns | min ns | max ns | % |\n|---|---|---|---|---|---|\n")
        for r in stats:
            fmd.write(f"| `{short(r['Name'])[:80]}` | {r['Calls']} | {float(r['AverageNs']):.0f} | {r['MinNs']} | "
                      f"{r['MaxNs']} | {float(r['Percentage']):.2f} |\n")
        fmd.write("\n## Full-size dispatches of the RS kernels, with PMC traffic (separate passes)\n\n")
        fmd.write("| kernel | grid | n | avg ns | VGPR | FETCH x2 (B) | WRITE (B) | HBM B/launch | GB/s (HBM/avg) |\n")
        fmd.write("|---|---|---|---|---|---|---|---|---|\n")
        for k, v in summary.items():
            gbs = v["hbm_bytes"] / v["avg_ns"] if v["hbm_bytes"] else float("nan")
            fmd.write(f"| `{k}` | {v['grid']} | {v['dispatches']} | {v['avg_ns']:.0f} | {v['vgpr']} | "
                      f"{v['fetch_bytes_corrected']:.4g} | {v['write_bytes']:.4g} | {v['hbm_bytes']:.4g} | {gbs:.0f} |\n")
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
