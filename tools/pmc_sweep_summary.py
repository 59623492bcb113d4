"""Summarise tools/profile_kmsweep_pmc.sh output: per workload, the RS kernel's
full-size dispatches -- average duration (kernel trace), HBM bytes per launch
(FETCH_SIZE x 1024 x 2 + WRITE_SIZE x 1024, gfx950 corrections as in
tools/prof_summary.py) against the workload's algorithmic bytes (tools/ab_bench.py).

Usage: python tools/pmc_sweep_summary.py gpurun_out/pmc_<tag> <tag>
"""
import csv
import json
import os
import statistics
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import ab_bench  # noqa: E402


def rows(path):
    with open(path, newline="") as f:
        return list(csv.DictReader(f))


def full_size(vals):
    """Drop dispatches far below the median (the workload's small correctness-check
    launches run with the same capped grid as the full-size ones)."""
    med = statistics.median(vals)
    return [v for v in vals if v >= 0.5 * med]


def main():
    src, tag = sys.argv[1], sys.argv[2]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    lines = [f"# HBM traffic per launch, K/M sweep workloads ({tag})", "",
             "rocprofv3 --kernel-trace (durations) and separate --pmc FETCH_SIZE / WRITE_SIZE passes; "
             "FETCH_SIZE x 1024 x 2, WRITE_SIZE x 1024 (MI355X_MICROARCH.md §HBM).", "",
             "| workload | kernel | n | avg us | alg MB | fetch MB | write MB | HBM / alg | alg GB/s | % of 8 TB/s |",
             "|---|---|---|---|---|---|---|---|---|---|"]
    table = {}
    for w in sorted(os.listdir(src)):
        d = os.path.join(src, w)
        tr = os.path.join(d, "trace", "run_kernel_trace.csv")
        if not os.path.exists(tr) or w not in ab_bench.WORKLOADS:
            continue
        durs = defaultdict(list)
        for r in rows(tr):
            if "rs::" in r["Kernel_Name"]:
                durs[(r["Kernel_Name"], int(r["Grid_Size_X"]))].append(
                    int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
        (name, grid), ds = max(durs.items(), key=lambda kv: (len(kv[1]), kv[0][1]))
        ds = full_size(ds)  # the grid is capped, so small check launches share it

        def pmc(sub, counter):
            p = os.path.join(d, sub, "run_counter_collection.csv")
            if not os.path.exists(p):
                return None
            v = [float(r["Counter_Value"]) for r in rows(p)
                 if r["Counter_Name"] == counter and r["Kernel_Name"] == name and int(r["Grid_Size"]) == grid]
            return statistics.mean(full_size(v)) if v else None

        f, wr = pmc("fetch", "FETCH_SIZE"), pmc("write", "WRITE_SIZE")
        alg = ab_bench.alg_bytes(w)
        avg = statistics.mean(ds)
        fb = f * 1024 * 2 if f is not None else float("nan")
        wb = wr * 1024 if wr is not None else float("nan")
        short = name.replace("void ", "").split("(")[0]
        lines.append(f"| {w} | `{short}` | {len(ds)} | {avg / 1e3:.1f} | {alg / 1e6:.1f} | {fb / 1e6:.1f} | "
                     f"{wb / 1e6:.1f} | {(fb + wb) / alg:.3f} | {alg / avg:.0f} | {alg / avg / 80:.1f} |")
        table[w] = {"kernel": short, "dispatches": len(ds), "avg_ns": avg, "alg_bytes": alg,
                    "hbm_bytes": (fb + wb) if f is not None and wr is not None else None,
                    "hbm_frac": alg / avg / 8000.0}
    out = os.path.join(root, "profiles", f"{tag}_kmsweep_pmc.md")
    with open(out, "w") as fo:
        fo.write("\n".join(lines) + "\n")
    with open(os.path.join(root, "profiles", f"{tag}_kmsweep_pmc.json"), "w") as fo:
        json.dump({"tag": tag, "workloads": table}, fo, indent=1)
    print("\n".join(lines))


if __name__ == "__main__":
    main()
