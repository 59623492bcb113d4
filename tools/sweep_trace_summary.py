"""bench.py --sweep-only under rocprofv3 (tools/profile_sweep.sh): for every K/M-sweep
and config-3 leg, the HIP-event fraction the bench reported and the rocprof average
of the same dispatches in the same process, plus HBM traffic per dispatch from the
PMC passes (FETCH_SIZE x 1024 x 2 + WRITE_SIZE x 1024, MI355X_MICROARCH.md §HBM).

A leg's timed window is the reps + 2 dispatches of its kernel that follow an idle gap
of >= 2 ms (bench.py idles 3 ms before each window; kernel_ms_events issues two
warm-up launches, then the timed ones), the first such after the previous leg's
window.  The timed ones are the last reps.  The packed device-mask leg's row-offset
scan kernel (one per reconstruct) is left out of the windows: its bench fraction
includes the scan, its rocprof average does not; likewise the host-mask legs' mask
copy kernel (round 6: the masks reach the device through a copy kernel on the launch
stream).

Usage: python tools/sweep_trace_summary.py gpurun_out/sweep_<tag> <tag>
"""
import csv
import json
import os
import statistics
import sys

HBM_PEAK_GBS = 8000.0
SHAPES = {"rs42_64KiB": (4, 2, 16384), "rs84_64KiB": (8, 4, 8192), "rs104_64KiB": (10, 4, 6554)}
E_OF = {"encode": None, "encode_parity_pad": None, "reconstruct2": 2, "reconstruct1": 1,
        "reconstruct2_mslot_out": 2, "reconstruct1_mslot_out": 1, "reconstruct2_out_pad": 2, "reconstruct1_out_pad": 1, "reconstruct2_exact_rows": 2, "reconstruct1_exact_rows": 1,
        "reconstruct2_unbounded": 2, "reconstruct1_unbounded": 1,
        "reconstruct_mixed_unbounded": "mix", "reconstruct_mixed_host": "mix",
        "reconstruct_mixed_packed": "mix", "reconstruct_mixed_packed_host": "mix"}
CONFIG3 = {"rec1_per_stripe_out": 1, "rec_0_1_uniform_out": 2, "rec_0_4_uniform_out": 2,
           "rec_4_5_uniform_out": 2, "soa_encode": 2}


def rows(path):
    with open(path, newline="") as f:
        return list(csv.DictReader(f))


def short(name):
    return name.replace("void ", "").replace("rs::", "").split("(")[0].replace(" ", "")


def legs(doc):
    """(label, kernel, reps, alg_bytes, bench_frac) in execution order."""
    out = []
    for shape, ent in doc["kmsweep_64KiB_device"].items():
        k, m, S = SHAPES[shape]
        N = ent["stripes_per_gpu"]
        for leg in E_OF:
            if f"{leg}_launches" not in ent:
                continue
            e = E_OF[leg] if E_OF[leg] is not None else m
            alg = ent["mixed_alg_bytes"] if e == "mix" else N * S * (k + e)  # mixed: bench's exact count
            out.append((f"{shape} {leg}", ent["kernels"][leg], ent[f"{leg}_launches"], alg,
                        ent[f"{leg}_hbm_frac"]))
    for leg, ent in doc.get("config3_patterns_and_soa_rs42_4KiB", {}).items():
        e = CONFIG3[leg]
        out.append((f"rs42_4KiB {leg}", ent["kernel"], ent["launches"], 65536 * 1024 * (4 + e), ent["hbm_frac"]))
    return out


def windows(trace_csv, want):
    """Dispatches of each leg's timed window: reps + 2 dispatches of the leg's kernel
    starting right after an idle gap of >= 2 ms (bench.py sleeps 3 ms before each
    window); the first two are kernel_ms_events' warm-up launches."""
    aux = ("row_offsets_kernel", "words_copy_kernel")  # a call's helper launches, not legs
    ds = [r for r in rows(trace_csv) if "rs::" in r["Kernel_Name"] and not any(x in r["Kernel_Name"] for x in aux)]
    ds.sort(key=lambda r: int(r["Start_Timestamp"]))
    res, pos = [], 0
    for label, kern, reps, alg, frac in want:
        found = None
        for i in range(pos, len(ds) - reps - 1):
            if i > 0 and int(ds[i]["Start_Timestamp"]) - int(ds[i - 1]["End_Timestamp"]) < 2_000_000:
                continue
            if short(ds[i]["Kernel_Name"]) != kern.replace(" ", ""):
                continue
            if all(ds[j]["Kernel_Name"] == ds[i]["Kernel_Name"] for j in range(i, i + reps + 2)):
                found = ds[i + 2:i + reps + 2]
                pos = i + reps + 2
                break
        res.append(found)
    return res


def main():
    src, tag = sys.argv[1], sys.argv[2]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    doc = json.load(open(os.path.join(src, "trace.json")))
    want = legs(doc)
    tw = windows(os.path.join(src, "trace", "run_kernel_trace.csv"), want)
    traffic = {}
    for pas, counter in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE")):
        pdir = os.path.join(src, pas)
        if not os.path.exists(os.path.join(pdir, "run_counter_collection.csv")):
            continue
        pdoc = json.load(open(os.path.join(src, f"{pas}.json")))
        pw = windows(os.path.join(pdir, "run_kernel_trace.csv"), legs(pdoc))
        vals = {}
        for r in rows(os.path.join(pdir, "run_counter_collection.csv")):
            if r["Counter_Name"] == counter:
                vals[r["Dispatch_Id"]] = float(r["Counter_Value"])
        for (label, *_), win in zip(legs(pdoc), pw):
            if win:
                v = [vals[d["Dispatch_Id"]] for d in win if d["Dispatch_Id"] in vals]
                if v:
                    traffic.setdefault(label, {})[counter] = statistics.mean(v)
    lines = [f"# bench.py K/M sweep + config 3 under rocprofv3, same process ({tag})", "",
             "HIP-event fraction = what bench.py reported for the leg; rocprof = mean duration of the same "
             "timed dispatches in the same process; HBM from separate FETCH_SIZE / WRITE_SIZE passes "
             "(each its own bench.py --sweep-only process).", "",
             "| leg | kernel | dispatches | bench frac | rocprof avg us | rocprof frac | diff (points) | HBM / alg |",
             "|---|---|---|---|---|---|---|---|"]
    table, worst = {}, 0.0
    for (label, kern, reps, alg, frac), win in zip(want, tw):
        if not win:
            lines.append(f"| {label} | `{kern}` | (window not found) | {frac:.4f} | | | | |")
            continue
        avg = statistics.mean(int(d["End_Timestamp"]) - int(d["Start_Timestamp"]) for d in win)
        rf = alg / avg / HBM_PEAK_GBS
        diff = (frac - rf) * 100
        worst = max(worst, abs(diff))
        t = traffic.get(label, {})
        hb = ""
        if "FETCH_SIZE" in t and "WRITE_SIZE" in t:
            hb = f"{(t['FETCH_SIZE'] * 2048 + t['WRITE_SIZE'] * 1024) / alg:.3f}"
        lines.append(f"| {label} | `{kern}` | {len(win)} | {frac:.4f} | {avg / 1e3:.1f} | {rf:.4f} | {diff:+.2f} | {hb} |")
        table[label] = {"kernel": kern, "dispatches": len(win), "bench_frac": frac, "rocprof_avg_ns": avg,
                        "rocprof_frac": round(rf, 4), "hbm_over_alg": float(hb) if hb else None}
    lines += ["", f"largest |bench - rocprof|: {worst:.2f} points"]
    text = "\n".join(lines) + "\n"
    print(text)
    with open(os.path.join(root, "profiles", f"{tag}_sweep_trace.md"), "w") as f:
        f.write(text)
    with open(os.path.join(root, "profiles", f"{tag}_sweep_trace.json"), "w") as f:
        json.dump({"tag": tag, "legs": table, "max_abs_diff_points": round(worst, 2)}, f, indent=1)


if __name__ == "__main__":
    main()
