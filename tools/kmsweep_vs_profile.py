"""bench.py's sustained K/M sweep and config-3 patterns against the committed
rocprofv3 summaries of the same kernels (tools/profile_kmsweep_pmc.sh ->
tools/pmc_sweep_summary.py): both time >= 100 ms of back-to-back launches, so the
HIP-event fraction and the rocprof fraction should agree to about a point.

Usage: python tools/kmsweep_vs_profile.py <bench.json> <profiles/<tag>_kmsweep_pmc.json> [out.md]
"""
import json
import sys

# bench key -> (tools/ab_bench.py workload, bench field)
PAIRS = [
    ("rs42_64KiB", "encode", "rs42_64K_enc"),
    ("rs42_64KiB", "reconstruct2", "rs42_64K_rec2p_out"),
    ("rs42_64KiB", "reconstruct1", "rs42_64K_rec1pb_out"),
    ("rs84_64KiB", "encode", "rs84_64K_enc"),
    ("rs84_64KiB", "reconstruct2", "rs84_64K_rec2pb_out"),
    ("rs84_64KiB", "reconstruct1", "rs84_64K_rec1pb_out"),
    ("rs84_64KiB", "reconstruct2_unbounded", "rs84_64K_rec2p_out"),
    ("rs84_64KiB", "reconstruct1_unbounded", "rs84_64K_rec1p_out"),
    ("rs104_64KiB", "encode", "rs104_64K_enc"),
    ("rs104_64KiB", "reconstruct2", "rs104_64K_rec2pb_out"),
    ("rs104_64KiB", "reconstruct1", "rs104_64K_rec1pb_out"),
    ("rs104_64KiB", "reconstruct2_unbounded", "rs104_64K_rec2p_out"),
    ("rs104_64KiB", "reconstruct1_unbounded", "rs104_64K_rec1p_out"),
]
CONFIG3 = [("rec1_per_stripe_out", "rs42_4K_rec1pb_out"), ("rec_0_1_uniform_out", "rs42_4K_rec2u_out"),
           ("rec_0_4_uniform_out", "rs42_4K_rec04u_out"), ("rec_4_5_uniform_out", "rs42_4K_rec45u_out")]


def main():
    bench = json.load(open(sys.argv[1]))
    prof = json.load(open(sys.argv[2]))["workloads"]
    ex = bench["extras"]
    rows = ["| shape | leg | bench kernel | bench frac (HIP events, >= 100 ms) | rocprof workload | rocprof kernel "
            "| rocprof frac | HBM / alg | diff (points) |", "|---|---|---|---|---|---|---|---|---|"]
    worst = 0.0

    def add(shape, leg, kern, frac, w):
        nonlocal worst
        p = prof.get(w)
        if not p:
            rows.append(f"| {shape} | {leg} | `{kern}` | {frac:.4f} | {w} | (not profiled) | | | |")
            return
        d = (frac - p["hbm_frac"]) * 100
        worst = max(worst, abs(d))
        hb = f"{p['hbm_bytes'] / p['alg_bytes']:.3f}" if p.get("hbm_bytes") else ""
        rows.append(f"| {shape} | {leg} | `{kern}` | {frac:.4f} | {w} | `{p['kernel']}` | {p['hbm_frac']:.4f} | {hb} "
                    f"| {d:+.2f} |")

    for shape, leg, w in PAIRS:
        ent = ex["kmsweep_64KiB_device"].get(shape, {})
        if f"{leg}_hbm_frac" in ent:
            add(shape, leg, ent["kernels"].get(leg, ""), ent[f"{leg}_hbm_frac"], w)
    for leg, w in CONFIG3:
        ent = ex.get("config3_patterns_and_soa_rs42_4KiB", {}).get(leg)
        if ent:
            add("rs42_4KiB", leg, ent.get("kernel", ""), ent["hbm_frac"], w)
    rows.append("")
    rows.append(f"largest |bench - rocprof|: {worst:.2f} points")
    text = "\n".join(rows) + "\n"
    print(text)
    if len(sys.argv) > 3:
        open(sys.argv[3], "w").write(text)


if __name__ == "__main__":
    main()
