"""Pairs bench.py --sweep-only legs of the shipped library and of its compute-free
RS_PATTERN_ONLY twin run on the same box (tools/ceiling_probe.sh): per leg, the
shipped kernel's HBM fraction, the twin's (the ceiling of that kernel's memory
pattern on its shipped launch shape) and the headroom between them.

Writes <dir>/ceilings.json and .md; bench.py attaches the newest committed
profiles/*_pattern_ceilings.json to its K/M-sweep entries.
Usage: python tools/ceiling_summary.py gpurun_out/ceiling_<tag> <tag>
"""
import json
import os
import sys


def legs(doc):
    out = {}
    for shape, ent in doc.get("kmsweep_64KiB_device", {}).items():
        for key, kname in ent.get("kernels", {}).items():
            if f"{key}_hbm_frac" in ent:
                out[(shape, key)] = (kname, ent[f"{key}_hbm_frac"])
    for shape, sect in (("rs42_4KiB", doc.get("config3_patterns_and_soa_rs42_4KiB", {})),
                        ("rs42_4KiB", doc.get("headline_rs42_4KiB", {}))):
        for key, ent in sect.items():
            out[(shape, key)] = (ent["kernel"], ent["hbm_frac"])
    return out


def main():
    d, tag = sys.argv[1], sys.argv[2]
    shipped = legs(json.load(open(os.path.join(d, "shipped.json"))))
    twins = {}  # occupancy cap -> legs of the compute-free twin
    for fn in sorted(os.listdir(d)):
        if fn.startswith("pattern_c") and fn.endswith(".json"):
            twins[int(fn[len("pattern_c"):-len(".json")])] = legs(json.load(open(os.path.join(d, fn))))
    rows, doc = [], {"tag": tag, "source": "tools/ceiling_probe.sh (same box, back to back)",
                     "caps": sorted(twins), "legs": {}}
    for (shape, key), (kname, frac) in shipped.items():
        cands = [(tw[(shape, key)][1], cap) for cap, tw in twins.items() if (shape, key) in tw]
        if not cands:
            continue
        ceil, cap = max(cands)
        doc["legs"].setdefault(shape, {})[key] = {
            "kernel": kname, "shipped_frac": frac, "ceiling_frac": ceil, "ceiling_at_cap": cap,
            "twin_by_cap": {str(c): tw[(shape, key)][1] for c, tw in sorted(twins.items()) if (shape, key) in tw},
            "of_ceiling": round(frac / ceil, 4)}
        rows.append(f"| {shape} {key} | `{kname}` | {frac:.4f} | {ceil:.4f} (cap {cap or 'none'}) | "
                    f"{frac / ceil:.3f} | {(ceil - frac) * 100:+.1f} |")
    with open(os.path.join(d, "ceilings.json"), "w") as f:
        json.dump(doc, f, indent=1)
    md = [f"# Compute-free ceilings per leg ({tag})", "",
          "shipped = bench.py --sweep-only HBM fraction of the shipped kernel; ceiling = the best of the same sweep "
          "with the RS_PATTERN_ONLY=1 twin (same launches / loads / stores, one XOR per input dword instead of "
          "GF(2^8) arithmetic) at each occupancy cap (rs_set_occupancy_cap; none = uncapped), same box, back to "
          "back.", "",
          "| leg | kernel | shipped | ceiling | shipped / ceiling | headroom (points) |", "|---|---|---|---|---|---|"]
    md += sorted(rows, key=lambda r: -float(r.split("|")[-2]))
    with open(os.path.join(d, "ceilings.md"), "w") as f:
        f.write("\n".join(md) + "\n")
    print("\n".join(md))


if __name__ == "__main__":
    main()
