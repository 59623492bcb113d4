"""Markdown tables for DESIGN.md §5 / §6 from one tree's evidence files, so every
number there is taken from the committed profiles of that tree:
  profiles/<tag>_bench.json            bench.py line (tools/final_validate.sh a)
  profiles/<tag>_kernel_stats.md, _pmc.json   rocprofv3 of the bench (prof_summary.py)
  profiles/<tag>_sweep_trace.json      the bench's K/M-sweep windows under rocprofv3
  profiles/<tag>_pattern_ceilings.json compute-free twins (ceiling_probe.sh)
  profiles/<tag>_drop_in.log           tools/run_drop_in.sh
  profiles/<tag>_bench_gpus2.json      bench.py --gpus 2 with gloo on one GPU (final_validate.sh b)
Usage: python tools/design_tables.py <tag>   (prints markdown sections)
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P = os.path.join(ROOT, "profiles")


def load(name):
    path = os.path.join(P, name)
    return json.load(open(path)) if os.path.exists(path) else None


def main():
    tag = sys.argv[1]
    b = load(f"{tag}_bench.json")
    pmc = load(f"{tag}_pmc.json")
    sw = load(f"{tag}_sweep_trace.json")
    ce = load(f"{tag}_pattern_ceilings.json")
    out = []
    if b:
        r = b["roofline"]
        out.append(f"### Headline (`profiles/{tag}_bench.json`)\n")
        out.append("| quantity | value |\n|---|---|")
        out.append(f"| `value` | **{b['value']:,.0f} GiB/s** ({b['ms_per_step']} ms per step of encode + per-stripe "
                   f"2-erasure reconstruct, 65 536 × 4 KiB RS(4+2) stripes; sustained "
                   f"{b.get('sustained', {}).get('value_GiBps', 0):,.0f} GiB/s) |")
        km = r["kernel_ms"]
        alg = r["alg_bytes_per_launch"]
        for k in ("encode", "reconstruct"):
            frac = alg[k] / (km[k] * 1e-3) / 1e9 / 8000
            line = f"| {k} kernel, HIP events | {km[k] * 1e3:.2f} µs → **{frac:.3f}** of 8 TB/s"
            if pmc:
                ent = next((v for kk, v in pmc["kernels"].items() if ("true" in kk) == (k == "reconstruct")), None)
                if ent:
                    line += f"; rocprof {ent['avg_ns'] / 1e3:.2f} µs → {alg[k] / ent['avg_ns'] / 8000:.3f}"
                    line += f"; PMC HBM bytes / algorithmic {ent['hbm_bytes'] / alg[k]:.4f}"
            out.append(line + " |")
        out.append(f"| copy yardstick | the reconstruct at {r.get('frac_of_measured_copy')} of the measured copy "
                   f"({b['extras']['copy_kernel_peak_GBps_per_gpu']:,.0f} GB/s), {r.get('frac_of_guide_copy')} of "
                   f"the guide's 6.29 TB/s |")
        if r.get("pattern_ceiling_frac"):
            out.append(f"| compute-free twin of the reconstruct kernel | {r['pattern_ceiling_frac']} |")
        c = b.get("cpu_baseline")
        if c:
            out.append(f"| CPU baseline ({c['kind']}: C restatement of klauspost's AVX-512 GFNI kernels) | "
                       f"{c['value']} GiB/s on {c['cores']} threads, {c['value_1core']} GiB/s on 1 core "
                       f"({c['cpu_model']}); GPU line {b['value'] / c['value']:.0f}× the threaded figure |")
        out.append(f"| parity | `parity_check_full_size` {b['parity_check_full_size']}, `gpu_matches_cpu_sample` "
                   f"{c.get('gpu_matches_cpu_sample') if c else None} |")
        ex = b["extras"]
        out.append("")
        out.append("### Scrub, SHA-256, host-resident paths (same line's `extras`)\n")
        out.append("| leg | rate |\n|---|---|")
        for kk, v in ex.get("scrub_verify_device", {}).items():
            out.append(f"| scrub `{v['kernel']}` {kk} | {v['user_GiBps']:,.0f} GiB/s user, {v['hbm_frac']} of 8 TB/s, "
                       f"ok {v['ok']} |")
        sh = ex.get("sha256_cold_hash_4KiB")
        if sh:
            out.append(f"| batched SHA-256 (`cold_hash`) 65 536 × 4 KiB | {sh['GiBps']:,.0f} GiB/s "
                       f"(CPU {sh['cpu_kind']}, {sh['cpu_threads']} threads: {sh['cpu_baseline_GiBps']} GiB/s), ok {sh['ok']} |")
        he = ex.get("host_e2e_pinned_rs42_4KiB")
        if he:
            out.append(f"| host-resident RS(4+2) 4 KiB, 1 GiB user data, zero-copy (`rs_host_alloc`) | encode "
                       f"{he['zero-copy']['encode_GiBps']} / 1-erasure {he['zero-copy']['reconstruct1_GiBps']} GiB/s |")
            out.append(f"| same, staged (H2D → kernel → D2H) | encode {he['staged']['encode_GiBps']} / 1-erasure "
                       f"{he['staged']['reconstruct1_GiBps']} GiB/s (link {he['h2d_GBps']} GB/s H2D, "
                       f"{he['d2h_GBps']} GB/s D2H) |")
        hm = ex.get("healer_mix_config5")
        if hm:
            e = hm["e2e_GiBps"]
            out.append(f"| config 5 healer mix, 1 M objects 50/50 encode / 1-erasure, host memory | zero-copy "
                       f"**{e.get('zero-copy')} GiB/s** ({hm['e2e_objects_per_s'].get('zero-copy') / 1e6:.1f} M "
                       f"objects/s), staged **{e.get('staged')} GiB/s**; device-resident {hm['device_GiBps']:,.0f} GiB/s; "
                       f"sample ok {hm['ok_sample']} |")
        mc = ex.get("multi_ctx")
        if mc:
            out.append(f"| one context over every visible GPU (`rs_create_multi(4, 2, 0)`, devices {mc['devices']}) | "
                       f"host batch of {mc['objects']:,} × {mc['object_bytes'] // 1024} KiB through `fan_out`: "
                       f"zero-copy encode {mc['zero-copy']['encode_GiBps']} / 1-erasure "
                       f"{mc['zero-copy']['reconstruct1_GiBps']} GiB/s, staged {mc['staged']['encode_GiBps']} / "
                       f"{mc['staged']['reconstruct1_GiBps']} GiB/s; coalesced burst of {mc['coalesced_burst']['objects']:,} "
                       f"× {mc['coalesced_burst']['object_bytes'] // 1024} KiB in {mc['coalesced_burst']['batches']} "
                       f"batches; launches per device {mc['zero-copy']['launches_per_device']} / "
                       f"{mc['staged']['launches_per_device']} / {mc['coalesced_burst']['launches_per_device']}; "
                       f"ok {mc['ok']} |")
    g2 = load(f"{tag}_bench_gpus2.json")
    if g2:
        out.append("")
        out.append(f"### The N-rank line, rehearsed with 2 ranks on one GPU (`profiles/{tag}_bench_gpus2.json`)\n")
        out.append(f"`n_gpus` {g2['n_gpus']}, `physical_gpus` {g2['physical_gpus']}, `value` {g2['value']:,.0f} GiB/s, "
                   f"parity {g2['parity_check_full_size']}. Both ranks share the chip, so each rank alone runs at the "
                   f"GPU's rate and together at half of it: the efficiency fields read about 0.5 here and measure "
                   f"the real thing on distinct GPUs.\n")
        out.append("| leg | per rank concurrent (GiB/s) | per rank alone (GiB/s) | per-GPU efficiency |\n|---|---|---|---|")
        sc = g2.get("scaling_check")
        if sc:
            out.append(f"| headline step ({sc['steps']} steps) | {sc['per_rank_GiBps']} | {sc['solo_GiBps']} | "
                       f"{sc['per_gpu_efficiency']} |")
        for shape, ent in g2.get("extras", {}).get("kmsweep_64KiB_device", {}).items():
            for key in ("encode", "reconstruct2"):
                if f"{key}_per_gpu_efficiency" in ent:
                    out.append(f"| {shape} {key} | {ent[f'{key}_per_rank_GiBps']} | {ent[f'{key}_solo_GiBps']} | "
                               f"{ent[f'{key}_per_gpu_efficiency']} |")
        for path, v in g2.get("extras", {}).get("healer_mix_config5", {}).get("e2e_scaling_check", {}).items():
            out.append(f"| config 5 e2e, {path} | {v['per_rank_GiBps']} | {v['solo_GiBps']} | "
                       f"{v['per_gpu_efficiency']} |")
    if sw:
        out.append("")
        out.append(f"### K/M sweep and config 3 (`profiles/{tag}_sweep_trace.md`"
                   + (f", `profiles/{tag}_pattern_ceilings.json`)" if ce else ")") + "\n")
        out.append("bench = HIP events over ≥ 100 ms of back-to-back launches; rocprof = the same dispatches' average "
                   "in the same process; HBM/alg from separate FETCH_SIZE / WRITE_SIZE passes; ceiling = the "
                   "compute-free twin of the same kernel on the same launch shape, best over occupancy caps.\n")
        out.append("| leg | kernel | bench | rocprof | HBM / alg | ceiling | of ceiling |\n|---|---|---|---|---|---|---|")
        for name, leg in sw["legs"].items():
            leg = dict(leg, leg=name)
            shape, key = name.split(" ", 1)
            c = (ce or {}).get("legs", {}).get(shape, {}).get(key)
            cs = f"{c['ceiling_frac']:.3f}" if c and c["kernel"] == leg["kernel"] else "—"
            of = f"{leg['bench_frac'] / c['ceiling_frac']:.3f}" if c and c["kernel"] == leg["kernel"] else "—"
            out.append(f"| {leg['leg']} | `{leg['kernel']}` | {leg['bench_frac']:.3f} | {leg['rocprof_frac']:.3f} | "
                       f"{leg['hbm_over_alg']:.3f} | {cs} | {of} |" if leg.get("hbm_over_alg") is not None else
                       f"| {leg['leg']} | `{leg['kernel']}` | {leg['bench_frac']:.3f} | {leg['rocprof_frac']:.3f} | — | "
                       f"{cs} | {of} |")
    drop = os.path.join(P, f"{tag}_drop_in.log")
    if os.path.exists(drop):
        out.append("")
        out.append(f"### Per-object drop-in (`profiles/{tag}_drop_in.log`)\n")
        out.append(subprocess.run([sys.executable, os.path.join(ROOT, "tools", "coalesce_table.py"), drop],
                                  capture_output=True, text=True).stdout)
    print("\n".join(out))


if __name__ == "__main__":
    main()
