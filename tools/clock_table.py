"""Per-kernel clock/duration trajectory from tools/profile_clock.sh output
(clock_summary.py lines): first/last launches and medians, one row per kernel."""
import re
import statistics
import sys

for path in sys.argv[1:]:
    cur = None
    rows = {}
    for line in open(path):
        if line.startswith("gpurun_out"):
            cur = line.strip()
        m = re.match(r"\s+(\S.*?)\s+([\d.]+) us\s+([\d.]+) GHz", line)
        if m and cur:
            rows.setdefault((cur, m.group(1).strip()), []).append((float(m.group(2)), float(m.group(3))))
    for (w, k), v in rows.items():
        big = [r for r in v if r[0] > 150]
        if len(big) < 5:
            continue
        print(f"{w.split('/')[-1]:22s} {k[5:45]:40s} n={len(big):3d} first3 {[round(r[0]) for r in big[:3]]} "
              f"last5 {[round(r[0]) for r in big[-5:]]} median {statistics.median(r[0] for r in big):6.1f} us "
              f"@ {statistics.median(r[1] for r in big):.2f} GHz (last5 {statistics.mean(r[1] for r in big[-5:]):.2f})")
