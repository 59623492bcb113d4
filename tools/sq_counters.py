"""Summarise a rocprofv3 --pmc SQ_* counter collection per kernel (full-size
dispatches only): wave-cycle fractions busy / waiting, VALU instructions.
Usage: python tools/sq_counters.py <run_counter_collection.csv> [name-filter]"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
flt = sys.argv[2] if len(sys.argv) > 2 else "rs::"
by = defaultdict(lambda: defaultdict(float))
grid = defaultdict(int)
for r in rows:
    if flt not in r["Kernel_Name"]:
        continue
    key = (r["Kernel_Name"].split("(")[0].replace("void ", ""), r["Dispatch_Id"])
    by[key][r["Counter_Name"]] += float(r["Counter_Value"])
    grid[key] = int(r["Grid_Size"])
agg = defaultdict(lambda: defaultdict(list))
for (name, _), c in by.items():
    g = max(gv for (n, _), gv in grid.items() if n == name)
    if grid[(name, _)] != g:
        continue
    for k, v in c.items():
        agg[name][k].append(v)
for name, c in agg.items():
    avg = {k: sum(v) / len(v) for k, v in c.items()}
    wc = avg.get("SQ_WAVE_CYCLES", 0) or 1
    print(name)
    for k in sorted(avg):
        frac = f"  ({avg[k] / wc * 100:5.1f}% of wave-cycles)" if k.startswith(("SQ_WAIT", "SQ_ACTIVE", "SQ_BUSY")) else ""
        print(f"  {k:24s} {avg[k]:16.0f}{frac}")
