"""Per-dispatch duration and effective clock (GRBM_GUI_ACTIVE / 8 / duration) from a
rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE directory (tools/profile_clock.sh)."""
import csv
import glob
import sys

d, flt = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "rs::")
pmc = {}
for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if flt in r["Kernel_Name"]:
            key = r["Dispatch_Id"]
            pmc.setdefault(key, [r["Kernel_Name"].split("(")[0], 0.0])[1] += float(r["Counter_Value"])
dur = {}
for f in glob.glob(d + "/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        dur[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
print(d)
for k in sorted(pmc, key=int):
    name, cyc = pmc[k]
    us = dur.get(k)
    if us and us > 50:
        print(f"  {name[:44]:44s} {us:8.1f} us  {cyc / 8 / (us * 1e-6) / 1e9:5.2f} GHz")
