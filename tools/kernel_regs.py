"""VGPR / spill / occupancy per kernel of a gfx950 HIP file (compiler remarks).
Usage: python tools/kernel_regs.py [file.hip] [name-filter]"""
import re
import subprocess
import sys

import os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = os.path.abspath(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1] else ROOT + "/replication_erasurecoding_object_store_amd/csrc/rs_kernels.hip"
flt = sys.argv[2] if len(sys.argv) > 2 else ""
out = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-c", src, "-o",
                      "/tmp/_regs.o", "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True,
                     cwd="/tmp").stderr
rows, cur = [], None
keys = {"VGPRs": "vgpr", "SGPRs Spill": "sspill", "VGPRs Spill": "vspill", "Occupancy [waves/SIMD]": "occ",
        "ScratchSize [bytes/lane]": "scratch"}
for line in out.splitlines():
    m = re.search(r"remark: Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    for k, short in keys.items():
        m = re.search(r"remark:\s+" + re.escape(k) + r": (\d+)", line)
        if m and cur is not None:
            cur[short] = int(m.group(1))
for r in rows:
    if flt in r["name"]:
        print(f"{r['name'][:64]:64s} " + " ".join(f"{s}={r.get(s)}" for s in keys.values()))
