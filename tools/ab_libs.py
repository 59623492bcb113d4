"""A/B two builds of librsgpu.so (same ABI, different kernel code): runs
tools/ab_bench.py once per library per round, alternating, each in its own child
process (RSGPU_LIB selects the build), and prints the median GB/s per
(workload, blocks/CU, library).

Usage: python tools/ab_libs.py --libs a.so,b.so [--rounds 3] [ab_bench args...]
"""
import argparse
import os
import re
import subprocess
import sys
from collections import defaultdict

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LINE = re.compile(r"^(\S+)\s+v\d+ bpc=\s*(\d+): median\s+([\d.]+) GB/s")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", default="", help="comma-separated alternative builds of librsgpu.so")
    ap.add_argument("--env-variants", default="",
                    help="comma-separated VAR=VALUE settings, each run as its own variant on the default build")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--timeout", type=int, default=240, help="seconds per child run")
    ap.add_argument("--no-check", default="", help="comma-separated libs whose parity check is not enforced "
                                                   "(diagnostic builds that skip work)")
    args, rest = ap.parse_known_args()
    variants = [(os.path.basename(x), {"RSGPU_LIB": os.path.abspath(x)}) for x in args.libs.split(",") if x]
    for ev in [e for e in args.env_variants.split(",") if e]:
        k, v = ev.split("=", 1)
        variants.append((ev, {k: v}))
    res = defaultdict(list)
    for rnd in range(args.rounds):
        for lib, extra in variants:
            env = dict(os.environ, **extra)
            cmd = [sys.executable, os.path.join(HERE, "ab_bench.py"), "--rounds", "1", *rest]
            p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=args.timeout)
            if p.returncode != 0:
                print(p.stdout[-2000:], p.stderr[-4000:], flush=True)
                raise SystemExit(f"child failed ({p.returncode}) for {lib}")
            for line in p.stdout.splitlines():
                mm = LINE.match(line)
                if mm:
                    res[(mm.group(1), int(mm.group(2)), lib)].append(float(mm.group(3)))
                elif "parity-consistent" in line and "True" not in line and lib not in args.no_check.split(","):
                    raise SystemExit(f"parity check failed for {lib}: {line}")
            print(f"round {rnd} {lib} done", flush=True)
    for key in sorted(res):
        v = res[key]
        print(f"{key[0]:20s} bpc={key[1]:2d} {key[2]:28s} median {np.median(v):7.1f} GB/s "
              f"({np.median(v) / 80:4.1f}% of 8 TB/s)  n={len(v)}", flush=True)


if __name__ == "__main__":
    main()
