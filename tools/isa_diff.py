"""Per-kernel ISA comparison of two device-assembly files of rs_kernels.hip.

Produce each with
  hipcc -O3 -std=c++17 --offload-arch=gfx950 --cuda-device-only -S rs_kernels.hip -o X.s
Comments and basic-block label numbers are ignored, so a source change that leaves a
kernel's code alone (a removed switch, a reworded comment) reports it as identical.
Usage: python tools/isa_diff.py before.s after.s
"""
import re
import sys


def kernels(path):
    out, cur, name = {}, [], None
    for line in open(path).read().split("\n"):
        m = re.match(r"^(_ZN2rs\w+):", line)
        if m:
            name, cur = m.group(1), []
        if name:
            code = re.sub(r"\.LBB\d+_", ".LBB_", line.split(";")[0].rstrip())
            if code.strip():
                cur.append(code)
            if "s_endpgm" in line:
                out[name] = "\n".join(cur)
                name = None
    return out


def main():
    a, b = kernels(sys.argv[1]), kernels(sys.argv[2])
    for k in sorted(set(a) | set(b)):
        if k not in b:
            print("removed  ", k)
        elif k not in a:
            print("added    ", k)
        elif a[k] != b[k]:
            print("changed  ", k)
    same = sum(1 for k in a if k in b and a[k] == b[k])
    print(f"identical: {same} of {len(b)} kernels in {sys.argv[2]}")


if __name__ == "__main__":
    main()
