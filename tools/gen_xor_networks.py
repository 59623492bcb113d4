"""Generates csrc/rs_xor_networks.inc: bitsliced encode XOR programs for the fixed
encode matrices of the specialised (K, M) shapes.

Why: GF(2^8) multiplication by a constant f is GF(2)-linear, an 8x8 bit matrix.
With the data bitsliced (plane j = bit j of 32 bytes in one dword), one parity
plane is the XOR of the data planes whose matrix bit is set: full-rate v_xor_b32
instead of half-rate v_perm_b32 lookups (tools/valu_probe.hip).  The encode matrix
of RS(K, M) is fixed ([upstream klauspost matrix.go buildMatrix]: vandermonde(K+M,
K) x inv(top K x K)), so its XOR program is known at build time and common
subexpressions can be shared.

Inputs are streamed one at a time (input c's 8 planes are live only while its
contributions are folded into the 8M output planes), and the common pairs inside
one input's 8M row subsets are shared by Paar's greedy algorithm (repeatedly
materialise the pair that occurs in the most rows).  The generated step for input
c is straight-line code:  t_i = a ^ b; ...; y[p] = / ^= <one value>.

Also emitted: the parity rows each program was derived from (rs_create checks
them against the runtime encode matrix before the bitsliced kernel may run).

Usage: python tools/gen_xor_networks.py  (writes the .inc; committed)
"""
from __future__ import annotations

import os
from collections import Counter

SHAPES = [(4, 2), (8, 4), (10, 4), (6, 3)]
PAIR_SHAPES = [(8, 4), (10, 4)]  # 1 KiB-task pair programs (encode_bs16_kernel)
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                   "replication_erasurecoding_object_store_amd", "csrc", "rs_xor_networks.inc")

# ---- GF(2^8), poly 0x11d, generator 2 ([upstream klauspost galois.go]) ------------
EXP = [0] * 512
LOG = [0] * 256
x = 1
for i in range(255):
    EXP[i] = x
    LOG[x] = i
    x <<= 1
    if x & 0x100:
        x ^= 0x11D
for i in range(255, 512):
    EXP[i] = EXP[i - 255]


def mul(a: int, b: int) -> int:
    return 0 if a == 0 or b == 0 else EXP[LOG[a] + LOG[b]]


def gpow(a: int, n: int) -> int:
    if n == 0:
        return 1
    return 0 if a == 0 else EXP[(LOG[a] * n) % 255]


def inv_matrix(a):
    n = len(a)
    w = [row[:] + [1 if i == r else 0 for i in range(n)] for r, row in enumerate(a)]
    for col in range(n):
        piv = next(r for r in range(col, n) if w[r][col])
        w[col], w[piv] = w[piv], w[col]
        s = EXP[255 - LOG[w[col][col]]]
        w[col] = [mul(v, s) for v in w[col]]
        for r in range(n):
            if r != col and w[r][col]:
                f = w[r][col]
                w[r] = [v ^ mul(f, u) for v, u in zip(w[r], w[col])]
    return [row[n:] for row in w]


def parity_rows(k: int, m: int):
    v = [[gpow(r, c) for c in range(k)] for r in range(k + m)]
    ti = inv_matrix(v[:k])
    enc = [[0] * k for _ in range(k + m)]
    for r in range(k + m):
        for c in range(k):
            acc = 0
            for i in range(k):
                acc ^= mul(v[r][i], ti[i][c])
            enc[r][c] = acc
    return enc[k:]


# ---- XOR programs ---------------------------------------------------------------
# Sharing pairs across groups of inputs (group size > 1: fewer XORs, more planes
# live) was measured level or slower on the GPU (round 4,
# profiles/r04r_ab_bitsliced_groups.log); program(..., cs) still takes a group.


def group_rows(rows, m, cs):
    """Output plane p = (r*8 + i) of parity row r < m needs the XOR of the input
    planes (ci*8 + j) of inputs cs[ci] whose GF(2) matrix bit is set:
    bit i of f_rc * 2^j."""
    out = []
    for r in range(m):
        for i in range(8):
            out.append(frozenset(ci * 8 + j for ci, c in enumerate(cs) for j in range(8)
                                 if (mul(rows[r][c], 1 << j) >> i) & 1))
    return out


def paar(subsets):
    """Greedy common-pair elimination.  Returns (temps, rows): temps = list of
    (name, a, b); rows = list of sets of operand names (x<j> / t<i>)."""
    rows = [set(f"x{j}" for j in s) for s in subsets]
    temps = []
    while True:
        cnt = Counter()
        for r in rows:
            ls = sorted(r)
            for a in range(len(ls)):
                for b in range(a + 1, len(ls)):
                    cnt[(ls[a], ls[b])] += 1
        if not cnt:
            break
        (a, b), n = max(cnt.items(), key=lambda kv: (kv[1], kv[0]))
        if n < 2:
            break
        name = f"t{len(temps)}"
        temps.append((name, a, b))
        for r in rows:
            if a in r and b in r:
                r.discard(a)
                r.discard(b)
                r.add(name)
    return temps, rows


def program(k, m, cs):
    """XOR program of inputs cs (a group, or one input): (temps, rows)."""
    return paar(group_rows(parity_rows(k, m), m, cs))


def evaluate(k, m, planes_by_input, group=1):
    """Reference evaluation of the programs (tests): planes_by_input[c] = 8 plane
    words of input c; returns the 8m parity plane words."""
    y = [0] * (8 * m)
    for c0 in range(0, k, group):
        cs = list(range(c0, min(k, c0 + group)))
        temps, red = program(k, m, cs)
        env = {f"x{ci * 8 + j}": planes_by_input[c][j] for ci, c in enumerate(cs) for j in range(8)}
        for name, a, b in temps:
            env[name] = env[a] ^ env[b]
        for p, r in enumerate(red):
            for o in r:
                y[p] ^= env[o]
    return y


def _operand(o):
    return f"x[{o[1:]}]" if o[0] == "x" else o


def emit(k, m, c):
    """bs_step<k, m, c>: input c's contribution to every parity plane."""
    temps, red = program(k, m, [c])
    first = c == 0
    lines = [f"template <> __device__ __forceinline__ void bs_step<{k}, {m}, {c}>(const uint32_t (&x)[8], "
             f"uint32_t (&y)[{8 * m}]) {{"]
    nx = 0
    for name, a, b in temps:
        lines.append(f"  const uint32_t {name} = {_operand(a)} ^ {_operand(b)};")
        nx += 1
    for p, r in enumerate(red):
        ops = [_operand(o) for o in sorted(r)]
        if not ops:
            if first:
                lines.append(f"  y[{p}] = 0u;")
            continue
        expr = " ^ ".join(ops)
        nx += len(ops) - 1
        if first:
            lines.append(f"  y[{p}] = {expr};")
        else:
            lines.append(f"  y[{p}] ^= {expr};")
            nx += 1
    lines.append("}")
    return lines, nx


# ---- 1 KiB-task programs on input pairs ----------------------------------------
# The encode matrices of RS(8+4) and RS(10+4) satisfy C[r ^ 1][c] = C[r][c ^ 1].  A
# lane holding 16 B of inputs c (even) and c ^ 1 transposes them together: plane j,
# low nibble of every byte = bit j of 4 bytes of input c, high nibble = of input c ^ 1.
# For an even row r, A = C[r][c] and B = C[r][c ^ 1]:  A * P + B * nibswap(P) carries
# row r's terms of both inputs in the low nibbles and row r ^ 1's in the high nibbles.
# The kernel accumulates A * P (ya) and B * P (yb) and combines ya ^ nibswap(yb) once
# per column, so one program over M / 2 packed rows serves all M rows.


def pair_symmetric(k: int, m: int) -> bool:
    rows = parity_rows(k, m)
    return k % 2 == 0 and m % 2 == 0 and all(
        rows[r ^ 1][c] == rows[r][c ^ 1] for r in range(m) for c in range(k))


def pair_program(k, m, p):
    """Program of input pair (2p, 2p+1): output planes 0..4m-1 = ya (A terms of the
    packed rows 0, 2, ..), 4m..8m-1 = yb (B terms)."""
    rows = parity_rows(k, m)
    coefs = [rows[r][2 * p] for r in range(0, m, 2)] + [rows[r][2 * p + 1] for r in range(0, m, 2)]
    subsets = []
    for f in coefs:
        for i in range(8):
            subsets.append(frozenset(j for j in range(8) if (mul(f, 1 << j) >> i) & 1))
    return paar(subsets)


def evaluate_pairs(k, m, planes_by_input):
    """Reference evaluation of the pair programs on 32-bit planes whose low 16 bits
    hold the input of the pair's even member and high 16 bits its odd member (the
    kernel's nibbles, spread for the test): returns the 8m parity planes, row r's
    plane i in the low 16 bits of y[(r // 2) * 8 + i] when r is even, high when odd."""
    half = 4 * m
    ya, yb = [0] * half, [0] * half
    for p in range(k // 2):
        P = [(planes_by_input[2 * p][j] & 0xFFFF) | ((planes_by_input[2 * p + 1][j] & 0xFFFF) << 16)
             for j in range(8)]
        temps, red = pair_program(k, m, p)
        env = {f"x{j}": P[j] for j in range(8)}
        for name, a, b in temps:
            env[name] = env[a] ^ env[b]
        for q, r in enumerate(red):
            for o in r:
                if q < half:
                    ya[q] ^= env[o]
                else:
                    yb[q - half] ^= env[o]
    swap = [((v >> 16) | (v << 16)) & 0xFFFFFFFF for v in yb]
    return [a ^ b for a, b in zip(ya, swap)]


def emit_pair(k, m, p):
    """bs16_step<k, m, p>: input pair p's contribution to ya / yb."""
    temps, red = pair_program(k, m, p)
    half = 4 * m
    first = p == 0
    lines = [f"template <> __device__ __forceinline__ void bs16_step<{k}, {m}, {p}>(const uint32_t (&x)[8], "
             f"uint32_t (&ya)[{half}], uint32_t (&yb)[{half}]) {{"]
    nx = 0
    for name, a, b in temps:
        lines.append(f"  const uint32_t {name} = {_operand(a)} ^ {_operand(b)};")
        nx += 1
    for q, r in enumerate(red):
        dst = f"ya[{q}]" if q < half else f"yb[{q - half}]"
        ops = [_operand(o) for o in sorted(r)]
        if not ops:
            if first:
                lines.append(f"  {dst} = 0u;")
            continue
        nx += len(ops) - 1
        if first:
            lines.append(f"  {dst} = {' ^ '.join(ops)};")
        else:
            lines.append(f"  {dst} ^= {' ^ '.join(ops)};")
            nx += 1
    lines.append("}")
    return lines, nx


def main():
    out = ["// rs_xor_networks.inc -- GENERATED by tools/gen_xor_networks.py; do not edit.",
           "// Bitsliced encode XOR programs for the fixed RS(K, M) encode matrices",
           "// ([upstream klauspost matrix.go buildMatrix]); see rs_kernels.hip.", ""]
    summary = []
    for k, m in SHAPES:
        rows = parity_rows(k, m)
        out.append(f"// ---- RS({k}+{m}) parity rows: {rows}")
        flat = ", ".join(str(v) for r in rows for v in r)
        out.append(f"template <> struct BsNet<{k}, {m}> {{")
        out.append("  static constexpr bool kAvailable = true;")
        out.append(f"  static constexpr uint8_t kRows[{k * m}] = {{{flat}}};")
        out.append("};")
        total = 0
        for c in range(k):
            lines, nx = emit(k, m, c)
            out += lines
            total += nx
        out.append("")
        summary.append(f"RS({k}+{m}): {total} v_xor_b32 per 32-byte column")
        if (k, m) in PAIR_SHAPES:
            assert pair_symmetric(k, m), (k, m)
            out.append(f"template <> struct Bs16Net<{k}, {m}> {{")
            out.append("  static constexpr bool kAvailable = true;")
            out.append("};")
            total = 0
            for p in range(k // 2):
                lines, nx = emit_pair(k, m, p)
                out += lines
                total += nx
            out.append("")
            summary.append(f"RS({k}+{m}) pairs: {total} v_xor_b32 per 16-byte column")
    out.insert(3, "// " + "; ".join(summary))
    with open(OUT, "w") as f:
        f.write("\n".join(out) + "\n")
    print("\n".join(summary))


if __name__ == "__main__":
    main()
