#!/usr/bin/env python3
"""Static VALU issue-cost model of a kernel's gfx950 assembly.

Counts the instructions of one kernel in `make asm` output
(neurokmer_amd/build/nk_kernels.s) and prices each VALU instruction with the
issue costs measured by tools/isabench.hip on MI355X (profiles/r02_s1/
isabench.log): full-rate ops ~2.4 clk per wave64 instruction, half-rate ops
(shifts left, alignbit, perm, 64-bit adds, multiplies, carry adds, cndmask,
compares, any VGPR op with an SGPR source) ~4.2.  Prints the per-class totals
and, with --per N, the cost per N units (e.g. k-mers per wave).

    python tools/valu_model.py k_part --per 1024      # 16 k-mers x 64 lanes
"""
import argparse
import re
import sys
from collections import Counter

FULL = {"v_xor_b32", "v_add_u32", "v_sub_u32", "v_subrev_u32", "v_and_b32", "v_or_b32",
        "v_mov_b32", "v_bitop3_b32", "v_lshrrev_b32", "v_not_b32"}
COST_FULL, COST_HALF, COST_MAD = 2.4, 4.2, 4.5


def kernel_lines(path, name):
    lines = open(path).read().split("\n")
    start = None
    for i, l in enumerate(lines):
        if re.match(r"^_ZN2nk\d+" + re.escape(name) + r"[A-Z0-9I].*:", l) or \
           re.match(r"^_ZN2nk\d+" + re.escape(name) + "ILb", l):
            start = i
            break
    if start is None:
        sys.exit(f"kernel {name} not found")
    out = []
    for l in lines[start + 1:]:
        if "s_endpgm" in l:
            break
        out.append(l)
    return lines[start], out


def price(op, args):
    base = re.sub(r"_e(32|64)$", "", op)
    if op.startswith("v_mad") or op.startswith("v_mul_hi") or op.startswith("v_mul_lo"):
        return COST_MAD if "mad" in op else COST_HALF, "mul"
    sgpr = re.search(r"\bs\[?\d", args) is not None and not base.startswith("v_cndmask") \
        and not base.startswith("v_cmp")
    if base in FULL and not sgpr:
        return COST_FULL, "full"
    return COST_HALF, "half"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("kernel")
    ap.add_argument("--asm", default="neurokmer_amd/build/nk_kernels.s")
    ap.add_argument("--per", type=float, default=1.0)
    a = ap.parse_args()
    head, body = kernel_lines(a.asm, a.kernel)
    ops, cost, cls = Counter(), Counter(), Counter()
    total = 0.0
    for l in body:
        m = re.match(r"^\s+(v_[a-z0-9_]+)\s*(.*)$", l)
        if not m:
            n = re.match(r"^\s+s_nop\s+(\d+)", l)
            if n:
                ops["s_nop"] += 1
            continue
        op, args = m.group(1), m.group(2)
        c, k = price(op, args)
        ops[op] += 1
        cost[op] += c
        cls[k] += c
        total += c
    print(head.split(":")[0][:100])
    print(f"VALU instructions {sum(v for k, v in ops.items() if k != 's_nop')}, "
          f"issue clk {total:.0f}, per unit {total / a.per:.2f}")
    for op, c in cost.most_common(25):
        print(f"  {op:28s} n={ops[op]:5d}  clk={c:8.1f}  per unit={c / a.per:6.2f}")
    print("  classes:", {k: round(v / a.per, 2) for k, v in cls.items()}, " s_nop:", ops["s_nop"])


if __name__ == "__main__":
    main()
