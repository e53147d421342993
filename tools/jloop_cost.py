#!/usr/bin/env python3
"""Static issue cost of ONE unrolled window iteration of K1a (the code between
two consecutive rank atomics, ds_add_rtn_u32), priced by tools/valu_model.py.
    python tools/jloop_cost.py <asm> <kernel-substring>"""
import re
import sys
sys.path.insert(0, __import__("os").path.dirname(__file__))
from valu_model import kernel_lines, price  # noqa: E402

asm, name = sys.argv[1], sys.argv[2]
_, body = kernel_lines(asm, name)
marks = [i for i, l in enumerate(body) if "ds_add_rtn_u32" in l]
costs = []
for a, b in zip(marks[:-1], marks[1:]):
    c = 0.0
    n = 0
    for l in body[a + 1:b]:
        m = re.match(r"^\s+(v_[a-z0-9_]+)\s*(.*)$", l)
        if m:
            c += price(m.group(1), m.group(2))[0]
            n += 1
    costs.append((n, round(c, 1)))
print(name, "iterations:", len(costs), "median clk:", sorted(x[1] for x in costs)[len(costs) // 2],
      costs)
