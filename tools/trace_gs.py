#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel trace of the config-5 count: per kernel the
calls and mean duration, and k_gen_split's per-launch durations of one step.
    python3 tools/trace_gs.py <dir with run_kernel_trace.csv> [tag]"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1] + "/run_kernel_trace.csv")))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
tag = sys.argv[2] if len(sys.argv) > 2 else ""
d = defaultdict(list)
for r in rows:
    d[r["Kernel_Name"].split("(")[0]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    if sum(v) > 1.0:
        print(tag, k[:40], len(v), "mean %.3f ms" % (sum(v) / len(v)), "sum %.1f" % sum(v))
gs = d.get("void nk::k_gen_split<2, true>", [])
if gs:
    print(tag, "k_gen_split first 6:", " ".join("%.3f" % x for x in gs[:6]), "| last step's 32:",
          "%.1f ms" % sum(gs[-32:]))
