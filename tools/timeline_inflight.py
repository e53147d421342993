#!/usr/bin/env python3
"""The count stream of the last timed steps of a bench.py kernel trace: per
step the gap before prep, prep, K1a, K1b and the finish kernels that ran
between two K1a launches (their time overlapping K1a or not).
    python3 tools/timeline_inflight.py <dir with run_kernel_trace.csv> [steps] [skip]
(skip: leave out the last `skip` K1a launches -- the bench's later phases,
one in flight and state written, follow the timed region in one trace)"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1] + "/run_kernel_trace.csv")))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 20
ev = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0].replace("void ", ""))
             for r in rows), key=lambda e: e[0])
k1a = [i for i, e in enumerate(ev) if e[2].startswith("nk::k_part<")]
skip = int(sys.argv[3]) if len(sys.argv) > 3 else 0
sel = k1a[:len(k1a) - skip][-(n + 1):]
print("step  K1a_us  K1a->K1a_us  kernels between (name: us, overlap with K1a us)")
tot = []
for a, b in zip(sel, sel[1:]):
    s0, e0 = ev[a][0], ev[a][1]
    s1 = ev[b][0]
    parts = []
    for i in range(a + 1, b):
        s, e, nm = ev[i]
        ov = max(0, min(e, e0) - max(s, s0))
        parts.append("%s %.1f/%.1f" % (nm.split("::")[-1][:14], (e - s) / 1e3, ov / 1e3))
    tot.append((s1 - s0) / 1e3)
    print("%6.1f %8.1f | %s" % ((e0 - s0) / 1e3, (s1 - s0) / 1e3, "; ".join(parts)))
print("mean K1a->K1a %.1f us over %d steps" % (sum(tot) / len(tot), len(tot)))
