#!/usr/bin/env python3
"""Per-step kernel timeline from a rocprofv3 kernel trace (not the metric).

    python tools/trace_gaps.py gpurun_out/prof_<tag>/trace/run_kernel_trace.csv [--steps 3]

Splits the trace at each k_prep launch (one per step) and prints every
kernel's start, duration and the idle gap before it, plus the gap to the next
step (host turnaround)."""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--first", default="k_prep")
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.csv)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if a.first in r["Kernel_Name"]]
    for n, st in enumerate(idx[-a.steps - 1:-1]):
        end = idx[idx.index(st) + 1]
        t0 = int(rows[st]["Start_Timestamp"])
        prev = None
        busy = 0
        for r in rows[st:end]:
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            gap = (s - prev) / 1e3 if prev else 0.0
            busy += e - s
            print(f"{r['Kernel_Name'][:34]:34s} start {(s - t0) / 1e3:8.1f} us  dur {(e - s) / 1e3:7.1f}"
                  f"  gap {gap:6.1f}")
            prev = e
        nxt = int(rows[end]["Start_Timestamp"])
        print(f"-- step {(nxt - t0) / 1e3:.1f} us, kernels {busy / 1e3:.1f} us, "
              f"turnaround to next step {(nxt - prev) / 1e3:.1f} us")


if __name__ == "__main__":
    main()
