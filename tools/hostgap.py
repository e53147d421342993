#!/usr/bin/env python3
"""Host overhead per step of the config-2 bench loop (not the metric).

    python tools/hostgap.py [--steps 50]

Times the same process_parallel_device step three ways: as bench.py runs it
(reset + process + last_timings), without the timings read, and as one raw
ctypes call; prints the medians so the per-step host cost can be attributed.
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from neurokmer_amd import SpikingKmerCounter, synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=50)
    a = ap.parse_args()
    bases, offs = synth.make_records(115_000_000, 7, repeats_per_mb=64, motif_len=200)
    d_b = torch.from_numpy(bases).cuda()
    d_o = torch.from_numpy(offs.view(np.int64)).cuda()
    torch.cuda.synchronize()
    ctr = SpikingKmerCounter(31, 1.0, 0.95, 2, 1.0, 2_000_000, True)
    s = torch.cuda.current_stream().cuda_stream
    L, h = ctr._L, ctr._h
    bp, op = d_b.data_ptr(), d_o.data_ptr()

    def bench_step():
        ctr.reset(s, blocking=False)
        ctr.process_parallel_device(bp, op, 7, bases.size, s)
        ctr.last_timings()

    def no_timings():
        ctr.reset(s, blocking=False)
        ctr.process_parallel_device(bp, op, 7, bases.size, s)

    sp = C.c_void_p(s)

    def raw():
        L.nk_reset_async(h, sp)
        L.nk_process_parallel_device(h, bp, op, 7, bases.size, sp)

    out = {}
    for name, f in (("bench_step", bench_step), ("no_timings", no_timings), ("raw_ctypes", raw)):
        for _ in range(5):
            f()
        ts = []
        for _ in range(a.steps):
            t0 = time.perf_counter()
            f()
            ts.append(time.perf_counter() - t0)
        tl = ctr.last_timings()
        out[name] = {"median_ms": round(float(np.median(ts)) * 1e3, 4),
                     "min_ms": round(min(ts) * 1e3, 4), "gpu_total_ms": round(tl.get("total", 0), 4)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
