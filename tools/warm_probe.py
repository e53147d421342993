#!/usr/bin/env python3
"""Why the first timed steps after a device synchronisation run slow (not the
metric): config-2 steps, then a pause of each kind, then 8 steps; prints the
per-step host time and the count kernel's hipEvent time."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from neurokmer_amd import SpikingKmerCounter, synth  # noqa: E402


def main():
    bases, offs = synth.make_records(115_000_000, 7, repeats_per_mb=64, motif_len=200)
    d_b = torch.from_numpy(bases).cuda()
    d_o = torch.from_numpy(offs.view(np.int64)).cuda()
    st = torch.cuda.Stream()
    torch.cuda.set_stream(st)
    s = st.cuda_stream
    ctr = SpikingKmerCounter(31, 1.0, 0.95, 2, 1.0, 2_000_000, True)

    def step():
        ctr.reset(s, blocking=False)
        ctr.process_parallel_device(d_b.data_ptr(), d_o.data_ptr(), 7, bases.size, s)

    for _ in range(400):
        step()
    torch.cuda.synchronize()
    for pause in ("none", "sync", "sync+sleep1ms", "sleep10ms", "sync", "none"):
        for _ in range(50):
            step()
        if pause == "sync":
            torch.cuda.synchronize()
        elif pause == "sync+sleep1ms":
            torch.cuda.synchronize()
            time.sleep(0.001)
        elif pause == "sleep10ms":
            time.sleep(0.01)
        marks = [time.perf_counter()]
        for _ in range(8):
            step()
            marks.append(time.perf_counter())
        k1 = ctr.count_history(8)
        print(f"{pause:14s} host " + " ".join(f"{(b - a) * 1e3:.3f}" for a, b in zip(marks, marks[1:])) +
              " | k1 " + " ".join(f"{x:.3f}" for x in k1), flush=True)


if __name__ == "__main__":
    main()
