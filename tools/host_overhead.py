#!/usr/bin/env python3
"""Host time of one count's enqueue (bench.py's start(): nk_reset_async +
nk_accumulate_device) and of its parts, on config 2's input resident in HBM,
with the GPU left to drain between batches of calls: the host's share of a
step when it is on the critical path (the multi-GPU finish with two batches in
flight).  Also a ctypes no-op for the binding's own cost.
    python3 tools/host_overhead.py [reps]"""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from neurokmer_amd import SpikingKmerCounter, synth  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    bases, offs = synth.make_records(115_000_000, 7, seed=synth.SEED, repeats_per_mb=64, motif_len=200)
    dev = torch.device("cuda", 0)
    d_b = torch.from_numpy(np.concatenate([bases, np.zeros(16, np.uint8)])).to(dev)
    d_o = torch.from_numpy(offs.astype(np.uint64).view(np.int64)).to(dev)
    st = torch.cuda.Stream()
    sh = st.cuda_stream
    c = SpikingKmerCounter(31, 1.0, 0.95, 2, 1.0, 2_000_000, True)
    n_recs, n_bases = offs.size - 1, bases.size
    for _ in range(5):
        c.reset(sh, blocking=False)
        c.accumulate_device(d_b.data_ptr(), d_o.data_ptr(), n_recs, n_bases, sh)
        c.finalize(False, sh)
    torch.cuda.synchronize()
    out = {}
    for name, fn in (
            ("reset_async", lambda: c.reset(sh, blocking=False)),
            ("accumulate_device", lambda: c.accumulate_device(d_b.data_ptr(), d_o.data_ptr(), n_recs, n_bases, sh)),
            ("ctypes_noop", lambda: c._L.nk_last_error()),
    ):
        ts = []
        for i in range(reps):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
            if i % 8 == 7:
                torch.cuda.synchronize()
        torch.cuda.synchronize()
        ts.sort()
        out[name] = (round(ts[len(ts) // 2] * 1e6, 1), round(ts[len(ts) // 10] * 1e6, 1))
    print({k: {"median_us": v[0], "p10_us": v[1]} for k, v in out.items()})


if __name__ == "__main__":
    main()
