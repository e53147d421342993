"""Config 3's resident count (31.6 M reads x 150 bp, k=31, pool 16 M) through
each count path: the Part count (K1a into 489 buckets of 32768 neurons) and the
wide two-level count (NK_WIDE_BITS=b: K1g into coarse buckets of 2^b neurons,
then K1s into the 32768-neuron buckets).  Prints each path's accumulate time
(hipEvents, median of reps), the step with the finish, and checks the currents
and top rows equal across paths.  Usage: python tools/c3_paths.py [reads]"""
import hashlib
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from neurokmer_amd import SpikingKmerCounter, synth  # noqa: E402

n_reads = int(sys.argv[1]) if len(sys.argv) > 1 else 31_600_000
modes = sys.argv[2].split(",") if len(sys.argv) > 2 else ["part", "17", "18"]
L, k, pool = 150, 31, 16_000_000
dev = torch.device("cuda", 0)
n_b = n_reads * L
d_b = torch.zeros(n_b + 16, dtype=torch.uint8, device=dev)
synth.random_bases_torch(n_b, synth.SEED, 0, dev, out=d_b)
offs = np.arange(n_reads + 1, dtype=np.uint64) * np.uint64(L)
d_o = torch.from_numpy(offs.view(np.int64)).to(dev)
s = torch.cuda.Stream(device=dev)
ref = None
for mode in modes:
    if mode == "part":
        os.environ.pop("NK_WIDE_BITS", None)
    else:
        os.environ["NK_WIDE_BITS"] = mode
    r = SpikingKmerCounter(k, 1.0, 0.95, 2, 1.0, pool, True, device=0)
    cms, tot = [], []
    for i in range(4):
        r.reset()
        e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
        torch.cuda.synchronize()
        e0.record(s)
        r.accumulate_device(d_b.data_ptr(), d_o.data_ptr(), n_reads, n_b, s.cuda_stream)
        e1.record(s)
        r.finalize(True, s.cuda_stream)
        e2.record(s)
        torch.cuda.synchronize()
        if i:
            cms.append(e0.elapsed_time(e1))
            tot.append(e0.elapsed_time(e2))
    cur = r.currents()
    top = r.top_abundant_neurons(20)
    sha = hashlib.sha1(cur.tobytes()).hexdigest()[:16]
    same = None
    if ref is None:
        ref = (sha, top)
    else:
        same = (sha, top) == ref
    print(f"mode {mode}: count {np.median(cms):.2f} ms, step {np.median(tot):.2f} ms, "
          f"sum {int(cur.sum())} (N_k {n_reads * (L - k + 1)}), sha {sha}, same_as_first {same}",
          flush=True)
    r.close()
os.environ.pop("NK_WIDE_BITS", None)
