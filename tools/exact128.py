"""The exact k-mer table with 128-bit keys (k = 63, config 5's key mode and pool)
at growing input sizes: the step with the table (`exact_counts=True`: the
sorted build, nk_exact.hip) against the same step without it, so the table's
own cost per k-mer can be projected to config 5's per-GPU share (VERDICT r5,
"missing" item 1).  Usage: python tools/exact128.py [bases ...]"""
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from neurokmer_amd import SpikingKmerCounter as Counter, synth  # noqa: E402

K, POOL, RECS = 63, 256_000_000, 7
sizes = [int(float(a)) for a in sys.argv[1:]] or [115_000_000, 1_000_000_000]
for n in sizes:
    d_b, offs = synth.make_records_torch(n, RECS, seed=synth.SEED, repeats_per_mb=64, motif_len=200)
    d_o = torch.from_numpy(offs.view("int64")).cuda()
    torch.cuda.synchronize()
    nk = n - RECS * (K - 1)
    res = {}
    for exact in (False, True):
        c = Counter(K, 1.0, 0.95, 2, 1.0, POOL, True, kmer_width=128, exact_counts=exact)

        def step():
            c.reset()
            c.process_parallel_device(d_b.data_ptr(), d_o.data_ptr(), RECS, n)

        step()
        ts = []
        for _ in range(3):
            torch.cuda.synchronize()
            t = time.perf_counter()
            step()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t)
        res[exact] = statistics.median(ts) * 1e3
        if exact:
            res["distinct"] = c.distinct_kmers()
            res["top_same"] = None
        c.close()
        print(f"bases {n:,} exact {exact}: {res[exact]:.2f} ms", flush=True)
    tab = res[True] - res[False]
    print(f"bases {n:,} k-mers {nk:,}: step {res[False]:.2f} ms, with the table {res[True]:.2f} ms, "
          f"table {tab:.2f} ms = {nk / tab / 1e6:.2f} G k-mers/s ({tab * 1e6 / nk:.3f} ns per k-mer), "
          f"distinct {res['distinct']:,}", flush=True)
    del d_b, d_o
    torch.cuda.empty_cache()
