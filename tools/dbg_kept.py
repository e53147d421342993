import os, sys
sys.path.insert(0, os.getcwd())
import numpy as np, torch
from neurokmer_amd import SpikingKmerCounter, synth
from oracle import cbind
k, pool, canon, width = 33, 30_000_001, False, 64
bases, offs = synth.make_records(1_500_000, 5, seed=170 + k, repeats_per_mb=3000, motif_len=120, n_rate=0.002, mixed_case=True)
r = cbind.OracleCounter(k, 1.0, 0.95, 2, 1.0, pool, canon, width=width)
r.process_parallel_arrays(bases, offs, 8)
want = r.top_abundant_neurons(20)
for env in [{}, {"NK_UNIQ_TILE_LIST": "2"}, {"NK_NO_GEN_KEEP": "1"}, {"NK_NO_WRITE_THROUGH": "1"}, {"NK_NO_GEN_KEEP": "1", "NK_NO_WRITE_THROUGH": "1"}]:
    for kk in ("NK_UNIQ_TILE_LIST", "NK_NO_GEN_KEEP", "NK_NO_WRITE_THROUGH"):
        os.environ.pop(kk, None)
    os.environ.update(env)
    g = SpikingKmerCounter(k, 1.0, 0.95, 2, 1.0, pool, canon, kmer_width=width)
    g.process_parallel_arrays(bases, offs)
    got = g.top_abundant_neurons(20)
    diff = [(i, a, b) for i, (a, b) in enumerate(zip(got, want)) if a != b]
    print(env, "OK" if not diff else diff, flush=True)
    g.close()
