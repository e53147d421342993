"""Debug aid for the exact table's wave sort (k_xgroup_ws): kmer_per_neuron of
the grouped table against the oracle, per build mode (env), on the table
tests' first input."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from neurokmer_amd import SpikingKmerCounter, synth  # noqa: E402
from oracle import cbind  # noqa: E402

k, pool, canon = 31, 2_000_000, True
bases, offs = synth.make_records(600_000, 5, repeats_per_mb=2000, motif_len=120,
                                 n_rate=0.005, mixed_case=True, seed=41 + k)
r = cbind.OracleCounter(k, 1.0, 0.95, 2, 1.0, pool, canon)
r.process_parallel_arrays(bases, offs)
want = r.kmer_per_neuron().astype(np.int64)
for envs in ({"NK_XG_HASH": "1"}, {}, {"NK_XG_WS1": "1"}, {"NK_EXACT_SORT": "1"}):
    for exact in (True, False):
        old = dict(os.environ)
        os.environ.update(envs)
        g = SpikingKmerCounter(k, 1.0, 0.95, 2, 1.0, pool, canon, exact_counts=exact)
        g.process_parallel_arrays(bases, offs)
        got = g.kmer_per_neuron().astype(np.int64)
        os.environ.clear()
        os.environ.update(old)
        d = got - want
        bad = np.nonzero(d)[0]
        print(envs, "exact" if exact else "standalone", "distinct", g.distinct_kmers(), r.distinct_kmers(),
              "bad", bad.size, "plus", int((d > 0).sum()), "minus", int((d < 0).sum()), flush=True)
        if bad.size:
            print("  first", bad[:8].tolist(), "got", got[bad[:8]].tolist(), "want", want[bad[:8]].tolist())
            print("  bad neurons mod 128 hist", np.bincount(bad % 128, minlength=128)[:32].tolist())
            print("  want hist of bad", np.bincount(want[bad])[:8].tolist(), "got", np.bincount(got[bad])[:8].tolist())
        g.close()
