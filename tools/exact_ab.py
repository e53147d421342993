"""A/B timing of the exact_counts step (config 2 input, the bench's exact step)
for the in-tree library or NK_AB_LIB: prints median ms, distinct k-mers and a
checksum of kmer_per_neuron, so variants can be compared for equal results."""
import statistics
import sys
import time
import zlib

import numpy as np
import torch

sys.path.insert(0, __import__("os").path.join(__import__("os").path.dirname(__import__("os").path.abspath(__file__)), ".."))
from neurokmer_amd import SpikingKmerCounter as Counter, synth  # noqa: E402

tag = sys.argv[1] if len(sys.argv) > 1 else "A"
bases, offs = synth.make_records(115_000_000, 7, seed=synth.SEED, repeats_per_mb=64, motif_len=200)
d_b = torch.from_numpy(np.concatenate([bases, np.zeros(16, np.uint8)])).cuda()
d_o = torch.from_numpy(offs.view(np.int64)).cuda()
torch.cuda.synchronize()
x = Counter(31, 1.0, 0.95, 2, 1.0, 2_000_000, True, exact_counts=True)


def step():
    x.reset()
    x.process_parallel_device(d_b.data_ptr(), d_o.data_ptr(), offs.size - 1, bases.size)


step()
ts = []
for _ in range(7):
    torch.cuda.synchronize()
    t = time.perf_counter()
    step()
    torch.cuda.synchronize()
    ts.append(time.perf_counter() - t)
kpn = x.kmer_per_neuron()
print(tag, "exact_ms_median", round(statistics.median(ts) * 1e3, 3), "best", round(min(ts) * 1e3, 3),
      "distinct", x.distinct_kmers(), "kpn_crc", zlib.crc32(kpn.tobytes()), flush=True)
