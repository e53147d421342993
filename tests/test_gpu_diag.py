"""The key-gather diagnostic (nk_diag_key_gather_ms; VERDICT r4 item 4: the
cost of an exact table that recomputes keys from positions, measured): every
record the partitioned count kept has its key recomputed from its (tile,
position) and the bases; the XOR of those keys must equal the XOR of the
reference's keys of every k-mer of the input (oracle/pyref.py kmer_keys,
src/spiking_hash.rs:102-138) -- each k-mer is one kept record, once.
Cases: 61 buckets, 489 buckets with a sub-region per XCD (PartArgs::sub_shift;
NK_PART_BIG=1 keeps that pool on the one-level Part count, which pools past
4.2 M leave for the wide two-level count since round 6), non-canonical keys
with N bytes.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("no GPU", allow_module_level=True)

from neurokmer_amd import SpikingKmerCounter  # noqa: E402
from oracle import pyref  # noqa: E402

from test_gpu_parity import ragged_records  # noqa: E402


@pytest.mark.parametrize("k,pool,canon", [(31, 2_000_000, True), (21, 16_000_000, True),
                                          (25, 100_003, False)])
def test_key_gather_checksum(k, pool, canon, monkeypatch):
    if pool > 4_200_000:
        monkeypatch.setenv("NK_PART_BIG", "1")
    bases, offs = ragged_records(total=150_000, n_rate=0.003, repeats_per_mb=3000, motif_len=90,
                                 seed=k)
    g = SpikingKmerCounter(k, 1.0, 0.95, 2, 1.0, pool, canon)
    g.process_parallel_arrays(bases, offs)
    ms, cs = g.diag_key_gather(reps=1)
    want = 0
    raw = bases.tobytes()
    for a, b in zip(offs[:-1], offs[1:]):
        for key in pyref.kmer_keys(raw[int(a):int(b)], k, canon):
            want ^= key
    assert cs == want
    assert ms > 0.0
