"""Associative memory on the device (neurokmer_amd/csrc/nk_assoc.hip) vs the
CPU restatement of src/associative.rs (oracle/nk_assoc_oracle.c): Willshaw
store / recall bit-exact over pattern sizes and step counts, and
KmerAssociativeMemory's BLAKE3 patterns, store_kmer and find_similar
(results as (kmer, f32 similarity), similarity descending, ties by k-mer)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("no GPU", allow_module_level=True)

from neurokmer_amd import NeuroKmerError  # noqa: E402
from neurokmer_amd.assoc import KmerAssociativeMemory, WillshawNetwork  # noqa: E402
from oracle import cbind  # noqa: E402


@pytest.mark.parametrize("n,dens,npat", [(2, 0.5, 3), (31, 0.2, 8), (64, 0.1, 20),
                                         (100, 0.05, 30), (1000, 0.01, 200), (1024, 0.01, 500),
                                         (3000, 0.004, 60)])
def test_willshaw_store_recall(n, dens, npat):
    rng = np.random.default_rng(n * 7 + npat)
    g, o = WillshawNetwork(n), cbind.OracleWillshaw(n)
    pats = []
    for _ in range(npat):
        p = ((rng.random(n) < dens) * rng.integers(1, 256, n)).astype(np.uint8).tobytes()
        pats.append(p)
        g.store(p)
        o.store(p)
    assert g.stored_count == o.stored_count == npat
    for steps in (0, 1, 2, 10):
        for q in pats[:4] + [((rng.random(n) < 2 * dens) * 255).astype(np.uint8).tobytes()]:
            # a stored pattern with bits dropped / added (the noisy cue)
            qq = bytearray(q)
            for i in rng.integers(0, n, max(1, n // 50)):
                qq[int(i)] = 0 if qq[int(i)] else 7
            for cue in (q, bytes(qq)):
                assert g.recall(cue, steps) == o.recall(cue, steps)
    with pytest.raises(NeuroKmerError):
        g.store(b"\x00" * (n + 1))
    with pytest.raises(NeuroKmerError):
        g.recall(b"\x00" * (n + 1), 3)


@pytest.mark.parametrize("k,nstore", [(3, 40), (7, 300), (10, 2000), (12, 3000), (31, 600)])
def test_kmer_associative_memory(k, nstore):
    rng = np.random.default_rng(k)
    g, o = KmerAssociativeMemory(k), cbind.OracleAssoc(k)
    assert g.pattern_size == o.pattern_size
    kmers = rng.integers(0, 2**63, nstore, dtype=np.uint64)
    kmers[::17] = kmers[0]  # duplicates: one entry per distinct k-mer
    counts = rng.integers(1, 100, nstore).astype(np.uint32)
    half = nstore // 2
    g.store_kmers(kmers[:half], counts[:half])  # a batch
    for x, c in zip(kmers[half:], counts[half:]):  # one at a time
        g.store_kmer(int(x), int(c))
    for x, c in zip(kmers, counts):
        o.store_kmer(int(x), int(c))
    queries = [int(x) for x in kmers[:6]] + [int(x) for x in rng.integers(0, 2**63, 4, dtype=np.uint64)]
    for q in queries:
        for md in (0, 3, 12, 40, g.pattern_size):
            got, want = g.find_similar(q, md), o.find_similar(q, md)
            assert got == want, (q, md)
