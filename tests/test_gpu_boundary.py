"""The drop-in boundary without preconditions the reference does not have
(VERDICT r1 "What's weak" 10): top_abundant_neurons(n) for any n, get_count /
kmer_per_neuron / process_sequence without opts.exact_counts (the table of the
last input built on demand), and the exact table for 128-bit keys.

Reference: src/spiking_hash.rs:157-172 (counts, kmer_per_neuron), :203-273
(process_sequence), :661-673 (top_abundant_neurons, any n), :675-682
(get_count).  Every comparison is bit-exact against oracle/nk_oracle.c.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("no GPU", allow_module_level=True)

from neurokmer_amd import SpikingKmerCounter, synth  # noqa: E402
from oracle import cbind  # noqa: E402

from test_gpu_parity import _keys_of, assert_exact_same, assert_same, ragged_records  # noqa: E402


def _pair(k, pool, canon, width=64, exact=False, top_n=20):
    g = SpikingKmerCounter(k, 1.0, 0.95, 2, 1.0, pool, canon, top_n=top_n, kmer_width=width,
                           exact_counts=exact)
    r = cbind.OracleCounter(k, 1.0, 0.95, 2, 1.0, pool, canon, width=width)
    return g, r


@pytest.mark.parametrize("k,pool,canon,width", [(31, 2_000_000, True, 64), (21, 100_000, True, 64),
                                                (15, 5_003, False, 64), (40, 50_021, True, 64),
                                                (63, 1_000_003, True, 128), (25, 7_001, False, 128)])
def test_top_rows_any_n(k, pool, canon, width):
    """Rows past top_n: the whole pool ranked on the device (ties by index) and
    the uniques of every row from the table of the last input."""
    bases, offs = synth.make_records(400_000, 9, repeats_per_mb=5_000, motif_len=90, seed=k,
                                     n_rate=0.002, mixed_case=True)
    g, r = _pair(k, pool, canon, width)
    g.process_parallel_arrays(bases, offs)
    r.process_parallel_arrays(bases, offs)
    assert_same(g, r)
    for n in (21, 64, 1000, 4097, pool, pool + 5):
        assert g.top_abundant_neurons(n) == r.top_abundant_neurons(n), n
    assert g.top_abundant_neurons(7) == r.top_abundant_neurons(7)  # the call's own rows


def test_top_rows_any_n_streaming_file(tmp_path):
    """process_file_streaming (held input: the device-parsed file), rows past top_n."""
    reads, roffs = synth.make_reads(3000, 150, seed=21)
    path = str(tmp_path / "r.fq")
    synth.write_fastq(path, reads, roffs)
    g, r = _pair(31, 16_000_000, True)
    g.process_file_streaming(path)
    from neurokmer_amd.fastx import stream_sequences
    r.process_streaming(list(stream_sequences(path)))
    assert_same(g, r)
    for n in (20, 500, 10_000):
        assert g.top_abundant_neurons(n) == r.top_abundant_neurons(n), n


@pytest.mark.parametrize("k,canon", [(21, True), (31, False), (33, True), (5, True)])
def test_table_on_demand(k, canon):
    """get_count / distinct / kmer_per_neuron without exact_counts: built from the
    held input when first asked, equal to the eager table."""
    bases, offs = ragged_records(total=80_000, n_rate=0.01, mixed_case=True, seed=500 + k,
                                 repeats_per_mb=20_000, motif_len=70)
    g, r = _pair(k, 4099, canon)
    g.process_parallel_arrays(bases, offs)
    r.process_parallel_arrays(bases, offs)
    assert_same(g, r)
    assert_exact_same(g, r, _keys_of(bases, offs, k, canon), 4099)
    # a second call replaces counts (src/spiking_hash.rs:157): the table follows
    b2, o2 = ragged_records(total=30_000, seed=600 + k)
    g.process_parallel_arrays(b2, o2)
    r.process_parallel_arrays(b2, o2)
    assert_exact_same(g, r, _keys_of(b2, o2, k, canon), 4099)


@pytest.mark.parametrize("canon", [True, False])
def test_process_sequence_without_exact_counts(canon):
    """process_parallel then process_sequence reads with the default options:
    the previous call's table is built first, then counts and kmer_per_neuron
    accumulate as in the reference."""
    k, pool = 17, 997
    bases, offs = synth.make_records(60_000, 4, repeats_per_mb=30_000, motif_len=50, seed=18,
                                     n_rate=0.003)
    reads, roffs = synth.make_reads(60, 90, seed=19)
    rl = synth.records_list(reads, roffs)
    g, r = _pair(k, pool, canon)
    g.process_parallel_arrays(bases, offs)
    r.process_parallel_arrays(bases, offs)
    keys = _keys_of(bases, offs, k, canon)
    for rd in rl:
        g.process_sequence(rd)
        r.process_sequence(rd)
        keys.update(int(x) for x in cbind.kmer_keys(rd, k, canon))
    assert_same(g, r)
    assert_exact_same(g, r, keys, pool)
    assert g.top_abundant_neurons(300) == r.top_abundant_neurons(300)


@pytest.mark.parametrize("k,canon,exact", [(63, True, True), (40, False, True), (21, True, False),
                                           (64, True, False)])
def test_exact_table_128(k, canon, exact):
    """kmer_width=128: the exact table (eager or on demand): distinct keys,
    kmer_per_neuron, get_count of u128 keys, uniques of rows past top_n."""
    bases, offs = ragged_records(total=70_000, n_rate=0.01, mixed_case=True, seed=700 + k,
                                 repeats_per_mb=20_000, motif_len=90)
    pool = 20_011
    g, r = _pair(k, pool, canon, width=128, exact=exact)
    g.process_parallel_arrays(bases, offs)
    r.process_parallel_arrays(bases, offs)
    assert_same(g, r)
    np.testing.assert_array_equal(g.kmer_per_neuron(), r.kmer_per_neuron())
    assert g.distinct_kmers() == r.distinct_kmers()
    keys = set()
    for i in range(offs.size - 1):
        keys.update(cbind.kmer_keys128(bases[int(offs[i]):int(offs[i + 1])].tobytes(), k, canon))
    probe = sorted(keys)[:3000]
    rng = np.random.default_rng(k)
    probe += [int(a) | (int(b) << 64) for a, b in zip(rng.integers(0, 2**63, 300, dtype=np.uint64),
                                                       rng.integers(0, 2**20, 300, dtype=np.uint64))]
    cnt, pres = g.get_counts128(probe)
    for kk, c, p in zip(probe, cnt, pres):
        assert (int(c) if p else None) == r.get_count(kk), hex(kk)
    assert g.top_abundant_neurons(2000) == r.top_abundant_neurons(2000)


@pytest.mark.parametrize("k,pool,canon,width,exact", [
    (31, 2_000_000, True, 64, False),   # Part path, uniques from the kept records
    (31, 2_000_000, True, 64, True),    # uniques from the exact table's kmer_per_neuron
    (21, 100_003, False, 64, False),
    (40, 50_021, True, 64, False),      # Gen path (compat k > 32)
    (63, 1_000_003, True, 128, False),  # 128-bit keys
    (31, 20_000_003, True, 64, False),  # Wide path, top-N past the fused selection
])
def test_simulate_spikes_auto(k, pool, canon, width, exact):
    """SpikingKmerCounter::simulate_spikes_auto (src/spiking_hash.rs:697-714,
    AVX2 branch :544-659) after process_parallel, repeated, at other step
    counts (0: no-op), then rows past top_n: bit-exact vs the oracle."""
    bases, offs = synth.make_records(300_000, 7, repeats_per_mb=6_000, motif_len=90, seed=900 + k,
                                     n_rate=0.002, mixed_case=True)
    g, r = _pair(k, pool, canon, width, exact=exact)
    g.process_parallel_arrays(bases, offs)
    r.process_parallel_arrays(bases, offs)
    for steps in (1000, 1000, 0, 333):
        g.set_steps(steps)
        r.set_steps(steps)
        g.simulate_spikes_auto()
        r.simulate_spikes_auto()
        assert_same(g, r)
    assert g.top_abundant_neurons(500) == r.top_abundant_neurons(500)


def test_simulate_spikes_auto_edges(tmp_path):
    """simulate on a fresh counter (all currents zero; threshold 0 makes zero-
    current neurons spike under the streaming rule), after process_sequence
    (currents zeroed, :271), after process_file_streaming, and on device input."""
    g = SpikingKmerCounter(21, 0.0, 0.9, 1, 2.5, 3_001, True)
    r = cbind.OracleCounter(21, 0.0, 0.9, 1, 2.5, 3_001, True)
    g.simulate_spikes_auto()
    r.simulate_spikes_auto()
    assert r.total_spikes > 0
    assert_same(g, r)
    reads, roffs = synth.make_reads(40, 80, seed=31)
    for rd in synth.records_list(reads, roffs)[:5]:
        g.process_sequence(rd)
        r.process_sequence(rd)
    g.simulate_spikes_auto()
    r.simulate_spikes_auto()
    assert_same(g, r)
    # file -> streaming rule, then simulate on the held currents
    reads, roffs = synth.make_reads(3000, 150, seed=32)
    path = str(tmp_path / "s.fq")
    synth.write_fastq(path, reads, roffs)
    g2, r2 = _pair(31, 16_000_000, True)
    g2.process_file_streaming(path)
    from neurokmer_amd.fastx import stream_sequences
    r2.process_streaming(list(stream_sequences(path)))
    g2.simulate_spikes_auto()
    r2.simulate_spikes_auto()
    assert_same(g2, r2)
    # device input (kept resident by the caller)
    bases, offs = synth.make_records(200_000, 3, seed=33, repeats_per_mb=8_000, motif_len=80)
    d_b = torch.from_numpy(np.concatenate([bases, np.zeros(16, np.uint8)])).cuda()
    d_o = torch.from_numpy(offs.view(np.int64)).cuda()
    torch.cuda.synchronize()
    g3, r3 = _pair(31, 2_000_000, True)
    g3.process_parallel_device(d_b.data_ptr(), d_o.data_ptr(), offs.size - 1, bases.size)
    r3.process_parallel_arrays(bases, offs)
    g3.simulate_spikes_auto()
    r3.simulate_spikes_auto()
    assert_same(g3, r3)


@pytest.mark.parametrize("k,pool,canon,width", [(31, 20_000_003, True, 64), (40, 16_777_217, False, 64),
                                                (63, 40_000_000, True, 128), (21, 3_001, True, 128)])
def test_kmer_per_neuron_by_partition(k, pool, canon, width):
    """kmer_per_neuron of the table: its distinct keys hashed and partitioned like
    the count (narrow buckets, or coarse buckets + k_split past 16.7 M neurons),
    against the oracle and against the per-key atomic kernel (NK_KPN_ATOMIC)."""
    bases, offs = ragged_records(total=300_000, n_rate=0.005, mixed_case=True, seed=800 + k,
                                 repeats_per_mb=20_000, motif_len=90)
    g, r = _pair(k, pool, canon, width=width, exact=True)
    g.process_parallel_arrays(bases, offs)
    r.process_parallel_arrays(bases, offs)
    kpn = g.kmer_per_neuron()
    np.testing.assert_array_equal(kpn, r.kmer_per_neuron())
    assert int(kpn.sum(dtype=np.int64)) == g.distinct_kmers() == r.distinct_kmers()
    os.environ["NK_KPN_ATOMIC"] = "1"
    try:
        a = SpikingKmerCounter(k, 1.0, 0.95, 2, 1.0, pool, canon, kmer_width=width,
                               exact_counts=True)
        a.process_parallel_arrays(bases, offs)
        np.testing.assert_array_equal(a.kmer_per_neuron(), kpn)
    finally:
        del os.environ["NK_KPN_ATOMIC"]
    # a second input on the same handle: the partition's scratch is clean again
    b2, o2 = synth.make_records(150_000, 5, seed=k)
    g.process_parallel_arrays(b2, o2)
    r.process_parallel_arrays(b2, o2)
    np.testing.assert_array_equal(g.kmer_per_neuron(), r.kmer_per_neuron())
