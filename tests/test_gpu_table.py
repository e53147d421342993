"""The exact k-mer table grouped by neuron (neurokmer_amd/csrc/nk_table.hip)
against the oracle: kmer_per_neuron, distinct k-mers and get_count of every key
of the input plus absent probes, in each way the table can be built:

  * fused:      opts.exact_counts, the count's own K1a writes each record's key;
  * standalone: no exact_counts, the table on demand from the held input (its
                own K1a<KEYS> pass, the currents untouched);
  * sorted:     NK_EXACT_SORT=1, the global radix sort (the reference layout);
  * side:       NK_XHASH_MAX small, so groups leave the LDS table for the
                key-sorted side part, mixed with grouped neurons;
  * fallback:   NK_XSIDE_CAP tiny, the side list overflows into the sorted build;
and skewed inputs whose bucket regions overflow in K1a (spilled keys, side
buckets) and the k = 32 all-T key (~0, kept beside the LDS table).

Reference: src/spiking_hash.rs:157-172 (`counts`, kmer_per_neuron), :675-682
(get_count); the oracle is oracle/nk_oracle.c.  Bit-exact throughout.
"""
import contextlib
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("no GPU", allow_module_level=True)

from neurokmer_amd import SpikingKmerCounter, synth  # noqa: E402
from oracle import cbind  # noqa: E402


@contextlib.contextmanager
def env(**kv):
    old = {k: os.environ.get(k) for k in kv}
    os.environ.update({k: str(v) for k, v in kv.items()})
    try:
        yield
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def keys_of(bases, offs, k, canon):
    out = set()
    for i in range(offs.size - 1):
        rec = bases[int(offs[i]):int(offs[i + 1])].tobytes()
        out.update(int(x) for x in cbind.kmer_keys(rec, k, canon))
    return out


def check_table(g, r, keys, n_probe_keys=None, seed=0):
    np.testing.assert_array_equal(g.kmer_per_neuron(), r.kmer_per_neuron())
    assert g.distinct_kmers() == r.distinct_kmers() == len(keys)
    rng = np.random.default_rng(seed)
    probe = sorted(keys)
    if n_probe_keys is not None and len(probe) > n_probe_keys:
        probe = [probe[i] for i in rng.choice(len(probe), n_probe_keys, replace=False)]
    probe += [int(x) for x in rng.integers(0, 2**62, 2000, dtype=np.uint64)]  # mostly absent
    probe += [0, 2**64 - 1]
    cnt, pres = g.get_counts(np.array(probe, dtype=np.uint64))
    want = [r.get_count(kk) for kk in probe]
    got = [int(c) if p else None for c, p in zip(cnt, pres)]
    assert got == want


def run(bases, offs, k, pool, canon, exact=True, **envkw):
    with env(**envkw):
        g = SpikingKmerCounter(k, 1.0, 0.95, 2, 1.0, pool, canon, exact_counts=exact)
        g.process_parallel_arrays(bases, offs)
        if not exact:
            g.distinct_kmers()  # builds the table on demand under this environment
        return g


def oracle(bases, offs, k, pool, canon):
    r = cbind.OracleCounter(k, 1.0, 0.95, 2, 1.0, pool, canon)
    r.process_parallel_arrays(bases, offs)
    return r


MODES = [
    pytest.param(dict(exact=True), id="fused"),
    pytest.param(dict(exact=False), id="standalone"),
    pytest.param(dict(exact=True, NK_EXACT_SORT=1), id="sorted"),
    pytest.param(dict(exact=True, NK_XHASH_MAX=40), id="side"),
    pytest.param(dict(exact=False, NK_XHASH_MAX=40), id="side-standalone"),
    pytest.param(dict(exact=True, NK_XHASH_MAX=40, NK_XSIDE_CAP=1000), id="fallback"),
]


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("k,pool,canon", [(31, 2_000_000, True), (21, 100_003, False),
                                          (32, 40_000, False), (11, 5_000, True),
                                          # k > 32 (NK_KMER_COMPAT u64 keys): the table's
                                          # own K1g<KEYS> pass (k_part_gen_keys)
                                          (40, 50_021, True), (63, 1_000_003, False),
                                          (33, 7_001, True)])
def test_grouped_table(mode, k, pool, canon):
    bases, offs = synth.make_records(600_000, 5, repeats_per_mb=2000, motif_len=120,
                                     n_rate=0.005, mixed_case=True, seed=41 + k)
    g = run(bases, offs, k, pool, canon, **mode)
    r = oracle(bases, offs, k, pool, canon)
    check_table(g, r, keys_of(bases, offs, k, canon), n_probe_keys=20_000, seed=k)
    assert g.top_abundant_neurons(20) == r.top_abundant_neurons(20)
    np.testing.assert_array_equal(g.currents(), r.currents())


@pytest.mark.parametrize("exact,k", [(True, 31), (False, 31), (True, 45), (False, 45)])
def test_overflowed_regions_spill_to_the_side(exact, k):
    """One k-mer dominates (a long poly-A record): its bucket's K1a (k > 32:
    K1g<KEYS>) region overflows, the excess keys spill, the bucket goes
    through the side part."""
    rnd, _ = synth.make_records(300_000, 1, seed=5)
    bases = np.concatenate([np.full(400_000, ord("A"), np.uint8), rnd,
                            np.frombuffer(b"AAAAT" * 20_000, np.uint8)])
    offs = np.array([0, 400_000, 700_000, bases.size], np.uint64)
    g = run(bases, offs, k, 2_000_000, True, exact=exact)
    r = oracle(bases, offs, k, 2_000_000, True)
    check_table(g, r, keys_of(bases, offs, k, True), n_probe_keys=20_000)
    np.testing.assert_array_equal(g.currents(), r.currents())
    assert g.top_abundant_neurons(20) == r.top_abundant_neurons(20)


@pytest.mark.parametrize("mode", [dict(exact=True), dict(exact=True, NK_XHASH_MAX=8)],
                         ids=["grouped", "side"])
@pytest.mark.parametrize("run_t", [5_000, 90])
def test_all_t_key_k32(mode, run_t):
    """k = 32 non-canonical: the all-T window is the key ~0 (the LDS table's
    empty marker), counted beside the table; a long T run (one hot neuron) and
    a short one (~70 records of ~0 among its neuron's others)."""
    rnd, _ = synth.make_records(50_000, 1, seed=9)
    bases = np.concatenate([rnd[:20_000], np.full(run_t, ord("T"), np.uint8), rnd[20_000:],
                            np.full(40, ord("t"), np.uint8)])
    offs = np.array([0, 30_000, bases.size], np.uint64)
    g = run(bases, offs, 32, 3_001, False, **mode)
    r = oracle(bases, offs, 32, 3_001, False)
    keys = keys_of(bases, offs, 32, False)
    assert 2**64 - 1 in keys
    check_table(g, r, keys)


def test_repeated_calls_replace_the_table():
    """Each process call replaces `counts` (src/spiking_hash.rs:157): the second
    input's table, built fused, then on demand after a plain call."""
    a, ao = synth.make_records(200_000, 3, seed=1, repeats_per_mb=500)
    b, bo = synth.make_records(150_000, 2, seed=2)
    g = SpikingKmerCounter(25, 1.0, 0.95, 2, 1.0, 70_001, True, exact_counts=True)
    r = cbind.OracleCounter(25, 1.0, 0.95, 2, 1.0, 70_001, True)
    for bases, offs in ((a, ao), (b, bo), (a, ao)):
        g.process_parallel_arrays(bases, offs)
        r.process_parallel_arrays(bases, offs)
        check_table(g, r, keys_of(bases, offs, 25, True))
    g2 = SpikingKmerCounter(25, 1.0, 0.95, 2, 1.0, 70_001, True)
    for bases, offs in ((b, bo), (a, ao)):
        g2.process_parallel_arrays(bases, offs)
    check_table(g2, r, keys_of(a, ao, 25, True))


def test_process_sequence_on_a_grouped_table():
    """process_sequence adds to `counts` on top of the grouped table: keys new to
    the table count as distinct, existing ones add to their counts."""
    bases, offs = synth.make_records(120_000, 3, seed=12, repeats_per_mb=1000)
    g = SpikingKmerCounter(15, 1.0, 0.95, 2, 1.0, 9_973, True, exact_counts=True)
    r = cbind.OracleCounter(15, 1.0, 0.95, 2, 1.0, 9_973, True)
    g.process_parallel_arrays(bases, offs)
    r.process_parallel_arrays(bases, offs)
    keys = keys_of(bases, offs, 15, True)
    for seq in (bases[1000:1400].tobytes(), b"ACGTTGCA" * 30, bases[50_000:50_100].tobytes()):
        g.process_sequence(seq)
        r.process_sequence(seq)
        keys |= set(int(x) for x in cbind.kmer_keys(seq, 15, True))
    check_table(g, r, keys)
    np.testing.assert_array_equal(g.spike_counts(), r.spike_counts())
