"""GPU parity: the HIP path (through the C ABI) vs the CPU restatement.

Every comparison is bit-exact: u64 currents, u64 spike counts, f32 voltages
(bitwise), u32 refractory ticks, total spikes, energy, top-N rows including
"unique k-mers colliding".  Inputs are seeded synthetic records with N runs,
lowercase bases, other IUPAC bytes, empty records and records shorter than k.
"""
import contextlib
import json
import os
import subprocess

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")  # import first: one shared HIP runtime
if not torch.cuda.is_available():
    pytest.skip("no GPU", allow_module_level=True)

from neurokmer_amd import SpikingKmerCounter, synth  # noqa: E402
from neurokmer_amd import _lib  # noqa: E402
from oracle import cbind, pyref  # noqa: E402

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def ragged_records(total=60_000, seed=7, max_len=4000, **kw):
    bases, _ = synth.make_records(total, 1, seed=seed, **kw)
    rng = np.random.default_rng(seed)
    lens = []
    s = 0
    while s < total:
        L = int(rng.integers(0, max_len))
        if rng.random() < 0.1:
            L = int(rng.integers(0, 40))  # short (often < k) and empty records
        L = min(L, total - s)
        lens.append(L)
        s += L
    offs = np.zeros(len(lens) + 1, np.uint64)
    np.cumsum(lens, out=offs[1:])
    return bases, offs


def assert_same(gpu, ref, n=20):
    np.testing.assert_array_equal(gpu.currents(), ref.currents())
    np.testing.assert_array_equal(gpu.spike_counts(), ref.spike_counts())
    np.testing.assert_array_equal(gpu.voltages().view(np.uint32), ref.voltages().view(np.uint32))
    np.testing.assert_array_equal(gpu.refractory(), ref.refractory())
    assert gpu.energy.total_spikes() == ref.total_spikes
    assert gpu.energy_used() == ref.energy_used()
    assert gpu.top_abundant_neurons(n) == ref.top_abundant_neurons(n)


def run_both(bases, offs, k, pool, canon, thr=1.0, leak=0.95, refr=2, cost=1.0, steps=None,
             top_n=20, streaming=False, width=64):
    g = SpikingKmerCounter(k, thr, leak, refr, cost, pool, canon, top_n=top_n, kmer_width=width)
    r = cbind.OracleCounter(k, thr, leak, refr, cost, pool, canon, width=width)
    if steps is not None:
        g.set_steps(steps)
        r.set_steps(steps)
    if streaming:
        # the streaming LIF rule on in-memory records goes through the split API
        d_b = torch.from_numpy(np.concatenate([bases, np.zeros(16, np.uint8)])).cuda()
        d_o = torch.from_numpy(offs.view(np.int64)).cuda()
        torch.cuda.synchronize()
        g.accumulate_device(d_b.data_ptr(), d_o.data_ptr(), offs.size - 1, int(offs[-1]))
        g.finalize(streaming=True)
        r.process_streaming_arrays(bases, offs)
    else:
        g.process_parallel_arrays(bases, offs)
        r.process_parallel_arrays(bases, offs)
    return g, r


KS = (1, 2, 3, 5, 11, 15, 16, 17, 21, 31, 32, 33, 40, 63)


@pytest.mark.parametrize("canon", [True, False])
@pytest.mark.parametrize("k", KS)
def test_parity_mixed_bytes(k, canon):
    bases, offs = ragged_records(n_rate=0.01, mixed_case=True, seed=11 + k)
    g, r = run_both(bases, offs, k, 5003, canon)
    assert_same(g, r)


# 8_388_609 .. 1 << 24: the 512-bucket partition (config 3's 16 M pool);
# (1 << 24) + 1: past it (direct-atomic count)
@pytest.mark.parametrize("pool", [1, 2, 7, 64, 100_003, (1 << 20) + 7, 8_388_609, 16_000_000,
                                  1 << 24, (1 << 24) + 1])
def test_parity_pools(pool):
    bases, offs = ragged_records(total=120_000, repeats_per_mb=3000, motif_len=150, seed=3)
    g, r = run_both(bases, offs, 31, pool, True)
    assert_same(g, r)


@pytest.mark.parametrize("canon", [True, False])
def test_parity_wide_partition(canon):
    # several tiles per bucket at 489 buckets, N bytes, ragged records
    bases, offs = ragged_records(total=2_000_000, n_rate=0.002, repeats_per_mb=4000,
                                 motif_len=120, seed=23)
    g, r = run_both(bases, offs, 27, 16_000_000, canon)
    assert_same(g, r)


def test_parity_planted_repeats_ties():
    # hot neurons saturate (334 spikes) -> many ties in the top-N, broken by index
    bases, offs = synth.make_records(400_000, 7, repeats_per_mb=20_000, motif_len=60, seed=5)
    g, r = run_both(bases, offs, 21, 20_000, True, top_n=200)
    assert_same(g, r, n=200)


@pytest.mark.parametrize("canon,pool", [(True, (1 << 20) + 7), (False, (1 << 20) + 7),
                                        (True, 16_000_000)])
def test_parity_skewed_overflow(canon, pool):
    """Poly-A-heavy input: one bucket gets far more than its region (the excess
    is counted with direct atomics and the uniques fall back to a rescan), and
    the top rows need a bigger uniques hash set than the default.  At 16 M the
    bucket regions hold a sub-region per XCD (PartArgs::sub_shift): one of
    them overflows while its siblings do not."""
    bases, offs = synth.make_records(3_000_000, 6, seed=61, repeats_per_mb=2000, motif_len=40)
    bases[200_000:2_600_000] = ord("A")
    bases[1_000_000:1_000_050] = ord("N")
    g, r = run_both(bases, offs, 21, pool, canon)
    assert_same(g, r)


@pytest.mark.parametrize("steps", [0, 1, 7, 999, 5000, 20000])
def test_parity_steps(steps):
    # steps=20000 pushes spike counts past the 4095-bin histogram: exact radix refine
    bases, offs = synth.make_records(200_000, 3, repeats_per_mb=5000, motif_len=80, seed=9)
    g, r = run_both(bases, offs, 25, 3001, True, steps=steps)
    assert_same(g, r)


@pytest.mark.parametrize("thr,leak,refr,cost", [(0.5, 1.0, 0, 2.5), (0.0, 0.95, 2, 1.0),
                                                  (1.0, 0.0, 5, 0.001), (3.0, 0.99, 1, 1.0),
                                                  (1.0, 0.95, 1000, 1.0)])
def test_parity_lif_params(thr, leak, refr, cost):
    bases, offs = synth.make_records(150_000, 4, repeats_per_mb=4000, motif_len=90, seed=13)
    g, r = run_both(bases, offs, 19, 1999, True, thr=thr, leak=leak, refr=refr, cost=cost)
    assert_same(g, r)


@pytest.mark.parametrize("canon", [True, False])
def test_streaming_lif_rule(canon):
    bases, offs = ragged_records(total=80_000, n_rate=0.002, seed=21)
    g, r = run_both(bases, offs, 23, 40_000, canon, streaming=True, thr=0.0)
    assert_same(g, r)


def test_state_persists_across_calls():
    b1, o1 = synth.make_records(100_000, 3, repeats_per_mb=6000, motif_len=70, seed=1)
    b2, o2 = synth.make_records(90_000, 5, repeats_per_mb=9000, motif_len=50, seed=2)
    g = SpikingKmerCounter(17, 1.0, 0.95, 2, 1.0, 777, True)
    r = cbind.OracleCounter(17, 1.0, 0.95, 2, 1.0, 777, True)
    for b, o in ((b1, o1), (b2, o2), (b1, o1)):
        g.process_parallel_arrays(b, o)
        r.process_parallel_arrays(b, o)
        assert_same(g, r)
    g.reset()
    assert g.energy.total_spikes() == 0
    assert g.top_abundant_neurons(5) == [(i, 0, 0) for i in range(5)]


def test_reset_is_lazy_and_exact():
    """nk_reset only marks the state fresh; the next call must equal a fresh
    counter, and the copy-outs right after a reset must read zeros."""
    b1, o1 = synth.make_records(120_000, 3, repeats_per_mb=6000, motif_len=70, seed=4)
    b2, o2 = synth.make_records(110_000, 4, repeats_per_mb=9000, motif_len=50, seed=5)
    g = SpikingKmerCounter(21, 1.0, 0.95, 2, 1.0, 5003, True)
    g.process_parallel_arrays(b1, o1)
    g.reset()
    for arr in (g.currents(), g.spike_counts(), g.refractory()):
        assert not arr.any()
    assert not g.voltages().view(np.uint32).any()
    g.process_parallel_arrays(b1, o1)
    g.reset()  # no copy-out in between: the LIF must not read the stale state
    g.process_parallel_arrays(b2, o2)
    r = cbind.OracleCounter(21, 1.0, 0.95, 2, 1.0, 5003, True)
    r.process_parallel_arrays(b2, o2)
    assert_same(g, r)


@pytest.mark.parametrize("top_n", [1, 2, 63, 64, 65, 333])
def test_top_n_selection_paths(top_n):
    # <= 64 rows: selection fused into the LIF kernel; more: separate kernels.
    # Saturated repeats make long runs of ties broken by index.
    bases, offs = synth.make_records(300_000, 5, repeats_per_mb=20_000, motif_len=60, seed=17)
    g, r = run_both(bases, offs, 21, 70_001, True, top_n=top_n)
    assert_same(g, r, n=top_n)


def test_python_restatement_agrees():
    # tiny case through the pure-Python restatement as a second, independent oracle
    bases, offs = ragged_records(total=6000, n_rate=0.01, mixed_case=True, seed=99, max_len=900)
    seqs = synth.records_list(bases, offs)
    for k, canon in ((21, False), (31, True), (33, True)):
        g = SpikingKmerCounter(k, 1.0, 0.95, 2, 1.0, 211, canon)
        g.process_parallel(seqs)
        p = pyref.SpikingKmerCounter(k, 1.0, 0.95, 2, 1.0, 211, canon)
        p.process_parallel(seqs)
        assert list(g.currents()) == p.currents
        assert list(g.spike_counts()) == p.sc
        assert g.top_abundant_neurons(20) == p.top_abundant_neurons(20)


def test_device_entry_point_and_alignment():
    bases, offs = synth.make_records(300_000, 7, repeats_per_mb=500, seed=17)
    d_b = torch.from_numpy(bases).cuda()
    d_o = torch.from_numpy(offs.view(np.int64)).cuda()
    torch.cuda.synchronize()
    g = SpikingKmerCounter(31, 1.0, 0.95, 2, 1.0, 50_000, True)
    g.process_parallel_device(d_b.data_ptr(), d_o.data_ptr(), 7, bases.size)
    r = cbind.OracleCounter(31, 1.0, 0.95, 2, 1.0, 50_000, True)
    r.process_parallel_arrays(bases, offs)
    assert_same(g, r)
    with pytest.raises(_lib.NeuroKmerError):
        g.process_parallel_device(d_b.data_ptr() + 1, d_o.data_ptr(), 7, bases.size - 1)


def test_split_phase_two_shards_equals_whole():
    """Multi-GPU protocol on one device: two shards accumulated separately,
    currents summed (what RCCL all-reduce does), finalized on one counter,
    then the shards' top k-mer keys merged -> identical to the whole input."""
    bases, offs = synth.make_records(240_000, 8, repeats_per_mb=8000, motif_len=64, seed=23)
    cut = 4  # shard = whole records
    sh = []
    for lo, hi in ((0, cut), (cut, 8)):
        b = bases[int(offs[lo]):int(offs[hi])]
        o = (offs[lo:hi + 1] - offs[lo]).astype(np.uint64)
        sh.append((torch.from_numpy(np.concatenate([b, np.zeros(16, np.uint8)])).cuda(),
                   torch.from_numpy(o.view(np.int64)).cuda(), hi - lo, b.size))
    torch.cuda.synchronize()
    a = SpikingKmerCounter(21, 1.0, 0.95, 2, 1.0, 9001, True)
    b_ = SpikingKmerCounter(21, 1.0, 0.95, 2, 1.0, 9001, True)
    a.accumulate_device(sh[0][0].data_ptr(), sh[0][1].data_ptr(), sh[0][2], sh[0][3])
    b_.accumulate_device(sh[1][0].data_ptr(), sh[1][1].data_ptr(), sh[1][2], sh[1][3])
    tot = a.currents() + b_.currents()
    t = torch.from_numpy(tot.view(np.int64)).cuda()
    for c in (a, b_):  # what the RCCL all-reduce leaves on every rank
        cur = torch.as_tensor(_CAI(c.device_currents_ptr(), tot.size), device="cuda")
        cur.copy_(t)
        torch.cuda.synchronize()
        c.finalize(False)
    keys = []
    for c in (a, b_):
        p, n = c.top_kmers_device()
        keys.append(torch.as_tensor(_CAI(p, n), device="cuda").clone() if n
                    else torch.zeros(0, dtype=torch.int64, device="cuda"))
    allk = torch.cat(keys)
    a.merge_top_kmers(allk.data_ptr(), allk.numel())
    r = cbind.OracleCounter(21, 1.0, 0.95, 2, 1.0, 9001, True)
    r.process_parallel_arrays(bases, offs)
    assert_same(a, r)


@pytest.mark.parametrize("world", [2, 3])
def test_exact_table_across_shards(world):
    """Multi-GPU exact table on one device: `world` counters (ranks) with the
    table on, currents summed, tables exchanged by owner (what the all-to-all
    does), kmer_per_neuron summed (all-reduce) -> counts, distinct k-mers,
    kmer_per_neuron and the top rows' uniques of the whole input."""
    from neurokmer_amd import dist as nkdist
    k, pool = 23, 6007
    bases, offs = synth.make_records(300_000, 6, seed=31, repeats_per_mb=20000, motif_len=70,
                                     n_rate=0.002)
    ranks, keep = [], []
    for lo, hi, so, _ in nkdist.shard_records(offs, world, k):
        b = bases[lo:hi]
        d_b = torch.from_numpy(np.concatenate([b, np.zeros(16, np.uint8)])).cuda()
        d_o = torch.from_numpy(so.astype(np.uint64).view(np.int64)).cuda()
        c = SpikingKmerCounter(k, 1.0, 0.95, 2, 1.0, pool, True, exact_counts=True)
        torch.cuda.synchronize()
        c.accumulate_device(d_b.data_ptr(), d_o.data_ptr(), so.size - 1, b.size)
        ranks.append(c)
        keep += [d_b, d_o]
    tot = sum(c.currents() for c in ranks)
    t = torch.from_numpy(tot.view(np.int64)).cuda()
    for c in ranks:
        torch.as_tensor(_CAI(c.device_currents_ptr(), pool), device="cuda").copy_(t)
    parts = []
    for c in ranks:  # nk_exact_partition on every rank
        cnt, kp, cp = c.exact_partition(world)
        n = sum(cnt)
        kk = torch.as_tensor(_CAI(kp, n), device="cuda").clone() if n else \
            torch.zeros(0, dtype=torch.int64, device="cuda")
        cc = torch.as_tensor(_CAI(cp, n, "<i4"), device="cuda").clone() if n else \
            torch.zeros(0, dtype=torch.int32, device="cuda")
        parts.append((np.concatenate([[0], np.cumsum(cnt)]), kk, cc))
    for r, c in enumerate(ranks):  # all-to-all: rank r takes every source's slice r
        rk = torch.cat([kk[int(o[r]):int(o[r + 1])] for o, kk, _ in parts])
        rc = torch.cat([cc[int(o[r]):int(o[r + 1])] for o, _, cc in parts])
        torch.cuda.synchronize()
        c.exact_adopt(rk.data_ptr(), rc.data_ptr(), rk.numel())
    kpn = sum(c.kmer_per_neuron().astype(np.int64) for c in ranks)
    kt = torch.from_numpy(kpn.astype(np.int32)).cuda()
    for c in ranks:  # all-reduce of kmer_per_neuron
        torch.as_tensor(_CAI(c.device_kmer_per_neuron_ptr(), pool, "<i4"), device="cuda").copy_(kt)
        torch.cuda.synchronize()
        c.finalize(False)
    r = cbind.OracleCounter(k, 1.0, 0.95, 2, 1.0, pool, True)
    r.process_parallel_arrays(bases, offs)
    assert_same(ranks[0], r)
    np.testing.assert_array_equal(kpn, r.kmer_per_neuron())
    assert sum(c.distinct_kmers() for c in ranks) == r.distinct_kmers()
    keys = np.unique(np.concatenate([cbind.kmer_keys(bases[int(offs[i]):int(offs[i + 1])].tobytes(),
                                                     k, True) for i in range(3)]))[:3000]
    keys = np.concatenate([keys, np.array([12345, 2**40 + 7], np.uint64)])  # absent keys too
    own = nkdist.exact_owner(keys, world)
    got_c = np.zeros(keys.size, np.uint32)
    got_p = np.zeros(keys.size, bool)
    for rr, c in enumerate(ranks):
        m = own == rr
        got_c[m], got_p[m] = c.get_counts(keys[m])
    ref = [r.get_count(int(x)) for x in keys]
    assert got_p.tolist() == [x is not None for x in ref]
    assert got_c[got_p].tolist() == [x for x in ref if x is not None]


# ---- generic / wide partition (nk_wide.hip) ---------------------------------
@contextlib.contextmanager
def wide_bits(bits):
    """Force the wide (coarse -> fine) partition with 2^bits-bin coarse buckets."""
    old = os.environ.get("NK_WIDE_BITS")
    os.environ["NK_WIDE_BITS"] = str(bits)
    try:
        yield
    finally:
        if old is None:
            os.environ.pop("NK_WIDE_BITS", None)
        else:
            os.environ["NK_WIDE_BITS"] = old


@pytest.mark.parametrize("canon", [True, False])
@pytest.mark.parametrize("k,width,bits", [(21, 64, 16), (31, 64, 18), (33, 64, 17), (63, 64, 24),
                                          (45, 128, 17), (64, 128, 19)])
def test_wide_partition_forced(k, width, bits, canon):
    # several coarse buckets, each split into 2..512 fine buckets; ragged
    # records, N bytes and mixed case (compat keys near record starts)
    bases, offs = ragged_records(total=400_000, n_rate=0.01, mixed_case=True, seed=300 + k,
                                 repeats_per_mb=5000, motif_len=90)
    with wide_bits(bits):
        g, r = run_both(bases, offs, k, 700_001, canon, width=width)
    assert_same(g, r)


@pytest.mark.parametrize("k,width", [(31, 64), (40, 64), (63, 128)])
def test_wide_partition_large_pool(k, width):
    # past the 512-bucket narrow partition: coarse buckets of 2^17 bins
    bases, offs = synth.make_records(1_500_000, 5, seed=77 + k, n_rate=0.001,
                                     repeats_per_mb=8000, motif_len=100)
    g, r = run_both(bases, offs, k, 20_000_003, True, width=width)
    assert_same(g, r)


@pytest.mark.parametrize("k", [31, 40])
def test_wide_partition_streaming_ingest(tmp_path, k):
    # per-batch histograms of the generic/wide partition over FASTQ chunks
    reads, roffs = synth.make_reads(3000, 150, seed=k, n_rate=0.005, repeats_per_mb=40_000,
                                    motif_len=50)
    p = tmp_path / "w.fq"
    synth.write_fastq(str(p), reads, roffs)
    with wide_bits(17):
        _ingest_check(str(p), k, 400_009, True, True, 50_000)
    _ingest_check(str(p), k, 400_009, False, False, 50_000)  # Gen (k=40) / Part (k=31)


# ---- --kmer-width=128 (the build's true k <= 64 mode) -------
@pytest.mark.parametrize("canon", [True, False])
@pytest.mark.parametrize("k", [1, 17, 32, 33, 47, 49, 56, 63, 64])
def test_width128_parity(k, canon):
    bases, offs = ragged_records(n_rate=0.01, mixed_case=True, seed=211 + k)
    g, r = run_both(bases, offs, k, 5003, canon, width=128)
    assert_same(g, r)


def test_width128_repeats_large_pool():
    # config 5's shape in small: k=63, a pool past the fused top-N bound, repeats
    bases, offs = synth.make_records(400_000, 5, repeats_per_mb=20_000, motif_len=120, seed=41)
    g, r = run_both(bases, offs, 63, (1 << 24) + 3, True, width=128)
    assert_same(g, r)


def test_width128_golden_e2e():
    d = json.load(open(os.path.join(GOLD, "width128.json")))["e2e"]
    g = SpikingKmerCounter(d["k"], 1.0, 0.95, 2, 1.0, d["pool"], True, kmer_width=128)
    g.process_parallel([x.encode("latin-1") for x in d["records"]])
    assert list(g.currents()) == d["currents"]
    assert list(g.spike_counts()) == d["spike_counts"]
    assert list(g.voltages().view(np.uint32)) == d["voltage_bits"]
    assert [list(t) for t in g.top_abundant_neurons(20)] == d["top20"]


def test_width128_split_phase_two_shards():
    bases, offs = synth.make_records(200_000, 6, repeats_per_mb=9000, motif_len=70, seed=29)
    sh = []
    for lo, hi in ((0, 3), (3, 6)):
        b = bases[int(offs[lo]):int(offs[hi])]
        o = (offs[lo:hi + 1] - offs[lo]).astype(np.uint64)
        sh.append((torch.from_numpy(np.concatenate([b, np.zeros(16, np.uint8)])).cuda(),
                   torch.from_numpy(o.view(np.int64)).cuda(), hi - lo, b.size))
    torch.cuda.synchronize()
    cs = [SpikingKmerCounter(45, 1.0, 0.95, 2, 1.0, 7001, True, kmer_width=128) for _ in sh]
    for c, x in zip(cs, sh):
        c.accumulate_device(x[0].data_ptr(), x[1].data_ptr(), x[2], x[3])
    tot = cs[0].currents() + cs[1].currents()
    t = torch.from_numpy(tot.view(np.int64)).cuda()
    for c in cs:
        cur = torch.as_tensor(_CAI(c.device_currents_ptr(), tot.size), device="cuda")
        cur.copy_(t)
        torch.cuda.synchronize()
        c.finalize(False)
    keys = []
    for c in cs:
        p, n = c.top_kmers_device()  # n (lo, hi) pairs
        keys.append(torch.as_tensor(_CAI(p, 2 * n), device="cuda").clone() if n
                    else torch.zeros(0, dtype=torch.int64, device="cuda"))
    allk = torch.cat(keys)
    cs[0].merge_top_kmers(allk.data_ptr(), allk.numel() // 2)
    r = cbind.OracleCounter(45, 1.0, 0.95, 2, 1.0, 7001, True, width=128)
    r.process_parallel_arrays(bases, offs)
    assert_same(cs[0], r)


class _CAI:
    def __init__(self, ptr, n, typestr="<i8"):
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": typestr, "data": (ptr, False),
                                         "version": 3}


def _fasta(tmp_path, bases, offs, name="in.fa"):
    p = tmp_path / name
    synth.write_fasta(str(p), bases, offs, width=60)
    return str(p)


def test_file_streaming_fasta(tmp_path):
    bases, offs = ragged_records(total=70_000, n_rate=0.003, mixed_case=True, seed=31)
    path = _fasta(tmp_path, bases, offs)
    g = SpikingKmerCounter(27, 1.0, 0.95, 2, 1.0, 3333, True)
    g.process_file_streaming(path)
    r = cbind.OracleCounter(27, 1.0, 0.95, 2, 1.0, 3333, True)
    r.process_streaming_arrays(bases, offs)
    assert_same(g, r)


def test_file_streaming_fastq(tmp_path):
    bases, offs = synth.make_reads(2000, 150, seed=41, repeats_per_mb=20_000, motif_len=60)
    p = tmp_path / "in.fq"
    synth.write_fastq(str(p), bases, offs)
    g = SpikingKmerCounter(31, 1.0, 0.95, 2, 1.0, 7919, True)
    g.process_file_streaming(str(p))
    r = cbind.OracleCounter(31, 1.0, 0.95, 2, 1.0, 7919, True)
    r.process_streaming_arrays(bases, offs)
    assert_same(g, r)


@pytest.mark.parametrize("canon,streaming", [(True, False), (False, False), (True, True)])
def test_cli_stdout_block(tmp_path, canon, streaming):
    bases, offs = synth.make_records(50_000, 3, repeats_per_mb=20_000, motif_len=50, seed=51)
    path = _fasta(tmp_path, bases, offs)
    args = [_lib.CLI_PATH, "-i", path, "-k", "21", "--pool-size", "4001"]
    if canon:
        args.append("--canonical")
    if streaming:
        args.append("--streaming")
    out = subprocess.run(args, capture_output=True, check=True, text=True).stdout
    seqs = synth.records_list(bases, offs)
    p = pyref.SpikingKmerCounter(21, 1.0, 0.95, 2, 1.0, 4001, canon)
    (p.process_streaming if streaming else p.process_parallel)(seqs)
    block = pyref.cli_result_block(p, 4001, streaming)
    assert out.endswith(block), out[-2000:]
    if not streaming:
        assert f"  In-memory total current: {sum(p.currents)}\n" in out


def test_errors_fail_loudly():
    with pytest.raises(_lib.NeuroKmerError):
        SpikingKmerCounter(0, 1.0, 0.95, 2, 1.0, 100, True)
    g = SpikingKmerCounter(5, 1.0, 0.95, 2, 1.0, 0, True)
    with pytest.raises(_lib.NeuroKmerError):
        g.process_parallel([b"ACGTACGTAC"])
    g.process_parallel([b"ACG"])  # no k-mers: the reference does not panic either
    g2 = SpikingKmerCounter(5, 1.0, 0.95, 2, 1.0, 10, True)
    # a fresh counter: any n (min(n, pool) rows in index order), empty counts
    assert g2.top_abundant_neurons(21) == [(i, 0, 0) for i in range(10)]
    assert g2.get_count(0) is None
    with pytest.raises(_lib.NeuroKmerError):
        g2.get_counts128([1])  # 64-bit handle


@pytest.mark.parametrize("shape", ["config2"])
def test_full_size_properties(shape):
    """Config-2 size (115 Mbases, 7 records, k=31, pool=2M): size-independent
    properties at full size + bit-exact parity on a prefix."""
    bases, offs = synth.make_records(115_000_000, 7, repeats_per_mb=64, motif_len=200)
    d_b = torch.from_numpy(bases).cuda()
    d_o = torch.from_numpy(offs.view(np.int64)).cuda()
    torch.cuda.synchronize()
    g = SpikingKmerCounter(31, 1.0, 0.95, 2, 1.0, 2_000_000, True)
    g.process_parallel_device(d_b.data_ptr(), d_o.data_ptr(), 7, bases.size)
    cur1, sc1, top1 = g.currents(), g.spike_counts(), g.top_abundant_neurons(20)
    nk = int(np.clip(np.diff(offs.astype(np.int64)) - 30, 0, None).sum())
    assert int(cur1.sum()) == nk                      # every k-mer counted once
    assert int(sc1.sum()) == g.energy.total_spikes()  # spikes conserved
    g.reset()
    g.process_parallel_device(d_b.data_ptr(), d_o.data_ptr(), 7, bases.size)
    np.testing.assert_array_equal(g.currents(), cur1)  # deterministic
    assert g.top_abundant_neurons(20) == top1
    # linearity: per-record shards sum to the whole
    acc = np.zeros_like(cur1)
    h = SpikingKmerCounter(31, 1.0, 0.95, 2, 1.0, 2_000_000, True)
    for i in range(7):
        lo, hi = int(offs[i]), int(offs[i + 1])
        o = np.array([0, hi - lo], np.uint64)
        sub = torch.from_numpy(np.ascontiguousarray(bases[lo:hi])).cuda()
        so = torch.from_numpy(o.view(np.int64)).cuda()
        torch.cuda.synchronize()
        h.accumulate_device(sub.data_ptr(), so.data_ptr(), 1, hi - lo)
        acc += h.currents()
    np.testing.assert_array_equal(acc, cur1)
    # bit-exact vs the oracle on 2.1 Mbases: the first 300 kbases of each record
    # (the whole input is compared in test_config2_full_parity)
    per = 300_000
    segs = [bases[int(offs[i]):int(offs[i]) + per] for i in range(7)]
    po = np.arange(8, dtype=np.uint64) * per
    pb = np.concatenate(segs)
    gg, rr = run_both(pb, po, 31, 2_000_000, True)
    assert_same(gg, rr)


def test_config2_full_parity():
    """BASELINE.json configs[1] at its full size: 115,000,000 bases in 7
    records, k=31, pool=2M, canonical.  The GPU's process_parallel over the
    whole input against oracle/nk_oracle.c's process_parallel restatement
    (one thread per record like rayon, src/spiking_hash.rs:84-201), every
    output bit-exact: currents, spike counts, voltages (bitwise), refractory,
    total spikes, energy, top-20 rows with their uniques.  The same input
    bench.py times (synth seed, 64 x 200-bp planted repeats per MB)."""
    bases, offs = synth.make_records(115_000_000, 7, repeats_per_mb=64, motif_len=200)
    d_b = torch.from_numpy(np.concatenate([bases, np.zeros(16, np.uint8)])).cuda()
    d_o = torch.from_numpy(offs.view(np.int64)).cuda()
    torch.cuda.synchronize()
    g = SpikingKmerCounter(31, 1.0, 0.95, 2, 1.0, 2_000_000, True)
    g.process_parallel_device(d_b.data_ptr(), d_o.data_ptr(), 7, bases.size)
    del d_b
    r = cbind.OracleCounter(31, 1.0, 0.95, 2, 1.0, 2_000_000, True)
    r.process_parallel_arrays(bases, offs, 7)
    assert_same(g, r)
    nk = int(np.clip(np.diff(offs.astype(np.int64)) - 30, 0, None).sum())
    assert int(g.currents().sum()) == nk == 114_999_790
    g.close()


# ---- exact k-mer table and process_sequence (§8f-3) --------
def _keys_of(bases, offs, k, canon, width=64):
    out = set()
    for i in range(offs.size - 1):
        rec = bases[int(offs[i]):int(offs[i + 1])].tobytes()
        out.update(int(x) for x in cbind.kmer_keys(rec, k, canon))
    return out


def assert_exact_same(g, r, keys, pool):
    np.testing.assert_array_equal(g.kmer_per_neuron(), r.kmer_per_neuron())
    assert g.distinct_kmers() == r.distinct_kmers()
    rng = np.random.default_rng(len(keys))
    probe = sorted(keys)
    probe += [int(x) for x in rng.integers(0, 2**63, 500, dtype=np.uint64)]  # mostly absent
    cnt, pres = g.get_counts(np.array(probe, dtype=np.uint64))
    for kk, c, p in zip(probe, cnt, pres):
        want = r.get_count(kk)
        assert (int(c) if p else None) == want, kk
    if probe:
        assert g.get_count(probe[0]) == r.get_count(probe[0])


@pytest.mark.parametrize("k,canon", [(21, True), (21, False), (31, True), (32, False),
                                     (33, True), (40, False), (5, True)])
def test_exact_counts_table(k, canon):
    bases, offs = ragged_records(total=90_000, n_rate=0.01, mixed_case=True, seed=300 + k,
                                 repeats_per_mb=20_000, motif_len=70)
    g = SpikingKmerCounter(k, 1.0, 0.95, 2, 1.0, 4099, canon, exact_counts=True)
    r = cbind.OracleCounter(k, 1.0, 0.95, 2, 1.0, 4099, canon)
    g.process_parallel_arrays(bases, offs)
    r.process_parallel_arrays(bases, offs)
    assert_same(g, r)
    assert_exact_same(g, r, _keys_of(bases, offs, k, canon), 4099)


def test_exact_counts_partitioned_config2_shape():
    # the metric's path (k=31, pool 2M, partitioned count) with the table on
    bases, offs = synth.make_records(2_000_000, 7, repeats_per_mb=64, motif_len=200, seed=3)
    g = SpikingKmerCounter(31, 1.0, 0.95, 2, 1.0, 2_000_000, True, exact_counts=True)
    r = cbind.OracleCounter(31, 1.0, 0.95, 2, 1.0, 2_000_000, True)
    g.process_parallel_arrays(bases, offs)
    r.process_parallel_arrays(bases, offs)
    assert_same(g, r)
    np.testing.assert_array_equal(g.kmer_per_neuron(), r.kmer_per_neuron())
    assert g.distinct_kmers() == r.distinct_kmers()


def test_table_on_demand_needs_a_held_input():
    """Without exact_counts the table is built from the last input on demand;
    device input passed by pointer is the caller's, so those queries refuse."""
    g = SpikingKmerCounter(21, 1.0, 0.95, 2, 1.0, 1000, True)
    assert g.get_count(5) is None  # fresh: empty counts
    bases, offs = synth.make_records(20_000, 3, seed=4)
    d_b = torch.from_numpy(np.concatenate([bases, np.zeros(16, np.uint8)])).cuda()
    d_o = torch.from_numpy(offs.view(np.int64)).cuda()
    torch.cuda.synchronize()
    g.process_parallel_device(d_b.data_ptr(), d_o.data_ptr(), offs.size - 1, int(offs[-1]))
    for call in (lambda: g.get_count(5), lambda: g.top_abundant_neurons(500),
                 lambda: g.process_sequence(b"ACGT" * 20), g.distinct_kmers):
        with pytest.raises(_lib.NeuroKmerError) as e:
            call()
        assert e.value.code == _lib.NK_E_UNSUPPORTED
    assert len(g.top_abundant_neurons(20)) == 20  # the call's own rows need no table
    with pytest.raises(_lib.NeuroKmerError):
        SpikingKmerCounter(31, 1.0, 0.95, 2, 1.0, 1000, True, kmer_width=128).process_sequence(
            b"ACGT" * 20)


@pytest.mark.parametrize("canon", [True, False])
def test_process_sequence_matches_reference(canon):
    """process_parallel, then reads through process_sequence (single LIF step,
    accumulating counts and kmer_per_neuron), a reset, more reads."""
    k, pool = 17, 997
    bases, offs = synth.make_records(60_000, 4, repeats_per_mb=30_000, motif_len=50, seed=8,
                                     n_rate=0.003)
    reads, roffs = synth.make_reads(120, 90, seed=9)
    rl = synth.records_list(reads, roffs)
    rl[3] = rl[3][:10]           # shorter than k: no-op
    rl[5] = b"N" * 40 + rl[5]    # invalid bytes
    g = SpikingKmerCounter(k, 1.0, 0.95, 2, 1.0, pool, canon, exact_counts=True)
    r = cbind.OracleCounter(k, 1.0, 0.95, 2, 1.0, pool, canon)
    g.process_parallel_arrays(bases, offs)
    r.process_parallel_arrays(bases, offs)
    keys = _keys_of(bases, offs, k, canon)
    for i, rd in enumerate(rl):
        g.process_sequence(rd)
        r.process_sequence(rd)
        keys.update(int(x) for x in cbind.kmer_keys(rd, k, canon))
        if i % 30 == 29:
            assert_same(g, r)
            assert_exact_same(g, r, keys, pool)
    g.reset()
    r2 = cbind.OracleCounter(k, 1.0, 0.95, 2, 1.0, pool, canon)
    keys2 = set()
    for rd in rl[:40]:
        g.process_sequence(rd)
        r2.process_sequence(rd)
        keys2.update(int(x) for x in cbind.kmer_keys(rd, k, canon))
    assert_same(g, r2)
    assert_exact_same(g, r2, keys2, pool)


# ---- GPU FASTX ingest: chunked device parse ---------------
from neurokmer_amd.fastx import stream_sequences  # noqa: E402


def _ingest_check(path, k, pool, canon, streaming, chunk, exact=False, fastq_device=False,
                  max_rec=None):
    """fastq_device: the device FASTQ parse (NK_FASTQ_DEVICE, as gzip FASTQ
    takes) instead of the host extraction of an uncompressed FASTQ; max_rec:
    record ends per host window call (NK_FQ_MAX_REC)."""
    keys = {"NK_INGEST_CHUNK": str(chunk), "NK_FASTQ_DEVICE": "1" if fastq_device else None,
            "NK_FQ_MAX_REC": str(max_rec) if max_rec else None}
    old = {key: os.environ.get(key) for key in keys}
    for key, v in keys.items():
        if v is None:
            os.environ.pop(key, None)
        else:
            os.environ[key] = v
    try:
        g = SpikingKmerCounter(k, 1.0, 0.95, 2, 1.0, pool, canon, exact_counts=exact)
        (g.process_file_streaming if streaming else g.process_file_parallel)(path)
    finally:
        for key, v in old.items():
            if v is None:
                os.environ.pop(key, None)
            else:
                os.environ[key] = v
    recs = list(stream_sequences(path))  # the host reader's records (mirror)
    r = cbind.OracleCounter(k, 1.0, 0.95, 2, 1.0, pool, canon)
    (r.process_streaming if streaming else r.process_parallel)(recs)
    assert_same(g, r)
    if exact:
        np.testing.assert_array_equal(g.kmer_per_neuron(), r.kmer_per_neuron())
        assert g.distinct_kmers() == r.distinct_kmers()
    return recs


def _crlf(data: bytes) -> bytes:
    return data.replace(b"\n", b"\r\n")


@pytest.mark.parametrize("k,canon", [(5, True), (31, True), (31, False), (33, True), (63, False)])
@pytest.mark.parametrize("chunk", [4099, 65536, 1 << 26])
def test_ingest_fasta_chunks(tmp_path, k, canon, chunk):
    bases, offs = synth.make_records(120_000, 9, seed=k + chunk % 97, n_rate=0.01, mixed_case=True,
                                     repeats_per_mb=20_000, motif_len=60)
    p = tmp_path / "a.fa"
    synth.write_fasta(str(p), bases, offs, width=61)
    data = p.read_bytes()
    # an empty record and a record whose single line spans several chunks
    data = data.replace(b">s3\n", b">empty\n>s3\n", 1) + b">long\n" + b"ACGTTGCA" * 3000 + b"\n"
    p.write_bytes(_crlf(data) if k == 31 else data)
    recs = _ingest_check(str(p), k, 7001, canon, (k + chunk) % 2 == 1, chunk)
    assert len(recs) == 11


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_ingest_fasta_random_layout(tmp_path, seed):
    """Random FASTA layouts against the reader's rules (neurokmer_amd/fastx.py,
    src/utils.rs:9-24): lines of 0..200 bytes, headers with '>' and spaces
    inside, '>' and '\\r' inside sequence lines, CRLF on some lines, blank
    lines, no final newline -- at chunk sizes that cut lines and headers
    anywhere (the 16-B-group parse: each group's first byte's line start
    comes from the lane below or a load)."""
    rng = np.random.default_rng(seed)
    alpha = np.frombuffer(b"ACGTNacgt>\r", np.uint8)
    parts = []
    for r in range(int(rng.integers(20, 60))):
        hdr = bytes(rng.choice(np.frombuffer(b"abc >xyz_123", np.uint8), int(rng.integers(0, 90))))
        parts.append(b">" + hdr + (b"\r\n" if rng.random() < 0.3 else b"\n"))
        for _ in range(int(rng.integers(0, 12))):
            line = bytes(rng.choice(alpha, int(rng.integers(0, 200)),
                                    p=[0.235] * 4 + [0.01] * 5 + [0.005, 0.005]))
            if line.startswith(b">"):
                line = b"A" + line
            parts.append(line + (b"\r\n" if rng.random() < 0.3 else b"\n"))
    data = b"".join(parts)
    if rng.random() < 0.5:
        data = data.rstrip(b"\r\n")
    p = tmp_path / "r.fa"
    p.write_bytes(data)
    chunk = int(rng.integers(4099, 70_000))
    _ingest_check(str(p), 11, 997, True, False, chunk)


@pytest.mark.parametrize("chunk", [4099, 65536])
def test_ingest_fasta_long_header_and_inner_gt(tmp_path, chunk):
    """A header line longer than several chunks (its line state carried from
    chunk to chunk), '>' inside a sequence line (a base byte, not a record),
    a header as the file's last line without a newline."""
    bases, offs = synth.make_records(60_000, 3, seed=chunk % 89)
    p = tmp_path / "h.fa"
    synth.write_fasta(str(p), bases, offs, width=70)
    data = p.read_bytes()
    data = data.replace(b">s1\n", b">s1 " + b"x" * 10_000 + b"\n", 1)
    lines = data.split(b"\n")
    lines[5] = lines[5][:20] + b">" + lines[5][20:]
    data = b"\n".join(lines) + b">tail header, no newline"
    p.write_bytes(data)
    _ingest_check(str(p), 21, 5003, True, False, chunk)


@pytest.mark.parametrize("chunk", [1000, 30000, 1 << 26])
@pytest.mark.parametrize("streaming", [True, False])
@pytest.mark.parametrize("fastq_device", [False, True])
def test_ingest_fastq_chunks(tmp_path, chunk, streaming, fastq_device):
    reads, roffs = synth.make_reads(400, 150, seed=5, n_rate=0.005, repeats_per_mb=40_000,
                                    motif_len=50)
    longr, loffs = synth.make_reads(3, 2500, seed=6)  # records longer than a chunk
    p = tmp_path / "r.fq"
    synth.write_fastq(str(p), np.concatenate([reads, longr]),
                      np.concatenate([roffs, loffs[1:] + roffs[-1]]).astype(np.uint64))
    data = p.read_bytes()
    p.write_bytes(_crlf(data) if chunk == 30000 else data.rstrip(b"\n"))  # CRLF / no final '\n'
    recs = _ingest_check(str(p), 21, 5003, True, streaming, chunk, exact=chunk == 1000,
                         fastq_device=fastq_device)
    assert len(recs) == 403


def test_ingest_fastq_record_longer_than_carry_room(tmp_path):
    """A FASTQ record (~300 KB with its quality line) far past the carry room
    in front of a device chunk buffer (max(chunk / 8, 64 KB)): the buffers
    regrow, several times, while the next chunk's bytes are already up."""
    reads, roffs = synth.make_reads(300, 150, seed=15, n_rate=0.005)
    longr, loffs = synth.make_reads(2, 150_000, seed=16, n_rate=0.001)
    allr = np.concatenate([reads[:int(roffs[100])], longr, reads[int(roffs[100]):]])
    lens = np.concatenate([np.diff(roffs)[:100], np.diff(loffs), np.diff(roffs)[100:]])
    offs = np.zeros(lens.size + 1, np.uint64)
    np.cumsum(lens, out=offs[1:])
    p = tmp_path / "long.fq"
    synth.write_fastq(str(p), allr, offs)
    recs = _ingest_check(str(p), 25, 6007, True, True, 50_001)
    assert len(recs) == 302


@pytest.mark.parametrize("fastq_device,max_rec", [(False, None), (True, None), (False, 7)])
def test_ingest_fastq_stops_at_malformed_record(tmp_path, capfd, fastq_device, max_rec):
    reads, roffs = synth.make_reads(300, 120, seed=7)
    p = tmp_path / "bad.fq"
    synth.write_fastq(str(p), reads, roffs)
    lines = p.read_bytes().split(b"\n")
    lines[4 * 150 + 3] = lines[4 * 150 + 3][:-1]  # record 150: quality one byte short
    p.write_bytes(b"\n".join(lines))
    capfd.readouterr()
    recs = _ingest_check(str(p), 19, 3001, True, True, 2000, fastq_device=fastq_device,
                         max_rec=max_rec)
    assert len(recs) == 150
    # the reference's `warn!("Skipping malformed record: ...")` (src/utils.rs:17-19):
    # the library's own line (and the Python mirror's, which the check reads too)
    err = capfd.readouterr().err
    assert sum("Skipping malformed record" in ln and "record 150 of" in ln
               for ln in err.splitlines()) == 2, err


@pytest.mark.parametrize("fastq_device", [False, True])
def test_ingest_fastq_xcd_subregions_many_small_launches(tmp_path, fastq_device):
    """Pool > 4.2 M (K1a's per-XCD sub-regions) counted in many small launches
    (1 MB ingest windows): every launch's tiles fill the eight sub-regions
    evenly, and the result is the oracle's."""
    reads, roffs = synth.make_reads(24_000, 150, seed=8, n_rate=0.001, repeats_per_mb=2000,
                                    motif_len=70)
    p = tmp_path / "sub.fq"
    synth.write_fastq(str(p), reads, roffs)
    recs = _ingest_check(str(p), 31, 6_000_007, True, True, 1_000_003, fastq_device=fastq_device)
    assert len(recs) == 24_000


def test_ingest_fastq_blank_lines_use_host_reader(tmp_path):
    reads, roffs = synth.make_reads(200, 100, seed=8)
    p = tmp_path / "blank.fq"
    synth.write_fastq(str(p), reads, roffs)
    lines = p.read_bytes().split(b"\n")
    lines.insert(4 * 77, b"")  # a blank line between records: skipped by the reader
    p.write_bytes(b"\n".join(lines))
    recs = _ingest_check(str(p), 17, 2003, True, False, 3000)
    assert len(recs) == 200
    recs = _ingest_check(str(p), 17, 2003, True, True, 3000, fastq_device=True)
    assert len(recs) == 200


def test_ingest_gzip(tmp_path):
    import gzip
    bases, offs = synth.make_records(200_000, 5, seed=12, n_rate=0.002, repeats_per_mb=10_000,
                                     motif_len=80)
    p = tmp_path / "g.fa.gz"
    raw = tmp_path / "g.fa"
    synth.write_fasta(str(raw), bases, offs, width=70)
    p.write_bytes(gzip.compress(raw.read_bytes()))
    _ingest_check(str(p), 27, 9001, True, False, 50_000)
    q = tmp_path / "g.fq.gz"
    rq = tmp_path / "g.fq"
    reads, roffs = synth.make_reads(500, 130, seed=13)
    synth.write_fastq(str(rq), reads, roffs)
    q.write_bytes(gzip.compress(rq.read_bytes()))
    _ingest_check(str(q), 23, 4001, False, True, 20_000)
