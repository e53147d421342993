"""K1b deferred into the next handle's count kernel (nk_opts.defer_hist,
k_part_fused; bench.py's three batches in flight).  A handle's bucket
histogram then runs inside another handle's hash kernel -- in thirds of each
bucket, with the other thirds' LDS adds dropped past the allocation -- or, when
no count takes it, by whatever reads the handle's counts first.  Every batch's
results are compared bit-exactly with oracle/nk_oracle.c: currents, spike
counts, top rows with uniques, total spikes.

Reference: src/spiking_hash.rs:84-201 (process_parallel), :661-673 (top rows).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("no GPU", allow_module_level=True)

from neurokmer_amd import SpikingKmerCounter, synth  # noqa: E402
from oracle import cbind  # noqa: E402

K = 31
_CACHE = {}


def _inputs(pool, n, bases=5_300_000, k=K, canonical=True, **kw):
    """n inputs of >= 512 tiles (the fused count's minimum) and their oracle results."""
    key = (pool, n, bases, k, canonical, tuple(sorted(kw.items())))
    if key in _CACHE:
        return _CACHE[key]
    out = []
    for i in range(n):
        b, o = synth.make_records(bases + 131_071 * i, 6, seed=4200 + i,
                                  repeats_per_mb=kw.get("repeats", 400), motif_len=120)
        if kw.get("poly_a"):
            b[100_000:100_000 + 900_000] = ord("A")  # one hot neuron: ~900 k records in one bin
        ref = cbind.OracleCounter(k, 1.0, 0.95, 2, 1.0, pool, canonical)
        ref.process_parallel_arrays(b, o)
        d_b = torch.from_numpy(np.concatenate([b, np.zeros(16, np.uint8)])).cuda()
        d_o = torch.from_numpy(o.view(np.int64)).cuda()
        out.append((b, o, d_b, d_o, ref.top_abundant_neurons(20), ref.total_spikes,
                    ref.currents(), ref.spike_counts()))
    torch.cuda.synchronize()
    _CACHE[key] = out
    return out


def _check(c, inp, i):
    top, spikes, cur, sc = inp[4:]
    assert c.top_abundant_neurons(20) == top, i
    assert c.energy.total_spikes() == spikes, i
    np.testing.assert_array_equal(c.currents(), cur)
    np.testing.assert_array_equal(c.spike_counts(), sc)


def _pipeline(pool, m, n, inputs, one_stream=True, k=K, canonical=True, reset=True):
    ctrs = [SpikingKmerCounter(k, 1.0, 0.95, 2, 1.0, pool, canonical, defer_hist=True)
            for _ in range(m)]
    for c in ctrs:
        c.set_stage_timing(3)
    cs = torch.cuda.Stream()
    count_streams = [cs] * m if one_stream else [torch.cuda.Stream() for _ in range(m)]
    fin = torch.cuda.Stream(priority=torch.cuda.Stream.priority_range()[1])
    which = [(i * 3) % len(inputs) for i in range(n)]

    def start(i):
        c, st = ctrs[i % m], count_streams[i % m].cuda_stream
        b, o, d_b, d_o = inputs[which[i]][:4]
        if reset:
            c.reset(st, blocking=False)
        c.accumulate_device(d_b.data_ptr(), d_o.data_ptr(), o.size - 1, b.size, st)

    for j in range(m - 1):
        start(j)
    for i in range(n):
        if i + m - 1 < n:
            start(i + m - 1)
        c = ctrs[i % m]
        c.finalize(False, fin.cuda_stream)
        _check(c, inputs[which[i]], i)
    for c in ctrs:
        c.close()


@pytest.mark.parametrize("m", [3, 4])
def test_deferred_histogram_in_flight_matches_the_oracle(m):
    pool = 2_000_000
    _pipeline(pool, m, 9, _inputs(pool, 4))


@pytest.mark.parametrize("pool", [1_000_003, 6_000_007, 32_768, 100])
def test_deferred_histogram_pools(pool):
    """A partial last bucket, XCD sub-regions (184 buckets), one bucket, a tiny pool."""
    _pipeline(pool, 3, 6, _inputs(pool, 3))


def test_deferred_histogram_hot_bin_and_other_modes():
    """~900 k records in one bin (poly-A) through the fused thirds; k < 16 and
    non-canonical keys take the other fused kernels."""
    pool = 2_000_000
    _pipeline(pool, 3, 5, _inputs(pool, 3, poly_a=True))
    _pipeline(pool, 3, 4, _inputs(pool, 2, k=11), k=11)
    _pipeline(pool, 3, 4, _inputs(pool, 2, canonical=False), canonical=False)


def test_deferred_histogram_separate_streams_and_no_reset():
    """Counts on different streams are never fused (each histogram runs when its
    finish reads it); without a reset each count still replaces the currents
    (src/spiking_hash.rs:174-176 stores them), so a reader sees its last batch's
    -- whichever kernel ran that batch's histogram."""
    pool = 2_000_000
    inputs = _inputs(pool, 3)
    _pipeline(pool, 3, 6, inputs, one_stream=False)
    # no reset, no finish between the counts
    m, n = 3, 6
    ctrs = [SpikingKmerCounter(K, 1.0, 0.95, 2, 1.0, pool, True, defer_hist=True) for _ in range(m)]
    st = torch.cuda.Stream().cuda_stream
    for i in range(n):
        b, o, d_b, d_o = inputs[i % 3][:4]
        ctrs[i % m].accumulate_device(d_b.data_ptr(), d_o.data_ptr(), o.size - 1, b.size, st)
    for j, c in enumerate(ctrs):
        last = max(i for i in range(n) if i % m == j)
        np.testing.assert_array_equal(c.currents(), inputs[last % 3][6])
        c.close()


def test_deferred_histogram_owner_freed_or_reset():
    """A pending histogram whose owner is reset (voided) or freed is never run
    by the next count; the next handle's results are its own."""
    pool = 2_000_000
    inputs = _inputs(pool, 2)
    st = torch.cuda.Stream().cuda_stream
    a = SpikingKmerCounter(K, 1.0, 0.95, 2, 1.0, pool, True, defer_hist=True)
    b = SpikingKmerCounter(K, 1.0, 0.95, 2, 1.0, pool, True, defer_hist=True)
    x0, x1 = inputs
    a.accumulate_device(x0[2].data_ptr(), x0[3].data_ptr(), x0[1].size - 1, x0[0].size, st)
    a.reset(st, blocking=False)  # voids a's pending histogram
    b.accumulate_device(x1[2].data_ptr(), x1[3].data_ptr(), x1[1].size - 1, x1[0].size, st)
    a.accumulate_device(x0[2].data_ptr(), x0[3].data_ptr(), x0[1].size - 1, x0[0].size, st)
    a.close()  # a's histogram pending in the slot: dropped with the handle
    c = SpikingKmerCounter(K, 1.0, 0.95, 2, 1.0, pool, True, defer_hist=True)
    c.accumulate_device(x0[2].data_ptr(), x0[3].data_ptr(), x0[1].size - 1, x0[0].size, st)
    b.finalize(False, st)
    _check(b, x1, "b")
    c.finalize(False, st)
    _check(c, x0, "c")
    b.close()
    c.close()


def test_deferred_histogram_counted_on_one_thread_read_on_another():
    """Counts enqueued by a worker thread (each one's K1b taken by the next, the
    last left in the slot under that thread), then read from the main thread --
    one handle used by one thread at a time, as the header states -- while the
    main thread's own deferred counts on other handles never take the worker's
    pending histogram (a slot is taken only from the thread that left it)."""
    import threading
    pool = 2_000_000
    inputs = _inputs(pool, 3)
    ctrs = [SpikingKmerCounter(K, 1.0, 0.95, 2, 1.0, pool, True, defer_hist=True) for _ in range(3)]
    st = torch.cuda.Stream()
    err = []

    def worker():
        try:
            for i, c in enumerate(ctrs):
                b, o, d_b, d_o = inputs[i][:4]
                c.accumulate_device(d_b.data_ptr(), d_o.data_ptr(), o.size - 1, b.size, st.cuda_stream)
        except Exception as e:  # pragma: no cover - reported below
            err.append(e)

    t = threading.Thread(target=worker)
    t.start()
    t.join()
    assert not err, err
    # the main thread counts on two other handles on the same stream first
    other = [SpikingKmerCounter(K, 1.0, 0.95, 2, 1.0, pool, True, defer_hist=True) for _ in range(2)]
    for j, c in enumerate(other):
        b, o, d_b, d_o = inputs[2 - j][:4]
        c.accumulate_device(d_b.data_ptr(), d_o.data_ptr(), o.size - 1, b.size, st.cuda_stream)
    for i, c in enumerate(ctrs):
        c.finalize(False, st.cuda_stream)
        _check(c, inputs[i], i)
    for j, c in enumerate(other):
        c.finalize(False, st.cuda_stream)
        _check(c, inputs[2 - j], f"other{j}")
    for c in ctrs + other:
        c.close()
