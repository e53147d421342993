"""Batches in flight on one GPU (bench.py --inflight): handles
counting on their own streams while an earlier batch's finish runs on a shared
high-priority stream.  Each finish must see exactly its own batch's count --
the library orders a handle's calls across streams on the event recorded at the
end of nk_accumulate_device, not on one recorded when the stream switches
(which would also wait for other handles' work, or, recorded too early, miss
its own).  Every batch's results are compared bit-exactly with oracle/nk_oracle.c
on the same input (different inputs cycle through the handles, so a finish that
read another batch's or a stale count would differ).

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

K, POOL = 31, 200_003


def _inputs(n):
    out = []
    for i in range(n):
        b, o = synth.make_records(1_500_000 + 97_001 * i, 5, seed=900 + i, repeats_per_mb=3_000,
                                  motif_len=150)
        ref = cbind.OracleCounter(K, 1.0, 0.95, 2, 1.0, POOL, True)
        ref.process_parallel_arrays(b, o)
        d_b = torch.from_numpy(np.concatenate([b, np.zeros(16, np.uint8)])).cuda()
        d_o = torch.from_numpy(o.view(np.int64)).cuda()
        out.append((b, o, d_b, d_o, ref.top_abundant_neurons(20), ref.total_spikes,
                    ref.currents()))
    torch.cuda.synchronize()
    return out


@pytest.mark.parametrize("m", [2, 3])
def test_batches_in_flight_match_the_oracle(m):
    inputs = _inputs(4)
    ctrs = [SpikingKmerCounter(K, 1.0, 0.95, 2, 1.0, POOL, True) for _ in range(m)]
    for c in ctrs:
        c.set_stage_timing(3)
    count_streams = [torch.cuda.Stream() for _ in range(m)]
    fin = torch.cuda.Stream(priority=torch.cuda.Stream.priority_range()[1])
    n = 11
    which = [(i * 3) % len(inputs) for i in range(n)]  # the input of batch i

    def start(i):
        c, st = ctrs[i % m], count_streams[i % m].cuda_stream
        b, o, d_b, d_o = inputs[which[i]][:4]
        c.reset(st, blocking=False)
        c.accumulate_device(d_b.data_ptr(), d_o.data_ptr(), o.size - 1, b.size, st)

    for j in range(m - 1):
        start(j)
    for i in range(n):
        if i + m - 1 < n:
            start(i + m - 1)
        c = ctrs[i % m]
        c.finalize(False, fin.cuda_stream)
        top, spikes, cur = inputs[which[i]][4:]
        assert c.top_abundant_neurons(20) == top, i
        assert c.energy.total_spikes() == spikes, i
        np.testing.assert_array_equal(c.currents(), cur)
    for c in ctrs:
        c.close()


def test_finish_waits_for_its_count_only():
    """Handle A counts on stream X, handle B's (much larger) count is queued
    behind it on X, then A finishes on stream Y: A's results are its own, and
    B finishes afterwards on Y with its own."""
    small = _inputs(1)[0]
    b2, o2 = synth.make_records(8_000_000, 7, seed=77, repeats_per_mb=64, motif_len=200)
    ref2 = cbind.OracleCounter(K, 1.0, 0.95, 2, 1.0, POOL, True)
    ref2.process_parallel_arrays(b2, o2)
    d_b2 = torch.from_numpy(np.concatenate([b2, np.zeros(16, np.uint8)])).cuda()
    d_o2 = torch.from_numpy(o2.view(np.int64)).cuda()
    torch.cuda.synchronize()
    a = SpikingKmerCounter(K, 1.0, 0.95, 2, 1.0, POOL, True)
    b = SpikingKmerCounter(K, 1.0, 0.95, 2, 1.0, POOL, True)
    x, y = torch.cuda.Stream(), torch.cuda.Stream()
    bs, os_, d_b, d_o = small[:4]
    a.accumulate_device(d_b.data_ptr(), d_o.data_ptr(), os_.size - 1, bs.size, x.cuda_stream)
    b.accumulate_device(d_b2.data_ptr(), d_o2.data_ptr(), o2.size - 1, b2.size, x.cuda_stream)
    a.finalize(False, y.cuda_stream)
    assert a.top_abundant_neurons(20) == small[4]
    assert a.energy.total_spikes() == small[5]
    b.finalize(False, y.cuda_stream)
    assert b.top_abundant_neurons(20) == ref2.top_abundant_neurons(20)
    assert b.energy.total_spikes() == ref2.total_spikes
    a.close()
    b.close()
