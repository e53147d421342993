"""The RCCL (torch "nccl") device-tensor branches of neurokmer_amd/dist.py in a
1-rank process group on the test box's GPU: the
multi-rank tests run gloo, which host-stages every collective, so these are
the runs in which reduce_scatter_tensor, the device all_gather_into_tensor and
all_to_all_single on device tensors execute.  The "+comm" cases run the same
finishes inside the library with its own RCCL communicator (nk_comm_new,
nk_finalize_dist, nk_finalize_sliced_dist).  Each case checks the finished
state bit-exactly against oracle/nk_oracle.c on the same input.

Reference: src/spiking_hash.rs:84-201 (process_parallel), :157-172 (counts,
kmer_per_neuron), :661-673 (top rows), :675-682 (get_count); the exchange is
the build's own.
"""
import os
import socket
import traceback

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("no GPU", allow_module_level=True)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _input(total, seed, recs=5):
    from neurokmer_amd import synth
    return synth.make_records(total, recs, seed=seed, repeats_per_mb=20_000, motif_len=90,
                              n_rate=0.002, mixed_case=True)


def _check_same(g, r, n=20):
    np.testing.assert_array_equal(g.currents(), r.currents())
    np.testing.assert_array_equal(g.spike_counts(), r.spike_counts())
    np.testing.assert_array_equal(g.voltages().view(np.uint32), r.voltages().view(np.uint32))
    np.testing.assert_array_equal(g.refractory(), r.refractory())
    assert g.energy.total_spikes() == r.total_spikes
    assert g.energy_used() == r.energy_used()
    assert g.top_abundant_neurons(n) == r.top_abundant_neurons(n)


def _case(name):
    """One scenario in this (1-rank nccl) process; raises on a mismatch."""
    import torch.distributed as dist
    from neurokmer_amd import dist as nkdist
    assert dist.get_backend() == "nccl"
    comm = None
    if name.endswith("+comm"):  # the finish inside the library (nk_finalize_dist)
        comm = nkdist.Comm()
        name = name[:-5]
    try:
        _run(name, comm)
    finally:
        if comm is not None:
            comm.close()


def _run(name, comm):
    from neurokmer_amd import SpikingKmerCounter
    from neurokmer_amd import dist as nkdist
    from neurokmer_amd._lib import NK_E_UNSUPPORTED, NeuroKmerError
    from oracle import cbind

    def dev_input(bases, offs):
        d_b = torch.from_numpy(np.concatenate([bases, np.zeros(16, np.uint8)])).cuda()
        d_o = torch.from_numpy(offs.astype(np.uint64).view(np.int64)).cuda()
        torch.cuda.synchronize()
        return d_b, d_o

    if name.startswith("finalize_step"):
        k, pool = 31, 2_000_000
        bases, offs = _input(1_500_000, 61)
        d_b, d_o = dev_input(bases, offs)
        g = SpikingKmerCounter(k, 1.0, 0.95, 2, 1.0, pool, True)
        r = cbind.OracleCounter(k, 1.0, 0.95, 2, 1.0, pool, True)
        tk = int(offs[-1]) if name == "finalize_step_u32" else None
        for _ in range(3):  # state carries over between steps
            g.accumulate_device(d_b.data_ptr(), d_o.data_ptr(), offs.size - 1, bases.size)
            nkdist.finalize_step(g, total_kmers=tk, comm=comm)
            r.process_parallel_arrays(bases, offs, 4)
            torch.cuda.synchronize()
            _check_same(g, r)
        return
    if name.startswith("sliced"):
        width = 128 if name.endswith("128") else 64
        k, pool = 63, (1 << 24) + 5
        bases, offs = _input(1_000_000, 62)
        d_b, d_o = dev_input(bases, offs)
        g = SpikingKmerCounter(k, 1.0, 0.95, 2, 1.0, pool, True, kmer_width=width)
        r = cbind.OracleCounter(k, 1.0, 0.95, 2, 1.0, pool, True, width=width)
        tk = int(offs[-1]) if width == 64 else None  # u32 wire / u64 wire
        for _ in range(2):
            g.accumulate_device(d_b.data_ptr(), d_o.data_ptr(), offs.size - 1, bases.size)
            nkdist.finalize_step_sliced(g, total_kmers=tk, comm=comm)
            r.process_parallel_arrays(bases, offs, 4)
        torch.cuda.synchronize()
        st = nkdist.gather_state(g)
        np.testing.assert_array_equal(st["currents"], r.currents())
        np.testing.assert_array_equal(st["spike_counts"], r.spike_counts())
        np.testing.assert_array_equal(st["voltages"].view(np.uint32), r.voltages().view(np.uint32))
        np.testing.assert_array_equal(st["refractory"], r.refractory())
        assert g.top_abundant_neurons(20) == r.top_abundant_neurons(20)
        assert g.energy.total_spikes() == r.total_spikes
        # sharded state: whole-pool calls refuse until a reset
        for call in (lambda: g.finalize(False), lambda: g.top_abundant_neurons(21),
                     lambda: g.simulate_spikes_auto(),
                     lambda: g.process_parallel_arrays(bases[:1000], np.array([0, 1000], np.uint64))):
            try:
                call()
            except NeuroKmerError as e:
                assert e.code == NK_E_UNSUPPORTED, e
            else:
                raise AssertionError("a whole-pool call on sharded state did not refuse")
        g.reset()
        g.process_parallel_arrays(bases, offs)
        r2 = cbind.OracleCounter(k, 1.0, 0.95, 2, 1.0, pool, True, width=width)
        r2.process_parallel_arrays(bases, offs, 4)
        _check_same(g, r2)
        return
    if name == "exact_table":
        k, pool = 25, 7001
        bases, offs = _input(600_000, 63)
        d_b, d_o = dev_input(bases, offs)
        g = SpikingKmerCounter(k, 1.0, 0.95, 2, 1.0, pool, True, exact_counts=True)
        r = cbind.OracleCounter(k, 1.0, 0.95, 2, 1.0, pool, True)
        r.process_parallel_arrays(bases, offs, 4)
        g.accumulate_device(d_b.data_ptr(), d_o.data_ptr(), offs.size - 1, bases.size)
        nkdist.exchange_exact_table(g)
        nkdist.finalize_step(g, total_kmers=int(offs[-1]), comm=comm)
        torch.cuda.synchronize()
        _check_same(g, r)
        np.testing.assert_array_equal(g.kmer_per_neuron(), r.kmer_per_neuron())
        assert g.distinct_kmers() == r.distinct_kmers()
        keys = np.unique(cbind.kmer_keys(bases[int(offs[0]):int(offs[1])].tobytes(), k, True))
        keys = np.concatenate([keys[::13], np.array([5, 2**47 + 3], np.uint64)])
        cnt, pres = nkdist.get_counts(g, keys)
        for kk, c, p in zip(keys, cnt, pres):
            assert (int(c) if p else None) == r.get_count(int(kk)), kk
        return
    raise ValueError(name)


def _worker(port, name, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        _case(name)
        q.put((name, ""))
    except Exception:
        q.put((name, traceback.format_exc()))
    finally:
        dist.destroy_process_group()


CASES = ["finalize_step_u32", "finalize_step_u64", "sliced_64", "sliced_128", "exact_table"]


@pytest.mark.parametrize("name", CASES + [c + "+comm" for c in CASES])
def test_one_rank_rccl(name):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(_free_port(), name, q))
    p.start()
    got, err = q.get(timeout=300)
    p.join(timeout=60)
    assert got == name
    assert not err, err
    assert p.exitcode == 0
