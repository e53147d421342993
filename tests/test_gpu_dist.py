"""Multi-process rehearsal of the multi-GPU protocol on the HIP path (two
ranks on the one GPU of the test box, gloo for the collectives): shards,
all-reduce of the currents, the exact table exchanged by hash partition +
all-to-all (neurokmer_amd/dist.py), finalize, routed get_counts -> identical
to the whole input on the C restatement.  The driver's 8-GPU runs use the
same code with RCCL.
"""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


K, POOL = 25, 7001


def _input():
    from neurokmer_amd import synth
    return synth.make_records(400_000, 5, seed=44, repeats_per_mb=20000, motif_len=80,
                              n_rate=0.002)


class _CAI:
    def __init__(self, ptr, n, typestr="<i8"):
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": typestr,
                                         "data": (ptr, False), "version": 3}


def _rank(rank, world, port, keys, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from neurokmer_amd import SpikingKmerCounter
        from neurokmer_amd import dist as nkdist
        bases, offs = _input()
        lo, hi, so, _ = nkdist.shard_records(offs, world, K)[rank]
        b = bases[lo:hi]
        d_b = torch.from_numpy(np.concatenate([b, np.zeros(16, np.uint8)])).cuda()
        d_o = torch.from_numpy(so.astype(np.uint64).view(np.int64)).cuda()
        torch.cuda.synchronize()
        c = SpikingKmerCounter(K, 1.0, 0.95, 2, 1.0, POOL, True, exact_counts=True)
        c.accumulate_device(d_b.data_ptr(), d_o.data_ptr(), so.size - 1, b.size)
        cur = torch.as_tensor(_CAI(c.device_currents_ptr(), POOL), device="cuda")
        nkdist.allreduce_currents_(cur, total_kmers=int(offs[-1]))
        nkdist.exchange_exact_table(c)
        torch.cuda.synchronize()
        c.finalize(False)
        mine = keys[rank::world]
        cnt, pres = nkdist.get_counts(c, mine)
        q.put((rank, c.top_abundant_neurons(20), c.distinct_kmers(), c.energy.total_spikes(),
               mine.tolist(), cnt.tolist(), pres.tolist(), c.kmer_per_neuron().tolist()))
        c.close()
    finally:
        dist.destroy_process_group()


def test_two_ranks_exact_table_and_uniques():
    import torch.multiprocessing as mp
    from oracle import cbind
    bases, offs = _input()
    ref = cbind.OracleCounter(K, 1.0, 0.95, 2, 1.0, POOL, True)
    ref.process_parallel_arrays(bases, offs)
    keys = np.unique(np.concatenate([cbind.kmer_keys(bases[int(offs[i]):int(offs[i + 1])]
                                                     .tobytes(), K, True) for i in range(2)]))
    keys = np.concatenate([keys[::97], np.array([3, 2**45 + 11], np.uint64)])
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, 2, port, keys, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    top = ref.top_abundant_neurons(20)
    kpn = ref.kmer_per_neuron().tolist()
    for rank, t, _, spikes, mine, cnt, pres, kp in res:
        assert t == top
        assert spikes == ref.total_spikes
        assert kp == kpn
        exp = [ref.get_count(int(x)) for x in mine]
        assert pres == [x is not None for x in exp]
        assert [c for c, p in zip(cnt, pres) if p] == [x for x in exp if x is not None]
    assert sum(r[2] for r in res) == ref.distinct_kmers()


def _rank_union(rank, world, port, width, cap, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from neurokmer_amd import SpikingKmerCounter
        from neurokmer_amd import dist as nkdist
        bases, offs = _input()
        k = 41 if width == 128 else K
        lo, hi, so, skip = nkdist.shard_records(offs, world, k, kmer_width=width)[rank]
        b = bases[lo:hi]
        d_b = torch.from_numpy(np.concatenate([b, np.zeros(16, np.uint8)])).cuda()
        d_o = torch.from_numpy(so.astype(np.uint64).view(np.int64)).cuda()
        torch.cuda.synchronize()
        c = SpikingKmerCounter(k, 1.0, 0.95, 2, 1.0, POOL, True, kmer_width=width)
        c.accumulate_device_from(d_b.data_ptr(), d_o.data_ptr(), so.size - 1, b.size, skip)
        cur = torch.as_tensor(_CAI(c.device_currents_ptr(), POOL), device="cuda")
        nkdist.allreduce_currents_(cur)
        c.finalize(False)
        nkdist.union_top_kmers(c, cap=cap)
        q.put((rank, c.top_abundant_neurons(20)))
        c.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("width,cap", [(64, 4096), (64, 3), (128, 4096), (128, 3)])
def test_two_ranks_union_of_top_kmers(width, cap):
    # cap 3: some shard holds more keys -> every rank takes the variable-length path
    import torch.multiprocessing as mp
    from oracle import cbind
    bases, offs = _input()
    k = 41 if width == 128 else K
    ref = cbind.OracleCounter(k, 1.0, 0.95, 2, 1.0, POOL, True, width=width)
    ref.process_parallel_arrays(bases, offs)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_union, args=(r, 2, port, width, cap, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    top = ref.top_abundant_neurons(20)
    for _, t in res:
        assert t == top


SKEW_POOL = 200_003  # 7 buckets of 32768 neurons: the poly-A bucket overflows its region


def _skewed_input():
    """_input plus a 300 kb poly-A record: one neuron takes ~300 k k-mers, more
    than its bucket region holds (the partitioned count's direct-add overflow)."""
    bases, offs = _input()
    tail = np.full(300_000, ord("A"), np.uint8)
    return (np.concatenate([bases, tail]),
            np.concatenate([offs, [offs[-1] + tail.size]]).astype(np.uint64))


def _rank_step(rank, world, port, width, cap, steps, wire, q, skew=False):
    """dist.finalize_step (one host synchronisation per step), twice with a
    reset in between, then once more on the kept state."""
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from neurokmer_amd import SpikingKmerCounter
        from neurokmer_amd import dist as nkdist
        bases, offs = _skewed_input() if skew else _input()
        k = 41 if width == 128 else K
        lo, hi, so, skip = nkdist.shard_records(offs, world, k, kmer_width=width)[rank]
        b = bases[lo:hi]
        d_b = torch.from_numpy(np.concatenate([b, np.zeros(16, np.uint8)])).cuda()
        d_o = torch.from_numpy(so.astype(np.uint64).view(np.int64)).cuda()
        torch.cuda.synchronize()
        pool = SKEW_POOL if skew else POOL
        c = SpikingKmerCounter(k, 1.0, 0.95, 2, 1.0, pool, True, kmer_width=width)
        c.set_steps(steps)
        out = []
        for it in range(3):
            if it == 1:
                c.reset()
            c.accumulate_device_from(d_b.data_ptr(), d_o.data_ptr(), so.size - 1, b.size, skip)
            nkdist.finalize_step(c, total_kmers=int(offs[-1]) if wire else None, cap=cap)
            out.append((c.top_abundant_neurons(20), c.energy.total_spikes()))
        q.put((rank, out, c.currents().tolist(), c.spike_counts().tolist()))
        c.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("width,cap,steps,wire,skew", [
    (64, 4096, 1000, True, False),    # the fast path: u32 wire, exact export, one wait
    (64, 4096, 1000, False, False),   # u64 all-reduce of the currents
    (64, 3, 1000, True, False),       # truncated segments: every rank redoes, variable-length union
    (64, 4096, 20000, True, False),   # spike counts past the histogram: host refine on every rank
    (64, 4096, 1000, True, True),     # an overflowed bucket region (direct adds into the currents)
    (128, 4096, 1000, True, False),
    (128, 2, 1000, True, False),
])
def test_two_ranks_finalize_step(width, cap, steps, wire, skew):
    import torch.multiprocessing as mp
    from oracle import cbind
    bases, offs = _skewed_input() if skew else _input()
    k = 41 if width == 128 else K
    pool = SKEW_POOL if skew else POOL
    ref = cbind.OracleCounter(k, 1.0, 0.95, 2, 1.0, pool, True, width=width)
    ref.set_steps(steps)
    exp = []
    for it in range(3):
        if it == 1:
            ref = cbind.OracleCounter(k, 1.0, 0.95, 2, 1.0, pool, True, width=width)
            ref.set_steps(steps)
        ref.process_parallel_arrays(bases, offs)
        exp.append((ref.top_abundant_neurons(20), ref.total_spikes))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_step, args=(r, 2, port, width, cap, steps, wire, q, skew))
             for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for _, out, cur, sc in res:
        assert out == exp
        assert cur == ref.currents().tolist()
        assert sc == ref.spike_counts().tolist()


# ---- config 4 shape: k=31, pool 2M, byte-range shards that split records -----
C4_K, C4_POOL = 31, 2_000_000


def _config4_input():
    """3 long records (2.4 Mbases), planted repeats: 2 ranks cut the middle
    record, so one window range is counted across a k-1 base halo."""
    from neurokmer_amd import synth
    return synth.make_records(2_400_000, 3, seed=404, repeats_per_mb=300, motif_len=150,
                              n_rate=0.001)


def _rank_config4(rank, world, port, exact, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from neurokmer_amd import SpikingKmerCounter
        from neurokmer_amd import dist as nkdist
        bases, offs = _config4_input()
        lo, hi, so, _ = nkdist.shard_records(offs, world, C4_K)[rank]
        b = bases[lo:hi]
        d_b = torch.from_numpy(np.concatenate([b, np.zeros(16, np.uint8)])).cuda()
        d_o = torch.from_numpy(so.astype(np.uint64).view(np.int64)).cuda()
        torch.cuda.synchronize()
        c = SpikingKmerCounter(C4_K, 1.0, 0.95, 2, 1.0, C4_POOL, True, exact_counts=exact)
        c.accumulate_device(d_b.data_ptr(), d_o.data_ptr(), so.size - 1, b.size)
        if exact:
            nkdist.exchange_exact_table(c)
        # no manual synchronisation: finalize_step orders the LIF after the
        # all-reduce on the caller's stream (exact branch included)
        nkdist.finalize_step(c, total_kmers=int(offs[-1]))
        q.put((rank, (lo, hi, so.tolist()), c.currents().tolist(), c.spike_counts().tolist(),
               c.top_abundant_neurons(20), c.energy.total_spikes(),
               c.kmer_per_neuron().tolist() if exact else None))
        c.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("exact", [False, True])
def test_two_ranks_config4_split_records(exact):
    import torch.multiprocessing as mp
    from oracle import cbind
    from neurokmer_amd import dist as nkdist
    bases, offs = _config4_input()
    shards = nkdist.shard_records(offs, 2, C4_K)
    # the cut falls inside record 1: both shards hold part of it (+ halo)
    assert shards[0][1] > shards[1][0] and len(shards[0][2]) == 3 and len(shards[1][2]) == 3
    ref = cbind.OracleCounter(C4_K, 1.0, 0.95, 2, 1.0, C4_POOL, True)
    ref.process_parallel_arrays(bases, offs, 3)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_config4, args=(r, 2, port, exact, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    cur = ref.currents().tolist()
    sc = ref.spike_counts().tolist()
    top = ref.top_abundant_neurons(20)
    assert ref.total_spikes > 0
    for _, _, c, s, t, tot, kpn in res:
        assert c == cur
        assert s == sc
        assert t == top
        assert tot == ref.total_spikes
        if exact:
            assert kpn == ref.kmer_per_neuron().tolist()
