"""Config-5 shape across ranks: records of a
k > 32 input split inside (32-base warm-up for the reference's release-build
keys, k-1 halo for 128-bit keys) and the pool-sliced finish
(dist.finalize_step_sliced: reduce-scatter of the currents, LIF + top rows of
each rank's 1/world of the pool, all-gather of the slices' rows, union of the
shards' top keys).  Two processes share the test box's GPU over gloo; every
output is compared bit-exactly with oracle/nk_oracle.c on the whole input.

Reference: src/spiking_hash.rs:49-53,97 (the pool), :84-201 (process_parallel),
:661-673 (top rows); src/models.rs:260-266 (k > 32 reverse strand).
"""
import hashlib
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


def _input(total, seed):
    from neurokmer_amd import synth
    return synth.make_records(total, 3, seed=seed, repeats_per_mb=20_000, motif_len=110,
                              n_rate=0.002, mixed_case=True)


def _digest(a: np.ndarray) -> str:
    return hashlib.sha1(np.ascontiguousarray(a).view(np.uint8)).hexdigest()


def _rank(rank, world, port, k, pool, width, canon, total, seed, sliced, small, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from neurokmer_amd import SpikingKmerCounter
        from neurokmer_amd import dist as nkdist
        bases, offs = _input(total, seed)
        lo, hi, so, skip = nkdist.shard_records(offs, world, k, kmer_width=width,
                                                canonical=canon)[rank]
        b = bases[lo:hi]
        d_b = torch.from_numpy(np.concatenate([b, np.zeros(16, np.uint8)])).cuda()
        d_o = torch.from_numpy(so.astype(np.uint64).view(np.int64)).cuda()
        torch.cuda.synchronize()
        c = SpikingKmerCounter(k, 1.0, 0.95, 2, 1.0, pool, canon, kmer_width=width)
        tk = int(offs[-1]) if small else None  # None: the u64 wire
        for _ in range(2):  # state carries over between steps (no reset)
            c.accumulate_device_from(d_b.data_ptr(), d_o.data_ptr(), so.size - 1, b.size, skip)
            if sliced:
                nkdist.finalize_step_sliced(c, total_kmers=tk)
            else:
                nkdist.finalize_step(c, total_kmers=tk)
        torch.cuda.synchronize()
        st = nkdist.gather_state(c) if sliced else {
            "currents": c.currents(), "spike_counts": c.spike_counts(),
            "voltages": c.voltages(), "refractory": c.refractory()}
        q.put((rank, skip, c.top_abundant_neurons(20), c.energy.total_spikes(), c.energy_used(),
               {n: _digest(a) for n, a in st.items()}))
        c.close()
    finally:
        dist.destroy_process_group()


CASES = [
    # k, pool, width, canonical, bases, sliced, u32 wire
    (63, 1 << 26, 64, True, 1_500_000, True, True),     # config-5 shape, compat keys
    (63, (1 << 26) + 3, 128, True, 1_500_000, True, False),  # 128-bit keys, u64 wire
    (40, 50_021, 64, True, 600_000, True, False),
    (31, 7_001, 64, True, 600_000, True, True),
    (33, 20_011, 64, False, 600_000, True, True),
    (63, 100_003, 64, True, 600_000, False, True),      # warm-up shards, plain finish
]


@pytest.mark.parametrize("k,pool,width,canon,total,sliced,small", CASES)
def test_two_ranks_sliced_pool(k, pool, width, canon, total, sliced, small):
    import torch.multiprocessing as mp
    from oracle import cbind
    seed = k * 7 + pool % 97
    bases, offs = _input(total, seed)
    ref = cbind.OracleCounter(k, 1.0, 0.95, 2, 1.0, pool, canon, width=width)
    for _ in range(2):
        ref.process_parallel_arrays(bases, offs, 3)
    want = {"currents": _digest(ref.currents()), "spike_counts": _digest(ref.spike_counts()),
            "voltages": _digest(ref.voltages()), "refractory": _digest(ref.refractory())}
    top = ref.top_abundant_neurons(20)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, 2, port, k, pool, width, canon, total, seed,
                                             sliced, small, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=600) for _ in procs)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    if k > 32 and width == 64 and canon:
        assert res[1][1] == 32  # rank 1's shard starts inside a record, after a warm-up
    for rank, skip, t, spikes, energy, dig in res:
        assert t == top, rank
        assert spikes == ref.total_spikes
        assert energy == ref.energy_used()
        assert dig == want, rank
