"""CPU multi-process test (gloo, world_size 2) of the multi-GPU protocol in
neurokmer_amd/dist.py: shard the records (with in-record splits + k-1 halo),
accumulate per shard, all-reduce the u64 currents, LIF/top-N on the sum, and
union the shards' distinct top-N k-mers.  The per-shard work is done by the C
oracle here (no GPU); on the GPU box the same protocol drives the HIP path
(bench.py, tests/test_gpu_parity.py::test_split_phase_two_shards_equals_whole).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from neurokmer_amd import dist as nkdist
from neurokmer_amd import synth


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, k, pool, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import cbind
        bases, offs = synth.make_records(90_000, 3, seed=7, repeats_per_mb=30000, motif_len=50,
                                         n_rate=0.002)
        lo, hi, soffs, _ = nkdist.shard_records(offs, world, k)[rank]
        shard = bases[lo:hi]
        ctr = cbind.OracleCounter(k, 1.0, 0.95, 2, 1.0, pool, True)
        ctr.process_parallel_arrays(shard, soffs, 1)
        cur = torch.from_numpy(ctr.currents().view(np.int64).copy())
        cur32 = cur.clone()
        nkdist.allreduce_currents_(cur)
        nkdist.allreduce_currents_(cur32, total_kmers=int(offs[-1]))  # int32 on the wire
        assert torch.equal(cur, cur32)
        # identical LIF + top-N on every rank: reuse the oracle on the summed
        # currents by comparing against a whole-input run below
        whole = cbind.OracleCounter(k, 1.0, 0.95, 2, 1.0, pool, True)
        whole.process_parallel_arrays(bases, offs, 1)
        ok_cur = np.array_equal(cur.numpy().view(np.uint64), whole.currents())
        top = whole.top_abundant_neurons(20)
        top_idx = {t[0] for t in top}
        # this shard's distinct keys of the top neurons
        mine = set()
        for i in range(soffs.size - 1):
            rec = shard[int(soffs[i]):int(soffs[i + 1])].tobytes()
            for key in cbind.kmer_keys(rec, k, True):
                if int(cbind.lib().nko_map_kmer(int(key), pool)) in top_idx:
                    mine.add(int(key))
        t = torch.tensor(sorted(mine), dtype=torch.int64)
        allk = nkdist.gather_union(t)
        per = {}
        for key in set(allk.tolist()):
            n = int(cbind.lib().nko_map_kmer(key & (2**64 - 1), pool))
            per[n] = per.get(n, 0) + 1
        ok_uniq = all(per.get(i, 0) == u for i, _, u in top)
        q.put((rank, ok_cur, ok_uniq, int(hi - lo)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("k,pool", [(21, 5003), (31, 777)])
def test_gloo_two_ranks_match_whole_input(k, pool):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, k, pool, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, ok_cur, ok_uniq, nbytes in res:
        assert ok_cur, f"rank {rank}: all-reduced currents differ from the whole input"
        assert ok_uniq, f"rank {rank}: union of shard top k-mers differs"
        assert nbytes > 0


@pytest.mark.parametrize("world", [1, 2, 3, 8])
@pytest.mark.parametrize("k,canon", [(5, False), (31, True), (40, False), (40, True),
                                     (63, True), (96, True)])
def test_shard_records_cover_every_window_once(world, k, canon):
    """Every window's key is counted by exactly one shard — for k > 32 canonical
    (the reference's release-build keys, which depend on the record start for
    a record's first 32 windows) through the 32-base warm-up of a cut inside a
    record (the shard skips the windows that start in it)."""
    from oracle import cbind
    bases, offs = synth.make_records(20_000, 3, seed=world * 100 + k, n_rate=0.01)
    want = []
    for i in range(offs.size - 1):
        want += [int(x) for x in cbind.kmer_keys(bases[int(offs[i]):int(offs[i + 1])].tobytes(),
                                                 k, canon)]
    got = []
    splits = 0
    for lo, hi, so, skip in nkdist.shard_records(offs, world, k, canonical=canon):
        sh = bases[lo:hi]
        splits += skip > 0
        for i in range(so.size - 1):
            ks = [int(x) for x in cbind.kmer_keys(sh[int(so[i]):int(so[i + 1])].tobytes(), k,
                                                  canon)]
            got += ks[skip:] if i == 0 else ks  # windows starting before skip: context
    assert sorted(got) == sorted(want)
    if k > 32 and canon and world >= 2:
        assert splits > 0  # records were cut inside, not snapped to their starts


def test_exact_table_partition_protocol():
    """§8f-1 across ranks, the arithmetic of the protocol on the C restatement:
    per-shard (key, count) tables, partitioned by exact_owner, merged on the
    owners = the whole input's table; the owners' per-neuron distinct counts
    add up to the whole input's kmer_per_neuron."""
    from oracle import cbind
    k, pool, world = 19, 4001, 3
    bases, offs = synth.make_records(60_000, 5, seed=9, repeats_per_mb=20000, motif_len=40,
                                     n_rate=0.003)

    def table(b, o):
        d = {}
        for i in range(o.size - 1):
            for key in cbind.kmer_keys(b[int(o[i]):int(o[i + 1])].tobytes(), k, True):
                d[int(key)] = d.get(int(key), 0) + 1
        return d

    whole = table(bases, offs)
    owned = [dict() for _ in range(world)]
    for lo, hi, so, _ in nkdist.shard_records(offs, world, k):
        t = table(bases[lo:hi], so)
        keys = np.array(sorted(t), dtype=np.uint64)
        for key, r in zip(keys.tolist(), nkdist.exact_owner(keys, world).tolist()):
            owned[r][key] = owned[r].get(key, 0) + t[key]
    merged = {}
    for r in range(world):
        assert not set(merged) & set(owned[r])  # each key has one owner
        merged.update(owned[r])
    assert merged == whole
    kpn = np.zeros(pool, np.int64)
    for r in range(world):
        for key in owned[r]:
            kpn[int(cbind.lib().nko_map_kmer(key, pool))] += 1
    ref = np.zeros(pool, np.int64)
    for key in whole:
        ref[int(cbind.lib().nko_map_kmer(key, pool))] += 1
    assert np.array_equal(kpn, ref)


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_pool_slices_hold_the_global_top_rows(world):
    """The pool-sliced finish (dist.finalize_step_sliced, nk_adopt_slices): the
    slices [r*S, min(P, (r+1)*S)) tile the pool, and the global top rows
    (spikes desc, index asc; src/spiking_hash.rs:661-673) are the top rows of
    the union of every slice's own top rows — on the C restatement's state."""
    from oracle import cbind
    k, pool, n = 21, 10_007, 20
    bases, offs = synth.make_records(200_000, 4, seed=5, repeats_per_mb=40_000, motif_len=60)
    ref = cbind.OracleCounter(k, 1.0, 0.95, 2, 1.0, pool, True)
    ref.process_parallel_arrays(bases, offs, 1)
    sc = ref.spike_counts()
    covered = np.zeros(pool, np.int64)
    cand = []
    for r in range(world):
        lo, hi, S = nkdist.slice_bounds(pool, world, r)
        assert S == -(-pool // world)
        covered[lo:hi] += 1
        rows = sorted(range(lo, hi), key=lambda i: (-int(sc[i]), i))[:n]
        cand += [(int(sc[i]), i) for i in rows]
    assert (covered == 1).all()
    merged = [i for _, i in sorted(cand, key=lambda t: (-t[0], t[1]))[:n]]
    assert merged == [t[0] for t in ref.top_abundant_neurons(n)]
