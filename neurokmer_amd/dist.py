"""Multi-GPU data parallelism for the k-mer -> spike path (one process per GPU).

The path shards naturally: a k-mer's neuron depends only on
its window (k <= 32), and currents are a commutative u64 sum.  So:
  * every rank accumulates the currents of its own shard of the input
    (nk_accumulate_device) — no communication on the data path;
  * one exchange: all-reduce of the u64 currents vector (RCCL over xGMI with
    backend "nccl"; gloo on CPU in tests);
  * every rank then runs the identical LIF + top-N on the reduced currents;
  * "unique k-mers colliding" needs the UNION of the shards' distinct k-mers
    of the top-N neurons: each rank contributes its (small) distinct key list,
    all-gathered and merged (nk_merge_top_kmers).

With the exact k-mer table (nk_opts.exact_counts) the
shards' tables are combined by hash partition + all-to-all
(exchange_exact_table): every distinct key goes to one owner rank
(exact_owner), owners merge the counts, and the per-rank kmer_per_neuron
contributions are all-reduced; get_counts() routes queries to the owners.

shard_records() splits one input into world shards at record boundaries and,
where a record is longer than a shard, inside the record with a k-1 base halo,
so every window is counted by exactly one rank.  k > 32 canonical keys of the
reference's release build (NK_KMER_COMPAT) depend on the record start for the
first 32 windows of a record only (the rolling reverse strand's init residue,
src/models.rs:260-266): a cut at least 32 bases into a record keeps a 32-base
warm-up before it whose windows the shard does not count (`skip`, passed to
accumulate_device_from); a cut closer to the record start moves to it.  The
128-bit keys and non-canonical pack_kmer keys are pure functions of the window:
the k-1 halo alone suffices.

For very large pools (config 5) finalize_step_sliced() replaces the all-reduce
of the whole currents vector by a reduce-scatter: each rank runs the LIF and
the top-N selection on its 1/world slice of the pool only, the slices' top
rows are all-gathered (nk_finalize_slice / nk_adopt_slices).
"""
from __future__ import annotations

from typing import List, Tuple

import numpy as np


WARMUP = 32  # bases of context before a cut inside a k > 32 compat record


def shard_records(offsets: np.ndarray, world: int, k: int, kmer_width: int = 64,
                  canonical: bool = True) -> List[Tuple[int, int, np.ndarray, int]]:
    """-> per rank (byte_lo, byte_hi, shard_offsets, skip) with shard_offsets
    relative to byte_lo; the shard counts the windows that start at >= skip
    (accumulate_device_from).  The k-mer start positions of the input are split
    into world contiguous ranges of (nearly) equal size."""
    offsets = np.asarray(offsets, dtype=np.int64)
    n = int(offsets[-1])
    if world <= 1 or n == 0:
        return [(0, n, offsets.astype(np.uint64), 0)] + \
            [(n, n, np.zeros(1, np.uint64), 0)] * (world - 1)
    warm = WARMUP if (k > 32 and kmer_width == 64 and canonical) else 0
    cuts = [n * r // world for r in range(world + 1)]
    if warm:  # a cut within the first `warm` bases of a record moves to its start
        for r in range(1, world):
            c = cuts[r]
            s0 = int(offsets[np.searchsorted(offsets, c, side="right") - 1])
            if c - s0 < warm:
                cuts[r] = s0
        cuts = [max(cuts[:i + 1]) for i in range(world + 1)]  # monotone
    out = []
    for r in range(world):
        lo, hi = cuts[r], cuts[r + 1]
        if hi <= lo:
            out.append((lo, lo, np.zeros(1, np.uint64), 0))
            continue
        # records overlapping [lo, hi): starts in [lo, hi), the record holding lo
        i0 = int(np.searchsorted(offsets, lo, side="right")) - 1
        skip = warm if (warm and lo > int(offsets[i0])) else 0
        ends = []
        j = i0
        while j < offsets.size - 1 and offsets[j] < hi:
            e = int(offsets[j + 1])
            if e > hi:  # record continues past the cut: keep k-1 halo bases
                e = min(e, hi + k - 1)
            ends.append(e)
            j += 1
        b_lo = lo - skip
        rel = np.array([0] + [e - b_lo for e in ends], dtype=np.uint64)
        out.append((b_lo, int(b_lo + rel[-1]), rel, skip))
    return out


def allreduce_currents_(t, group=None, total_kmers=None) -> None:
    """In-place sum of a u64 currents vector held as int64 (same bits mod 2^64).

    total_kmers: an upper bound on the k-mers of ALL ranks together, the same
    on every rank.  Below 2^31 no neuron's summed current can leave int32, so
    the vector crosses xGMI as int32 (half the bytes of the ring all-reduce)."""
    import torch
    import torch.distributed as dist
    if total_kmers is not None and 0 <= total_kmers < (1 << 31):
        n = t.to(torch.int32)
        dist.all_reduce(n, op=dist.ReduceOp.SUM, group=group)
        t.copy_(n)
        return
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)


class Comm:
    """The library's own communicator for this rank (RCCL over xGMI;
    include/neurokmer.h nk_comm_*): rank 0 of `group` makes the id, the group
    broadcasts it, every rank builds its communicator (collective).  With one,
    finalize_step / finalize_step_sliced run the whole finish inside the
    library (nk_finalize_dist / nk_finalize_sliced_dist): the collectives are
    enqueued between the library's kernels with no Python in between."""

    def __init__(self, group=None, device: int | None = None):
        import ctypes as C

        import torch
        import torch.distributed as dist
        from . import _lib
        self._L = _lib.load()
        self._h = None
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.device = torch.cuda.current_device() if device is None else device
        idb = (C.c_uint8 * 128)()
        if self.rank == 0:
            _lib.check(self._L.nk_comm_unique_id(idb))
        obj = [bytes(idb)]
        src = 0 if group is None else dist.get_global_rank(group, 0)
        dist.broadcast_object_list(obj, src=src, group=group)
        idb = (C.c_uint8 * 128).from_buffer_copy(obj[0])
        h = self._L.nk_comm_new(idb, self.world, self.rank, self.device)
        if not h:
            raise _lib.NeuroKmerError(_lib.NK_E_DEVICE, _lib.last_error())
        self._h = h

    @classmethod
    def loopback(cls, group: "LoopbackGroup", rank: int, device: int = 0) -> "Comm":
        """Rank `rank` of an in-process loopback group (nk_comm_new_loopback):
        the ranks are host threads of this process on one device, the
        collectives device copies between host barriers.  A rehearsal of the
        multi-rank finish on one GPU, where RCCL refuses two ranks."""
        from . import _lib
        self = cls.__new__(cls)
        self._L = _lib.load()
        self._h = None
        self.world, self.rank, self.device = group.world, rank, device
        h = self._L.nk_comm_new_loopback(group._h, rank, device)
        if not h:
            raise _lib.NeuroKmerError(_lib.NK_E_INVALID, _lib.last_error())
        self._h = h
        return self

    def forget(self, ctr) -> None:
        """Free the device buffers this communicator holds for `ctr`
        (nk_comm_forget); call before closing a handle the comm outlives."""
        if self._h and getattr(ctr, "_h", None):
            self._L.nk_comm_forget(self._h, ctr._h)

    def close(self):
        if self._h:
            self._L.nk_comm_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class LoopbackGroup:
    """A loopback transport group of `world` ranks (nk_loop_group_new): each
    rank is a host thread of this process with its own Comm.loopback(...).
    Free it after every member Comm is closed."""

    def __init__(self, world: int):
        from . import _lib
        self._L = _lib.load()
        self.world = world
        self._h = self._L.nk_loop_group_new(world)
        if not self._h:
            raise _lib.NeuroKmerError(_lib.NK_E_INVALID, _lib.last_error())

    def close(self):
        if self._h:
            self._L.nk_loop_group_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


_U64_MAX = (1 << 64) - 1


def _comm_finish(ctr, comm, fn, total_kmers, cap, streaming):
    import torch
    from ._lib import check
    stream = torch.cuda.current_stream().cuda_stream
    if stream == 0:
        _on_side_stream(ctr, lambda: _comm_finish(ctr, comm, fn, total_kmers, cap, streaming))
        return
    tk = _U64_MAX if total_kmers is None or total_kmers < 0 else int(total_kmers)
    check(getattr(comm._L, fn)(ctr._h, comm._h, 1 if streaming else 0, tk, cap, stream))


def finalize_step(ctr, group=None, total_kmers=None, cap: int = 4096,
                  streaming: bool = False, between=None, comm: "Comm | None" = None) -> None:
    """After every rank's ctr.accumulate_device: the whole multi-GPU finish with
    ONE host synchronisation (include/neurokmer.h, nk_finalize_export):

      wire = this shard's currents as u32   (nk_wire32; u64 all-reduce when
                                             total_kmers is unknown or >= 2^31)
      all-reduce(wire)                      RCCL over xGMI
      LIF + top-N + uniques of this shard, its distinct top k-mers into a
      fixed-size segment                    (nk_finalize_export, enqueued)
      all-gather(segments)
      union -> uniques column, one readback (nk_merge_export)

    If any rank could not export exactly (the segment headers carry the
    reasons, so every rank decides alike) all ranks redo the slow way:
    nk_finalize_redo + union_top_kmers.  With the exact k-mer table the
    uniques come from kmer_per_neuron: plain finalize.

    between: called once the currents' all-reduce is enqueued, before the rest
    (a caller keeping batches in flight enqueues the next batch's count there:
    on another handle it starts when this all-reduce is done and runs beside
    this batch's finish; bench.py --inflight 2).

    comm: the library's communicator (Comm): the same protocol, all of it
    enqueued by one library call (nk_finalize_dist); `between` then runs
    before it."""
    import torch
    import torch.distributed as dist
    if comm is not None:
        if between is not None:
            between()
        _comm_finish(ctr, comm, "nk_finalize_dist", total_kmers, cap, streaming)
        return
    if torch.cuda.current_stream().cuda_stream == 0:
        # the library reads a NULL stream as its own stream: run the step on a
        # real torch stream so the collectives and our kernels share one order
        _on_side_stream(ctr, lambda: finalize_step(ctr, group, total_kmers, cap, streaming,
                                                   between))
        return
    stream = torch.cuda.current_stream().cuda_stream
    if getattr(ctr, "exact_counts", False):  # (after exchange_exact_table)
        cur = _currents_view(ctr, torch.device("cuda", torch.cuda.current_device()))
        allreduce_currents_(cur, group=group, total_kmers=total_kmers)
        if between is not None:
            between()
        # the LIF must run after the all-reduce on the SAME stream: the
        # library's own stream would not wait for torch's collective
        ctr.finalize(streaming, stream)
        return
    world = dist.get_world_size(group)
    dev = torch.device("cuda", torch.cuda.current_device())
    bufs = ctr.__dict__.setdefault("_dist_bufs", {})
    pool = ctr.pool_size
    wire_ptr = 0
    if total_kmers is not None and 0 <= total_kmers < (1 << 31):
        wire = bufs.get("wire")
        if wire is None or wire.numel() != max(pool, 1) or wire.device != dev:
            wire = bufs["wire"] = torch.empty(max(pool, 1), dtype=torch.int32, device=dev)
        ctr.wire32(wire.data_ptr(), stream)
        if pool:
            dist.all_reduce(wire[:pool], op=dist.ReduceOp.SUM, group=group)
        wire_ptr = wire.data_ptr()
    else:
        cur = _currents_view(ctr, dev)
        allreduce_currents_(cur, group=group)
    if between is not None:
        between()
    wpk = 2 if getattr(ctr, "kmer_width", 64) == 128 else 1
    stride = 1 + wpk * cap
    key = ("seg", world, stride)
    if key not in bufs:
        bufs[key] = (torch.empty(stride, dtype=torch.int64, device=dev),
                     torch.empty(world * stride, dtype=torch.int64, device=dev))
    seg, allb = bufs[key]
    ctr.finalize_export(wire_ptr, seg.data_ptr(), cap, streaming, stream)
    _all_gather_into(allb, seg, group=group)
    if ctr.merge_export(allb.data_ptr(), world, stride, cap, stream):
        ctr.finalize_redo(stream)
        union_top_kmers(ctr, group=group, cap=cap)


def slice_bounds(pool: int, world: int, rank: int) -> Tuple[int, int, int]:
    """-> (lo, hi, S): rank's neurons [lo, hi) of the pool-sliced finish, S =
    ceil(pool / world) entries per slice (the last slice may be short)."""
    S = -(-pool // world) if pool else 0
    lo = min(pool, rank * S)
    return lo, min(pool, lo + S), S


def finalize_step_sliced(ctr, group=None, total_kmers=None, cap: int = 4096,
                         streaming: bool = False, comm: "Comm | None" = None) -> None:
    """After every rank's accumulate: the finish for very large pools
    (SURVEY.md §5/§8e, config 5).  Instead of all-reducing the whole currents
    vector and running the LIF of the whole pool on every rank:

      wire (u32, or u64 when total_kmers is unknown or >= 2^31), zero-padded to
      world * S entries
      reduce-scatter(wire) -> this rank's S summed entries    RCCL over xGMI
      LIF + top rows of neurons [lo, hi) only                  (nk_finalize_slice)
      all-gather of the slices' top rows (3 + 3*N words each)
      global top rows, total spikes, this shard's uniques     (nk_adopt_slices)
      union of the shards' top keys                            (union_top_kmers)

    Afterwards a rank's neuron state is authoritative on its slice only
    (gather_state assembles the whole pool).  comm: all of it inside the
    library (nk_finalize_sliced_dist)."""
    import torch
    import torch.distributed as dist
    if comm is not None:
        _comm_finish(ctr, comm, "nk_finalize_sliced_dist", total_kmers, cap, streaming)
        return
    if torch.cuda.current_stream().cuda_stream == 0:
        _on_side_stream(ctr, lambda: finalize_step_sliced(ctr, group, total_kmers, cap, streaming))
        return
    stream = torch.cuda.current_stream().cuda_stream
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = torch.device("cuda", torch.cuda.current_device())
    pool = ctr.pool_size
    lo, hi, S = slice_bounds(pool, world, rank)
    bufs = ctr.__dict__.setdefault("_dist_bufs", {})
    small = total_kmers is not None and 0 <= total_kmers < (1 << 31)
    dt = torch.int32 if small else torch.int64
    key = ("slice", world, S, small)
    if key not in bufs:  # the padding past the pool stays zero
        bufs[key] = (torch.zeros(max(world * S, 1), dtype=dt, device=dev),
                     torch.empty(max(S, 1), dtype=dt, device=dev))
    wire, part = bufs[key]
    if small:
        ctr.wire32(wire.data_ptr(), stream)
    elif pool:
        wire[:pool].copy_(_currents_view(ctr, dev))
    if S:
        _reduce_scatter(part[:S], wire[:world * S], group=group)
    rows = min(ctr.top_n, pool)
    stride = 3 + 3 * rows
    skey = ("sseg", world, stride)
    if skey not in bufs:
        bufs[skey] = (torch.zeros(stride, dtype=torch.int64, device=dev),
                      torch.zeros(world * stride, dtype=torch.int64, device=dev))
    seg, allseg = bufs[skey]
    ctr.finalize_slice(part.data_ptr(), 32 if small else 64, lo, hi, seg.data_ptr(), rows,
                       streaming, stream)
    _all_gather_into(allseg, seg, group=group)
    ctr.adopt_slices(allseg.data_ptr(), world, stride, stream)
    union_top_kmers(ctr, group=group, cap=cap)


def _reduce_scatter(out, inp, group=None):
    """reduce_scatter_tensor (sum); gloo (CPU rehearsals) has none: the same
    result through an all-reduce in host memory."""
    import torch.distributed as dist
    if dist.get_backend(group) == "gloo":
        full = inp.cpu()
        dist.all_reduce(full, op=dist.ReduceOp.SUM, group=group)
        r, n = dist.get_rank(group), out.numel()
        out.copy_(full[r * n:(r + 1) * n])
        return
    dist.reduce_scatter_tensor(out, inp, op=dist.ReduceOp.SUM, group=group)


def gather_state(ctr, group=None) -> dict:
    """After finalize_step_sliced: the whole pool's state assembled from every
    rank's slice (host arrays; collective)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    pool = ctr.pool_size
    lo, hi, S = slice_bounds(pool, world, rank)
    out = {}
    for name, arr in (("currents", ctr.currents()), ("spike_counts", ctr.spike_counts()),
                      ("voltages", ctr.voltages()), ("refractory", ctr.refractory())):
        a64 = np.zeros(max(S, 1), np.int64)  # one slot per rank even for an empty pool
        a64[:hi - lo] = arr[lo:hi].view(np.int64) if arr.dtype.itemsize == 8 else \
            arr[lo:hi].view(np.int32).astype(np.int64)
        t = torch.from_numpy(a64)
        allt = torch.zeros(max(world * S, world), dtype=torch.int64)
        _all_gather_host(allt, t, group)
        full = allt.numpy()[:pool]
        out[name] = full.view(arr.dtype) if arr.dtype.itemsize == 8 else \
            full.astype(np.int32).view(arr.dtype)
    return out


def _all_gather_host(out, inp, group=None):
    """all_gather_into_tensor of host tensors (through the device for RCCL)."""
    import torch
    import torch.distributed as dist
    if dist.get_backend(group) == "gloo":
        dist.all_gather_into_tensor(out, inp, group=group)
        return
    dev = torch.device("cuda", torch.cuda.current_device())
    o = out.to(dev)
    dist.all_gather_into_tensor(o, inp.to(dev), group=group)
    out.copy_(o.cpu())


def _on_side_stream(ctr, fn):
    """Run fn with a cached non-default torch stream current (ordered after the
    caller's stream, and the caller's after it)."""
    import torch
    bufs = ctr.__dict__.setdefault("_dist_bufs", {})
    side = bufs.get("side")
    if side is None:
        side = bufs["side"] = torch.cuda.Stream()
    cur = torch.cuda.current_stream()
    side.wait_stream(cur)
    with torch.cuda.stream(side):
        fn()
    cur.wait_stream(side)


def _all_gather_into(out, inp, group=None):
    """all_gather_into_tensor; with gloo the device tensors go through host memory."""
    import torch.distributed as dist
    if dist.get_backend(group) == "gloo" and out.is_cuda:
        o = out.cpu()
        dist.all_gather_into_tensor(o, inp.cpu(), group=group)
        out.copy_(o)
        return
    dist.all_gather_into_tensor(out, inp, group=group)


def union_top_kmers(ctr, group=None, cap: int = 4096) -> None:
    """After finalize on every rank: the uniques column of the (identical) top
    rows from the union of every shard's distinct top-N k-mers.  One fixed-size
    all-gather of [n, keys...] segments (at most cap keys each) and no host
    round trip before the merge; if some shard has more than cap keys (every
    rank sees the same headers) all ranks fall back to the variable-length
    exchange (gather_union)."""
    import torch
    if torch.cuda.current_stream().cuda_stream == 0:
        _on_side_stream(ctr, lambda: union_top_kmers(ctr, group, cap))
        return
    world = torch.distributed.get_world_size(group)
    dev = torch.device("cuda", torch.cuda.current_device())
    stream = torch.cuda.current_stream().cuda_stream
    wpk = 2 if getattr(ctr, "kmer_width", 64) == 128 else 1
    stride = 1 + wpk * cap
    mine = torch.empty(stride, dtype=torch.int64, device=dev)
    ctr.top_kmers_padded(mine.data_ptr(), cap, stream)
    allb = torch.empty(world * stride, dtype=torch.int64, device=dev)
    _all_gather_into(allb, mine, group=group)
    if ctr.merge_top_kmers_padded(allb.data_ptr(), world, stride, cap, stream):
        return
    ptr, n = ctr.top_kmers_device()
    keys = _dev_view(ptr, n * wpk, "<i8", dev)
    allk = gather_union(keys, group)
    ctr.merge_top_kmers(allk.data_ptr(), allk.numel() // wpk, stream)


def gather_union(keys, group=None):
    """All-gather variable-length int64 key lists -> one concatenated tensor
    (the merge deduplicates).  Two collectives into single tensors and one
    host synchronisation (the sizes)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    n = torch.tensor([keys.numel()], dtype=torch.int64, device=keys.device)
    sizes_t = torch.empty(world, dtype=torch.int64, device=keys.device)
    _all_gather_into(sizes_t, n, group=group)
    sizes = sizes_t.tolist()
    width = max(max(sizes), 1)
    pad = torch.full((width,), -1, dtype=torch.int64, device=keys.device)
    pad[:keys.numel()] = keys
    parts = torch.empty(world * width, dtype=torch.int64, device=keys.device)
    _all_gather_into(parts, pad, group=group)
    return torch.cat([parts[r * width:r * width + s] for r, s in enumerate(sizes)])


class _CAI:
    """Wraps a raw device pointer for torch.as_tensor (no copy)."""

    def __init__(self, ptr: int, n: int, typestr: str):
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": typestr,
                                         "data": (ptr, False), "version": 3}


def _currents_view(ctr, dev):
    """The counter's device currents as an int64 tensor view.  A null pointer
    with a non-empty pool means the library could not materialise them (fold or
    sync error): raise with its error instead of all-reducing nothing."""
    ptr = ctr.device_currents_ptr()
    if not ptr and ctr.pool_size:
        from ._lib import NeuroKmerError, last_error
        raise NeuroKmerError(-7, "device currents unavailable: " + last_error())
    return _dev_view(ptr, ctr.pool_size, "<i8", dev)


def _dev_view(ptr: int, n: int, typestr: str, dev):
    import torch
    if not n or not ptr:
        return torch.empty(0, dtype=torch.int64 if typestr == "<i8" else torch.int32, device=dev)
    return torch.as_tensor(_CAI(ptr, n, typestr), device=dev)


def exact_owner(keys: np.ndarray, world: int) -> np.ndarray:
    """Owner rank of each u64 key (the library's nk_exact_owner: splitmix64
    finaliser, then a multiply-shift into [0, world))."""
    x = np.asarray(keys, dtype=np.uint64) + np.uint64(0x9E3779B97F4A7C15)
    x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    x ^= x >> np.uint64(31)
    return (((x >> np.uint64(32)) * np.uint64(world)) >> np.uint64(32)).astype(np.int64)


def _all_to_all(out, inp, out_splits=None, in_splits=None, group=None):
    """all_to_all_single; with gloo (CPU rehearsals of the multi-GPU path) the
    device tensors are staged through host memory."""
    import torch.distributed as dist
    if dist.get_backend(group) == "gloo" and out.is_cuda:
        o = out.cpu()
        dist.all_to_all_single(o, inp.cpu(), out_splits, in_splits, group=group)
        out.copy_(o)
        return
    dist.all_to_all_single(out, inp, out_splits, in_splits, group=group)


def exchange_exact_table(ctr, group=None) -> None:
    """After every rank's accumulate (exact_counts on): hash partition + all-to-all
    of the (key, count) pairs, merge on the owners, all-reduce kmer_per_neuron.
    Then ctr.finalize() takes the uniques column from the global kmer_per_neuron."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    dev = torch.device("cuda", torch.cuda.current_device())
    stream = torch.cuda.current_stream().cuda_stream
    send, kp, cp = ctr.exact_partition(world, stream)
    tot = sum(send)
    send_k = _dev_view(kp, tot, "<i8", dev)
    send_c = _dev_view(cp, tot, "<i4", dev)
    sc = torch.tensor(send, dtype=torch.int64, device=dev)
    rcnt = torch.empty_like(sc)
    _all_to_all(rcnt, sc, group=group)
    recv = rcnt.tolist()
    rk = torch.empty(sum(recv), dtype=torch.int64, device=dev)
    rc = torch.empty(sum(recv), dtype=torch.int32, device=dev)
    _all_to_all(rk, send_k, recv, send, group=group)
    _all_to_all(rc, send_c, recv, send, group=group)
    ctr.exact_adopt(rk.data_ptr(), rc.data_ptr(), rk.numel(), stream)
    kpn = _dev_view(ctr.device_kmer_per_neuron_ptr(), ctr.pool_size, "<i4", dev)
    dist.all_reduce(kpn, op=dist.ReduceOp.SUM, group=group)


def get_counts(ctr, keys: np.ndarray, group=None):
    """get_count for this rank's query keys against the distributed table:
    queries travel to their owners and the answers come back.  Collective:
    every rank calls it (possibly with no keys).  -> (counts u32, present bool)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    dev = torch.device("cuda", torch.cuda.current_device())
    keys = np.asarray(keys, dtype=np.uint64)
    own = exact_owner(keys, world)
    order = np.argsort(own, kind="stable")
    send = np.bincount(own, minlength=world).tolist()
    q = torch.from_numpy(keys[order].view(np.int64).copy()).to(dev)
    rcnt = torch.empty(world, dtype=torch.int64, device=dev)
    _all_to_all(rcnt, torch.tensor(send, dtype=torch.int64, device=dev), group=group)
    recv = rcnt.tolist()
    rq = torch.empty(sum(recv), dtype=torch.int64, device=dev)
    _all_to_all(rq, q, recv, send, group=group)
    mine = rq.cpu().numpy().view(np.uint64)
    cnt, pres = ctr.get_counts(mine) if mine.size else (np.zeros(0, np.uint32),
                                                       np.zeros(0, bool))
    ans = np.asarray(cnt, dtype=np.int64) | (np.asarray(pres, dtype=np.int64) << 32)
    back = torch.empty(keys.size, dtype=torch.int64, device=dev)
    _all_to_all(back, torch.from_numpy(ans).to(dev), send, recv, group=group)
    b = back.cpu().numpy()
    counts = np.empty(keys.size, np.uint32)
    present = np.empty(keys.size, bool)
    counts[order] = (b & 0xFFFFFFFF).astype(np.uint32)
    present[order] = (b >> 32) != 0
    return counts, present
