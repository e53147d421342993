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

shard_records() splits one input into world shards at record boundaries and,
where a record is longer than a shard, inside the record with a k-1 base halo,
so every window is counted by exactly one rank.  k > 32 (compat mode) keeps
whole records: its reverse strand depends on the record start
(src/models.rs:260-266).
"""
from __future__ import annotations

from typing import List, Tuple

import numpy as np


def shard_records(offsets: np.ndarray, world: int, k: int) -> List[Tuple[int, int, np.ndarray]]:
    """-> per rank (byte_lo, byte_hi, shard_offsets) with shard_offsets relative to
    byte_lo.  The k-mer start positions of the input are split into world
    contiguous ranges of (nearly) equal size."""
    offsets = np.asarray(offsets, dtype=np.int64)
    n = int(offsets[-1])
    if world <= 1 or n == 0:
        return [(0, n, offsets.astype(np.uint64))] + [(n, n, np.zeros(1, np.uint64))] * (world - 1)
    cuts = [n * r // world for r in range(world + 1)]
    if k > 32:  # snap to record starts
        cuts = [int(offsets[np.searchsorted(offsets, c, side="left")]) if c < n else n
                for c in cuts]
        cuts[0] = 0
    out = []
    for r in range(world):
        lo, hi = cuts[r], cuts[r + 1]
        if hi <= lo:
            out.append((lo, lo, np.zeros(1, np.uint64)))
            continue
        # records overlapping [lo, hi): starts in [lo, hi), the record holding lo
        i0 = int(np.searchsorted(offsets, lo, side="right")) - 1
        ends = []
        b_hi = hi
        j = i0
        while j < offsets.size - 1 and offsets[j] < hi:
            e = int(offsets[j + 1])
            if e > hi:  # record continues past the cut: keep k-1 halo bases
                e = min(e, hi + k - 1)
            ends.append(e)
            b_hi = max(b_hi, e)
            j += 1
        rel = np.array([0] + [e - lo for e in ends], dtype=np.uint64)
        out.append((lo, int(lo + rel[-1]), rel))
    return out


def allreduce_currents_(t, group=None) -> None:
    """In-place sum of a u64 currents vector held as int64 (same bits mod 2^64)."""
    import torch.distributed as dist
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)


def gather_union(keys, group=None):
    """All-gather variable-length int64 key lists -> one concatenated tensor
    (the merge deduplicates)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    n = torch.tensor([keys.numel()], dtype=torch.int64, device=keys.device)
    sizes = [torch.zeros(1, dtype=torch.int64, device=keys.device) for _ in range(world)]
    dist.all_gather(sizes, n, group=group)
    sizes = [int(s.item()) for s in sizes]
    mx = max(sizes) if sizes else 0
    pad = torch.full((max(mx, 1),), -1, dtype=torch.int64, device=keys.device)
    pad[:keys.numel()] = keys
    parts = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(parts, pad, group=group)
    return torch.cat([p[:s] for p, s in zip(parts, sizes)])
