#!/usr/bin/env python3
"""bench.py — NeuroKmer k-mer -> spike hot path on MI355X.

Metric (BASELINE.json): Mk-mers/s at k=31, pool=2M, total spikes bit-exact vs
the CPU reference restatement.

Workloads (--workload):
  config2 (default, weak scaling): 115,000,000 synthetic bases in 7 records
      per GPU, k=31, pool_size=2,000,000, --canonical, in-memory semantics
      (process_parallel).  The metric's configuration (BASELINE.json configs[1]).
  config3 (a side line: BASELINE.json configs[2]): a 10 GB synthetic FASTQ
      (150-bp reads) in /dev/shm streamed through nk_process_file_streaming,
      k=31, pool 16,000,000 (bench_side.py).
  config4 (strong scaling, a side line: configs[3]): one 100 Gbase input
      (--total-bases) in records of 115e6/7 bases, split into --shard-of
      shards (default: the world size) by dist.shard_records (byte ranges,
      records cut with a k-1 halo); rank r counts shard r.  On one GPU
      `--shard-of 8` times the per-GPU shard of the 8-GPU run (12.5 Gbases).
      k=31, pool 2M; currents all-reduced over RCCL.  Generated on the device.
  config5 (weak scaling, a side line: configs[4]): k=63 with 128-bit keys,
      pool 256,000,000, --bases per rank (default 12.5e9 = 100 Gbases / 8, in
      7 records, generated on the device); N>1 finishes pool-sliced
      (dist.finalize_step_sliced: reduce-scatter of the currents, LIF + top
      rows of each rank's 1/N of the pool).
  Side lines (rank 0, N=1) add `parity` (full-size properties + a bit-exact
  oracle compare on a 115 Mbase prefix), a prefix-timed `cpu_baseline` and
  the committed PMC traffic of their count kernels (profiles/pmc_<workload>.json).

One step = reset the neuron pool, then one full pass of the hot path over the
resident input: tile/record index -> K1a hash + partition -> K1b bucket
histograms -> [N>1: RCCL all-reduce of the currents] -> closed-form LIF ->
exact top-20 -> unique-k-mer pass for the top-20 rows [N>1: all-gather of the
top k-mer keys + merge] -> results in host memory.  Inputs are resident in HBM
before the timed region; timed steps run with no event between kernels
(stage_timing 3), K1a's duration comes from in-kernel s_memrealtime stamps.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload config2|config4]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU)

Without WORLD_SIZE in the environment, --gpus N > 1 starts N ranks itself
(torch.distributed.run on 127.0.0.1) before anything touches the GPU.  With
fewer visible devices than ranks the ranks share devices over gloo (a launch
rehearsal, labelled as such in config.parallelism; not a throughput figure).

Rank 0 at N=1 adds (config2):
  cpu_baseline  oracle/nk_oracle.c process_parallel restatement on the WHOLE
                115 Mbase input, parallel over the 7 records like rayon, and a
                full bit-compare of its outputs with the timed GPU run;
  end_to_end    file -> results (nk_process_file_parallel on a FASTA in the
                page cache) and host records -> results (nk_process_parallel,
                PCIe copy included): not `value`;
  exact_counts  the step with the exact k-mer table on (the drop-in shim's
                configuration).
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import socket
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

METRIC = "Mk-mers/sec at k=31, pool=2M; total-spikes bit-exact vs CPU ref"
SIDE_METRIC = {  # side lines (not BASELINE.json's metric): their own labels
    "config3": "Mk-mers/sec at k=31, pool=16M, 10 GB FASTQ streamed from the page cache",
    "config4": "Mk-mers/sec at k=31, pool=2M, one input split across the GPUs (strong scaling)",
    "config5": "Mk-mers/sec at k=63, pool=256M, 128-bit keys (BASELINE.json configs[4])",
}
K = 31
POOL = 2_000_000
BASES = 115_000_000
RECS = 7
REC_LEN4 = BASES // RECS  # config 4 record length
C4_TOTAL = 100_000_000_000  # config 4: 100 Gbases over the GPUs
C5_BASES = 12_500_000_000  # config 5: 100 Gbases / 8 per GPU
HOST_GEN_MAX = 1_000_000_000  # larger inputs are generated on the device
HBM_PEAK = 8.0e12  # B/s, MI355X spec (MI355X_MICROARCH.md chip table)


def n_kmers(offsets: np.ndarray, k: int) -> int:
    lens = np.diff(offsets.astype(np.int64))
    return int(np.clip(lens - k + 1, 0, None).sum())


def load_pmc():
    """The committed rocprofv3 PMC summary of K1a (profiles/pmc_count_kernel.json):
    HBM bytes and VALU instructions per launch of the config-2 workload."""
    try:
        with open(os.path.join(ROOT, "profiles", "pmc_count_kernel.json")) as f:
            return json.load(f)
    except Exception:
        return {}


def load_side_pmc(workload: str, n_bases: int, k: int, pool: int, width: int) -> dict:
    """profiles/pmc_<workload>.json (tools/pmc_side.py): HBM bytes and VALU
    instructions of one step's count kernels, when measured on this shape."""
    try:
        with open(os.path.join(ROOT, "profiles", f"pmc_{workload}.json")) as f:
            d = json.load(f)
    except Exception:
        return {}
    shape = d.get("shape", {})
    if (shape.get("bases"), shape.get("k"), shape.get("pool"), shape.get("width")) != \
            (n_bases, k, pool, width):
        return {}
    return d


class TorchRanks:
    """The N-rank job's host-side collectives: torch.distributed (gloo for
    bootstrap and timing; the data path uses the library's communicator)."""

    def __init__(self, on: bool):
        self.on = on

    def barrier(self):
        if self.on:
            import torch.distributed as dist
            dist.barrier()

    def max(self, x, dev):
        """max over ranks of a host number"""
        if not self.on:
            return x
        import torch
        import torch.distributed as dist
        t = torch.tensor([x], dtype=torch.float64 if isinstance(x, float) else torch.int64,
                         device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return type(x)(t.item())

    def gather_state(self, ctr):
        from neurokmer_amd import dist as nkdist
        return nkdist.gather_state(ctr)

    def close(self):
        if self.on:
            import torch.distributed as dist
            dist.destroy_process_group()


class LoopRanks:
    """--loopback N: the N-rank code path rehearsed on ONE
    GPU, every rank a host thread of this process with its own handles and
    streams, the library's collectives over its loopback transport
    (nk_loop_group_new: device copies + a sum kernel between host barriers,
    what RCCL does over xGMI).  Host-side barrier / max / state gather through
    shared memory.  Not a scaling figure: the ranks share one GPU."""

    def __init__(self, world: int):
        import threading
        self.world = world
        self.bar = threading.Barrier(world)
        self.slots = [None] * world
        self.local = threading.local()

    def barrier(self):
        self.bar.wait(timeout=600)

    def max(self, x, dev=None):
        self.slots[self.local.rank] = x
        self.bar.wait(timeout=600)
        m = max(self.slots)
        self.bar.wait(timeout=600)
        return type(x)(m)

    def gather_state(self, ctr):
        from neurokmer_amd import dist as nkdist
        r, pool = self.local.rank, ctr.pool_size
        lo, hi, _ = nkdist.slice_bounds(pool, self.world, r)
        self.slots[r] = {n: a[lo:hi].copy() for n, a in (
            ("currents", ctr.currents()), ("spike_counts", ctr.spike_counts()),
            ("voltages", ctr.voltages()), ("refractory", ctr.refractory()))}
        self.bar.wait(timeout=600)
        out = {n: np.concatenate([self.slots[q][n] for q in range(self.world)])
               for n in self.slots[0]}
        self.bar.wait(timeout=600)
        return out

    def close(self):
        pass


def loopback_main(args) -> int:
    """--loopback N: rank_main on N threads sharing one loopback group."""
    import copy
    import threading
    import traceback
    from neurokmer_amd import dist as nkdist
    n = args.loopback
    ctx = LoopRanks(n)
    grp = nkdist.LoopbackGroup(n)
    comms = [nkdist.Comm.loopback(grp, r, 0) for r in range(n)]
    rcs, errs = [1] * n, [None] * n

    def run(r):
        ctx.local.rank = r
        try:
            rcs[r] = rank_main(copy.copy(args), n, r, 0, ctx, comms[r])
        except Exception:
            errs[r] = traceback.format_exc()
            ctx.bar.abort()

    ts = [threading.Thread(target=run, args=(r,)) for r in range(n)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    for e in errs:
        if e:
            print(e, file=sys.stderr)
    for c in comms:
        c.close()
    grp.close()
    return 0 if all(rc == 0 for rc in rcs) and not any(errs) else 1


def spawn_ranks(n: int) -> int:
    """Start n ranks of this script (torch.distributed.run, 127.0.0.1) and
    return their exit code.  Runs before any GPU call in this process."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={n}", "--master-addr", "127.0.0.1", f"--master-port={port}",
           os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def cpu_baseline(bases: np.ndarray, offsets: np.ndarray, k: int, pool: int):
    """oracle/nk_oracle.c's restatement of process_parallel (src/spiking_hash.rs:
    84-201) over the whole input: one thread per record like rayon's par_iter
    over records (:94-95), exact k-mer map, serial merge, serial 1000-step LIF
    (memoised by count for fresh neurons: the port is faster than the reference
    there, so the GPU ratio is conservative)."""
    from oracle import cbind
    threads = offsets.size - 1
    ref = cbind.OracleCounter(k, 1.0, 0.95, 2, 1.0, pool, True)
    t0 = time.perf_counter()
    ref.process_parallel_arrays(bases, offsets, threads)
    dt = time.perf_counter() - t0
    return ref, dt, threads


def parity(gpu, ref) -> dict:
    """Bit-compare every output of the GPU handle with the restatement."""
    out = {
        "currents": bool(np.array_equal(gpu.currents(), ref.currents())),
        "spike_counts": bool(np.array_equal(gpu.spike_counts(), ref.spike_counts())),
        "voltages_bitwise": bool(np.array_equal(gpu.voltages().view(np.uint32),
                                                ref.voltages().view(np.uint32))),
        "refractory": bool(np.array_equal(gpu.refractory(), ref.refractory())),
        "total_spikes": [gpu.energy.total_spikes(), ref.total_spikes],
        "energy_used": [gpu.energy_used(), ref.energy_used()],
        "top20_with_uniques": gpu.top_abundant_neurons(20) == ref.top_abundant_neurons(20),
    }
    out["all_equal"] = bool(out["currents"] and out["spike_counts"] and out["voltages_bitwise"]
                            and out["refractory"] and out["top20_with_uniques"]
                            and out["total_spikes"][0] == out["total_spikes"][1]
                            and out["energy_used"][0] == out["energy_used"][1])
    return out


def log(msg: str) -> None:
    """Progress on stderr (a long run keeps its log growing)."""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def timed(fn, reps: int):
    """(best, median) wall seconds of fn() over reps runs after one warm run."""
    fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return min(ts), float(np.median(ts))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # the overlapped run's first two steps carry the pipeline's fill (~0.7 ms
    # extra in all): 50 steps amortise it (profiles/r02_s22)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", choices=("config2", "config3", "config4", "config5"),
                    default="config2")
    ap.add_argument("--bases", type=int, default=None,
                    help="config2/5: bases per rank (default 115e6 / 12.5e9)")
    ap.add_argument("--total-bases", type=int, default=C4_TOTAL, help="config4: bases in all")
    ap.add_argument("--shard-of", type=int, default=0,
                    help="config4: split the input into this many shards (default: the world size; 8 on one GPU)")
    ap.add_argument("--no-side-parity", action="store_true",
                    help="side lines: skip the properties / prefix oracle compare")
    ap.add_argument("--fastq", default=None, help="config3: the FASTQ (default: generated in /dev/shm)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extras", action="store_true",
                    help="skip end_to_end and the exact_counts step (rank 0, N=1)")
    ap.add_argument("--no-parity-ranks", action="store_true",
                    help="N > 1: skip the check of the N-rank result against one GPU")
    ap.add_argument("--settle", type=float, default=0.25,
                    help="seconds of untimed steps after the warmup (GPU clock settle)")
    # side measurements only (the metric is k=31, pool 2M)
    ap.add_argument("--pool", type=int, default=POOL)
    ap.add_argument("--k", type=int, default=K)
    ap.add_argument("--kmer-width", type=int, default=64, choices=(64, 128))
    ap.add_argument("--dist-backend", default=None, help="default: nccl (RCCL), gloo if ranks share a GPU")
    # rehearsal: the multi-rank step (wire all-reduce, key all-gather, merge) in
    # a 1-rank process group, to measure its overhead on a 1-GPU box
    ap.add_argument("--force-dist", action="store_true")
    # N > 1 over RCCL: the finish runs inside the library (nk_finalize_dist, its
    # own communicator) unless --dist-python drives it from Python with torch's
    # collectives between the library calls (the round-2 protocol, for A/B)
    ap.add_argument("--dist-python", action="store_true")
    # diagnosis: the process group (and the library's communicator) set up, the
    # step itself the plain one-GPU step (what RCCL's presence alone costs)
    ap.add_argument("--dist-init-only", action="store_true")
    ap.add_argument("--nk-comm", action="store_true", help="the library's communicator under gloo too")
    ap.add_argument("--finish", choices=("plain", "sliced"), default=None,
                    help="N > 1: all-reduce + the whole pool's LIF on every rank (plain), or "
                         "reduce-scatter + each rank's 1/N of the pool (sliced; default with the "
                         "in-library communicator, and always for config5)")
    ap.add_argument("--inflight", type=int, default=None, choices=(1, 2, 3, 4),
                    help="batches in flight (default: 3 on one GPU, 1 across ranks and for "
                         "config5): > 1 "
                         "overlaps a batch's finish with the next batch's count")
    ap.add_argument("--defer-hist", choices=("auto", "on", "off"), default="off",
                    help="each handle's bucket histogram (K1b) inside the next handle's count "
                         "kernel (nk_opts.defer_hist, k_part_fused); auto: on with >= 3 batches "
                         "in flight on one GPU.  Off by default: the fused kernel leaves the "
                         "finishes no window (0.56-0.57 vs 0.50-0.51 ms per step, profiles/r06_fuse)")
    ap.add_argument("--loopback", type=int, default=0,
                    help="N > 1: rehearse the N-rank path on ONE GPU, ranks as threads over the "
                         "library's loopback transport (not a scaling figure)")
    args = ap.parse_args()

    if args.loopback > 1:
        if args.workload not in ("config2", "config5"):
            print("bench.py: --loopback rehearses configs 2 and 5", file=sys.stderr)
            return 2
        args.gpus = args.loopback
        return loopback_main(args)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return spawn_ranks(args.gpus)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return rank_main(args, world, rank, local, None, None)


def rank_main(args, world: int, rank: int, local: int, ctx, lcomm) -> int:
    """One rank's bench (ctx None: this process is the rank, torch.distributed
    between ranks; else a LoopRanks thread with its loopback communicator)."""
    loop = ctx is not None
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; launch with "
              f"torchrun --nproc-per-node {args.gpus} (or no torchrun)", file=sys.stderr)
        return 2

    if args.workload == "config3":
        import bench_side
        return bench_side.config3(args)
    if args.bases is None:
        args.bases = C5_BASES if args.workload == "config5" else BASES

    import torch
    import torch.distributed as dist

    if args.workload == "config5":  # BASELINE.json configs[4]
        args.k, args.pool, args.kmer_width = 63, 256_000_000, 128
    pool, k = args.pool, args.k
    ndev = torch.cuda.device_count()  # counts devices without initialising them
    shared = world > ndev and not loop  # rehearsal: ranks share devices (gloo)
    dev_idx = local % max(ndev, 1)
    dist_on = world > 1 or args.force_dist
    # the device collectives: the library's own RCCL communicator (the whole
    # finish inside nk_finalize_dist) unless --dist-python drives torch's.  The
    # process group then only bootstraps it (the unique id) and times the run
    # (barriers, max over ranks): gloo.  A torch RCCL group in the process
    # slowed K1a by 5-20 % even when unused (1-rank rehearsal: 0.599-0.628 vs
    # 0.576-0.577 ms per step with gloo, plain 0.546-0.549, profiles/r03_s10..s12)
    lib_comm = dist_on and not shared and not args.dist_python
    if args.workload == "config5":
        args.finish = "sliced"
    elif args.finish is None:
        args.finish = "sliced" if lib_comm else "plain"
    backend = args.dist_backend or ("gloo" if shared or lib_comm else "nccl")
    if args.inflight is None:
        # config 5 (P = 256 M): its finish is a 256 M-neuron LIF + top-N pass
        # that gains nothing beside a count (5.15 vs 5.02-5.07 ms, r02_s29).
        # Across ranks with the in-library finish two batches in flight (the
        # next count enqueued before this batch's finish: 1-rank rehearsal
        # 0.5618 vs 0.5743 ms one at a time, profiles/r03_s17); three measured
        # slower (0.68 ms, r03_s12), and so did the Python-driven finish with
        # any overlap (0.698 vs 0.624 ms, profiles/r02_s21)
        if args.workload == "config5":
            args.inflight = 1
        elif dist_on:
            args.inflight = 2 if lib_comm else 1
        else:
            args.inflight = 3
    if dist_on and not loop:
        if "RANK" not in os.environ:  # --force-dist without a launcher: a 1-rank group
            with socket.socket() as sk:
                sk.bind(("127.0.0.1", 0))
                os.environ.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0",
                                  MASTER_ADDR="127.0.0.1",
                                  MASTER_PORT=str(sk.getsockname()[1]))
        torch.cuda.set_device(dev_idx)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev_idx))
        else:
            os.environ.setdefault("GLOO_SOCKET_IFNAME", "lo")  # one node, 127.0.0.1
            dist.init_process_group(backend)
    dev = torch.device("cuda", dev_idx)
    if loop:
        torch.cuda.set_device(dev_idx)
    else:
        ctx = TorchRanks(dist_on)

    from neurokmer_amd import SpikingKmerCounter, synth
    from neurokmer_amd import dist as nkdist
    from neurokmer_amd.counter import diag_hash_ms
    comm = lcomm if loop else \
        (nkdist.Comm(device=dev_idx) if (lib_comm or (dist_on and args.nk_comm)) else None)

    # ---- this rank's input (resident in HBM) -------------------------------
    bases = None  # host copy (host-generated inputs only)
    if args.workload in ("config2", "config5"):
        seed = synth.SEED ^ (rank * 0x9E37)
        if args.bases <= HOST_GEN_MAX:
            bases, offsets = synth.make_records(args.bases, RECS, seed=seed,
                                                repeats_per_mb=64, motif_len=200)
            d_bases = torch.from_numpy(bases).to(dev)
        else:  # the same stream generated on the device (bench_side.py checks a prefix)
            d_bases, offsets = synth.make_records_torch(args.bases, RECS, seed=seed,
                                                        repeats_per_mb=64, motif_len=200,
                                                        device=dev)
        n_bases = args.bases
        nk_rank = n_kmers(offsets, k)
        total_kmers = world * nk_rank  # same size on every rank
        scaling = "weak"
        workload = (f"config {args.workload[-1]}: {n_bases:,} bases in {RECS} records per GPU, "
                    f"k={k}, kmer_width={args.kmer_width}, pool_size={pool:,}, --canonical, "
                    + ("process_parallel" if world == 1 and not dist_on else
                       f"{args.finish} multi-GPU finish"))
    else:
        T = args.total_bases
        # one GPU holds the 12.5 Gbase shard of an 8-GPU run by default (the
        # whole 100 Gbase input would not fit one GPU's arena); --shard-of 1
        # asks for all of it
        n_shards = args.shard_of or (8 if world == 1 and T == C4_TOTAL else world)
        if n_shards < world:
            print("bench.py: --shard-of must be >= the world size", file=sys.stderr)
            return 2
        n_rec = max(1, -(-T // REC_LEN4))
        glob = np.minimum(np.arange(n_rec + 1, dtype=np.int64) * REC_LEN4, T).astype(np.uint64)
        shards = nkdist.shard_records(glob, n_shards, k)
        lo, hi, rel, _skip = shards[rank]  # k <= 32: no warm-up
        n_bases = hi - lo
        d_bases = torch.zeros(n_bases + 16, dtype=torch.uint8, device=dev)
        synth.random_bases_torch(n_bases, synth.SEED, lo, dev, out=d_bases)
        offsets = rel.astype(np.uint64)
        args.shard_lo = lo
        nk_rank = n_kmers(offsets, k)
        total_kmers = sum(n_kmers(sh[2].astype(np.uint64), k) for sh in shards[:world])
        scaling = "strong"
        workload = (f"config 4 (strong scaling): {T:,} bases in {n_rec} records of {REC_LEN4:,}, "
                    f"split by shard_records into {n_shards} shards"
                    + (f", rank r counts shard r (here: shard 0 of {n_shards} on {world} GPU)"
                       if n_shards != world else f" over {world} rank(s)")
                    + f", k={k}, pool_size={pool:,}, --canonical")
    n_recs = offsets.size - 1
    log(f"rank {rank}/{world}: {n_bases:,} bases, {n_recs} records on cuda:{dev_idx}")
    d_offs = torch.from_numpy(offsets.view(np.int64)).to(dev)
    torch.cuda.synchronize()

    # m handles (--inflight m): the counts of batches i+1 .. i+m-1 are enqueued
    # before batch i's finish (LIF, top-N, uniques, readback; N > 1: the
    # collectives) is awaited.  Finishes go on a high-priority stream (its own
    # hardware queue: two same-priority torch streams were measured sharing
    # one queue, which serialises them), so a batch's finish runs beside the
    # next batch's count.  The library orders a handle's calls across streams
    # itself (pick_stream: the finish waits for the end of ITS handle's count
    # only).  --inflight 1: one handle, one stream, one batch at a time.
    # K1b of batch i inside K1a of batch i+1 (k_part_fused): a batch's finish
    # then waits for the next count, so it needs three batches in flight (with
    # two the count stream would idle through every finish)
    defer_hist = (args.defer_hist == "on" or
                  (args.defer_hist == "auto" and args.inflight >= 3 and not dist_on))
    ctrs = [SpikingKmerCounter(k, 1.0, 0.95, 2, 1.0, pool, True, device=dev_idx,
                               kmer_width=args.kmer_width, defer_hist=defer_hist)
            for _ in range(args.inflight)]
    ctr = ctrs[0]
    # non-default streams: a NULL stream handle would mean the library's own.
    # (Count streams CU-masked to leave 8-32 CUs to the finishes slowed K1a by
    # 13-90 %, profiles/r02_s26, r02_s27: not used.)
    # All handles count on ONE stream: one hardware queue, so the counts queue
    # back to back and the count queue never idles while a finish is awaited
    # (the library orders each handle's finish on the end of its own count).
    # Measured slower and not kept: a stream per handle with 3 in flight (the
    # third count's queue was not served until the finish queue went idle,
    # 0.529-0.537 vs 0.507-0.514 ms, profiles/r02_s31); handles alternating
    # between two count streams (0.5166 vs 0.5026 ms, profiles/r03_cs2; round 6,
    # each count kernel ordered only after the previous batch's count kernel so
    # that it could start beside that batch's K1b: 0.523-0.531 vs 0.510-0.516
    # ms, profiles/r06_ab).
    count_streams = [torch.cuda.Stream(device=dev)] * args.inflight
    run_stream = count_streams[0]
    fin_stream = (torch.cuda.Stream(device=dev, priority=torch.cuda.Stream.priority_range()[1])
                  if args.inflight > 1 else run_stream)
    torch.cuda.set_stream(run_stream)
    s_handle = run_stream.cuda_stream

    start_host_s = []  # host time of each start() (the enqueue of a count)
    settle_each = [False]
    # side lines (configs 4/5): hipEvents on the count stream around each
    # step's whole count (a multi-GB input runs several batches per count)
    side = args.workload in ("config4", "config5")
    count_ev = []

    def start(j):
        """Enqueue one batch's count on handle j (returns at once)."""
        t_s = time.perf_counter()
        c, cs = ctrs[j], count_streams[j]
        sh = cs.cuda_stream
        c.reset(sh, blocking=False)
        if side:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(cs)
        c.accumulate_device(d_bases.data_ptr(), d_offs.data_ptr(), n_recs, n_bases, sh)
        if side:
            e1.record(cs)
            count_ev.append((e0, e1))
        start_host_s.append(time.perf_counter() - t_s)

    def finish(j, st, between=None):
        """LIF + top-N + uniques of handle j's batch on stream st, results read
        back (the one host wait).  N > 1: RCCL over xGMI -- the currents as
        u32 while every rank's k-mers together stay below 2^31, LIF + top-N +
        this shard's top k-mers into a fixed-size all-gather segment, the union
        merged on the device; `between` (the next batch's count) is enqueued
        once the all-reduce is, so that count waits for the all-reduce only."""
        c = ctrs[j]
        if not dist_on or args.dist_init_only:
            if between is not None:
                between()
            c.finalize(False, st.cuda_stream)
            if settle_each[0]:  # write out v / refractory / spike counts too (nk_settle)
                c.settle(st.cuda_stream)
            return
        with torch.cuda.stream(st):
            if args.finish == "sliced":
                if between is not None:
                    between()
                nkdist.finalize_step_sliced(c, total_kmers=total_kmers, comm=comm)
            else:
                nkdist.finalize_step(c, total_kmers=total_kmers, between=between, comm=comm)

    def run(n, inflight, marks=None):
        """n complete steps (count + finish of one batch each), at most
        `inflight` batches in flight; all n are finished on return."""
        if n <= 0:
            return
        if inflight == 1:
            for _ in range(n):
                start(0)
                finish(0, run_stream)
                if marks is not None:
                    marks.append(time.perf_counter())
            return
        m = inflight
        for j in range(min(m - 1, n)):
            start(j)
        for i in range(n):
            nxt = (lambda h=(i + m - 1) % m: start(h)) if i + m - 1 < n else None
            finish(i % m, fin_stream, nxt)
            if marks is not None:
                marks.append(time.perf_counter())

    def step():
        run(1, 1)

    per = float("inf")  # fastest warmup step (the first one allocates)
    for _ in range(max(args.warmup, 1 if args.settle > 0 else 0)):
        t_w = time.perf_counter()
        run(args.inflight, args.inflight)  # every handle allocates
        torch.cuda.synchronize()
        per = min(per, (time.perf_counter() - t_w) / args.inflight)
    # clock settle: the GPU reaches its sustained clock only after ~10-30 ms of
    # load, so untimed steps continue for about --settle seconds; every rank
    # runs the same number (the steps contain collectives)
    settle = 0
    if args.settle > 0:
        settle = min(int(args.settle / max(per, 1e-4)) + 1, 5000)
        if dist_on:
            settle = ctx.max(settle, dev)
        run(settle, args.inflight)
        torch.cuda.synchronize()
    # timed steps record no events at all (stage_timing 3); K1a's duration
    # comes from its in-kernel stamps
    timed_level = 3
    for c in ctrs:
        c.set_stage_timing(timed_level)
    # one more untimed round in the timed mode: the first step after the switch
    # measured ~0.18 ms slower on the host side (profiles/r02_s2/bench_default.log,
    # step_ms_host[0]) while its K1a span was normal
    run(args.inflight, args.inflight)
    torch.cuda.synchronize()

    def timed(n, inflight, marks):
        if dist_on:
            ctx.barrier()
        torch.cuda.synchronize()
        t_a = time.perf_counter()
        run(n, inflight, marks)
        torch.cuda.synchronize()
        if dist_on:
            ctx.barrier()
        torch.cuda.synchronize()
        d = time.perf_counter() - t_a
        if dist_on:
            d = ctx.max(d, dev)
        return t_a, d

    marks = []
    del start_host_s[:]
    del count_ev[:]
    t0, dt = timed(args.steps, args.inflight, marks)
    count_ms = [a.elapsed_time(b) for a, b in count_ev]
    start_ms = sorted(start_host_s)
    start_ms = (round(start_ms[len(start_ms) // 2] * 1e3, 4), round(start_ms[-1] * 1e3, 4)) \
        if start_ms else None
    # both handles' last batches (same input) gave the same results
    same_inflight = None
    if args.inflight > 1:
        same_inflight = all(c.top_abundant_neurons(20) == ctrs[0].top_abundant_neurons(20) and
                            c.energy.total_spikes() == ctrs[0].energy.total_spikes()
                            for c in ctrs[1:])
    # the same K steps one batch at a time: the step latency, and K1a's
    # duration without the other batch's finish beside it (the roofline)
    marks1 = []
    _, dt1 = timed(args.steps, 1, marks1) if args.inflight > 1 else (t0, dt)

    log(f"timed {args.steps} steps: {dt / args.steps * 1e3:.4f} ms/step")
    # K1a of every step of the one-at-a-time run (in-kernel stamps), and of
    # handle 1's steps in the overlapped run (the other batch's finish beside it)
    spans = ctr.count_spans(args.steps)
    spans2 = ctrs[1].count_spans(args.steps // args.inflight) if args.inflight > 1 else []
    # the overlapped run's count kernels (handles 1.., whose last counts are that
    # run's; handle 0's are the one-in-flight run's): with defer_hist each is
    # k_part_fused (K1a of its batch + K1b of the batch before)
    spans_ov = [x for c in ctrs[1:] for x in c.count_spans(args.steps // args.inflight)] \
        if args.inflight > 1 else []
    # the same steps writing the per-neuron state out in each (the reference
    # writes v, refractory and spike counts in every call, src/spiking_hash.rs:
    # 186-200; the step above leaves them derived from the currents until a
    # reader asks, nk_settle): what that write costs per step
    dt_settle = None
    if not dist_on:
        settle_each[0] = True
        _, dt_settle = timed(args.steps, args.inflight, [])
        settle_each[0] = False
    total_spikes = ctr.energy.total_spikes()
    # cross-check: K1a between hipEvents in 5 extra (untimed) steps
    ctr.set_stage_timing(0)
    for _ in range(5):
        step()
    torch.cuda.synchronize()
    ev_ms = [x for x in ctr.count_history(5) if x == x and x > 0]
    stages = ctr.last_timings()
    ctr.set_stage_timing(timed_level)
    # N > 1: the N-rank result against one GPU counting every rank's shard
    pr = None
    if world > 1 and not args.no_parity_ranks:
        log("parity_ranks: the union of every rank's input on rank 0's GPU")
        pr = parity_ranks(args, ctr, world, rank, dev_idx, nkdist, SpikingKmerCounter, synth,
                          total_kmers, ctx)
        ctx.barrier()

    if rank == 0:
        ms_step = dt / args.steps * 1e3
        value = total_kmers / (dt / args.steps) / 1e6 if scaling == "strong" else \
            world * nk_rank / (dt / args.steps) / 1e6
        sp = [x for x in spans if x > 0]
        k1_ms = float(np.mean(sp)) if sp else (float(np.mean(ev_ms)) if ev_ms else float("nan"))
        k1a_alone_ms = k1_ms  # K1a without K1b (the one-in-flight run)
        fused = defer_hist and args.workload == "config2" and k <= 32 and pool <= (1 << 23)
        if fused:
            # the metric's dominant kernel is then k_part_fused, as it runs in
            # the timed overlapped steps (the next batch's finish beside it):
            # the count's whole work, K1a's hash + K1b's histogram, per launch
            sp = [x for x in spans_ov if x > 0]
            k1_ms = float(np.mean(sp)) if sp else k1_ms
        # roofline of the dominant kernel (K1a), algorithmic bytes per launch =
        # input bases read once + one 8-B counter update per k-mer
        alg_bytes = n_bases + 8 * nk_rank
        cm = float(np.median(count_ms)) if (side and count_ms) else None
        if cm:  # side lines: the whole count of a step (every batch) between hipEvents
            k1_ms = cm
        achieved = alg_bytes / (k1_ms * 1e-3)
        pmc = load_pmc()
        cfg2 = args.workload == "config2" and args.bases == BASES and k == K and pool == POOL
        traffic = pmc.get("hbm_bytes_per_launch") if cfg2 else None
        side_pmc = load_side_pmc(args.workload, n_bases, k, pool, args.kmer_width) if side else {}
        if side_pmc:
            traffic = side_pmc.get("hbm_bytes_per_count")
        # the limiter, measured in this run: the same GPU's rate for the hash
        # work alone (SipHash-1-3 + exact % pool of register-generated keys, no
        # memory traffic: nk_diag_hash_ms) against K1a's k-mer rate
        floor_ms = diag_hash_ms(nk_rank, pool, dev_idx, reps=5, width=args.kmer_width) \
            if pool < (1 << 30) else None
        valu = {"kmers_per_launch": nk_rank,
                "k1a_gkmers_per_s": round(nk_rank / (k1_ms * 1e-3) / 1e9, 2)}
        if floor_ms:
            valu.update({"hash_only_ms": round(floor_ms, 4),
                         "hash_only_gkmers_per_s": round(nk_rank / (floor_ms * 1e-3) / 1e9, 2),
                         "frac_of_hash_only": round(floor_ms / k1_ms, 4)})
        if side_pmc.get("valu_instr_per_count"):
            valu["valu_instr_per_count"] = side_pmc["valu_instr_per_count"]
        if cfg2 and pmc.get("valu_instr_per_launch"):
            valu["valu_instr_per_launch"] = pmc["valu_instr_per_launch"]
            valu["pmc_source"] = pmc.get("source")
        hbm_frac = achieved / HBM_PEAK
        frac_h = valu.get("frac_of_hash_only", 0.0)
        bound = "valu" if frac_h >= 0.6 and frac_h >= hbm_frac else ("hbm" if hbm_frac >= 0.6 else "latency")
        out = {
            "metric": METRIC if args.workload == "config2" else SIDE_METRIC[args.workload],
            "value": round(value, 3), "unit": "Mk-mers/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "settle_steps": settle,
            "ms_per_step": round(ms_step, 4),
            "inflight": args.inflight,
            "defer_hist": defer_hist,
            "rehearsal": bool(loop or shared),
            "ms_per_step_one_in_flight": round(dt1 / args.steps * 1e3, 4),
            "ms_per_step_state_written": (round(dt_settle / args.steps * 1e3, 4)
                                          if dt_settle is not None else None),
            "state_written_note": ("the same steps (same batches in flight) with nk_settle after "
                                   "each finish: v, refractory and spike counts written to HBM "
                                   "as the reference does every call; `value` is the step "
                                   "without that write (the state is derived on demand, "
                                   "bit-identical when read)"),
            "inflight_handles_same_results": same_inflight,
            "start_host_ms_median_max": start_ms,
            "higher_is_better": True, "scaling": scaling, "vs_baseline": None, "dtype": "u64",
            "data": ("synthetic (splitmix64 i.i.d. ACGT, seed 0x4E4B4D52" +
                     ("^rank, 64x200-bp planted repeats per MB)" if args.workload != "config4"
                      else ", one global stream sharded by byte range)")),
            "config": {"workload": workload, "k": k, "kmer_width": args.kmer_width,
                       "pool_size": pool, "bases_rank0": int(n_bases), "records_rank0": n_recs,
                       "kmers_rank0": nk_rank, "kmers_total": total_kmers,
                       "parallelism": f"dp{world}" + (
                           f" (REHEARSAL, not a scaling figure: {world} ranks as threads of one "
                           f"process on 1 GPU, the library's loopback transport)" if loop else
                           f" (rehearsal: {world} ranks on {ndev} GPU, {backend})" if shared else ""),
                       "finish": args.finish if dist_on else None,
                       "collectives": ((f"in-library communicator ("
                                        f"{'nk_finalize_sliced_dist' if args.finish == 'sliced' else 'nk_finalize_dist'})"
                                        + (" over the loopback transport; host barrier/max between "
                                           "threads" if loop else
                                           f" over RCCL; torch.distributed {backend} for bootstrap "
                                           "and timing"))
                                       if comm is not None
                                       else (f"torch.distributed {backend} from Python" if dist_on
                                             else None))},
            "roofline": {"bound": bound,
                         "kernel": ("the count of a step: every batch's K1 (k_part / k_part_gen "
                                    "+ k_split) + K1b (k_bucket_hist)" if cm else
                                    "k_part_fused (K1a of batch i+1 + K1b of batch i: the "
                                    "count's hash and histogram, one launch per step)" if fused else
                                    "k_part<canonical> (K1a)" if k <= 32 and pool <= (1 << 24)
                                    else "the count: k_part_gen (K1g) + k_split (K1s)"),
                         "k1a_alone_ms": round(k1a_alone_ms, 4) if fused else None,
                         "achieved": round(achieved / 1e9, 2), "peak": HBM_PEAK / 1e9,
                         "unit": "GB/s", "frac": round(hbm_frac, 4),
                         "traffic": traffic,
                         "traffic_source": ((side_pmc.get("source") if side_pmc else pmc.get("source"))
                                            if traffic else None),
                         "alg_bytes_per_launch": alg_bytes, "avg_launch_ms": round(k1_ms, 4),
                         "avg_launch_source": (
                             "hipEvents on the count stream around each timed step's count "
                             "(every batch's K1 + K1b), median" if cm else
                             "in-kernel s_memrealtime span over the timed (overlapped) steps' "
                             "count kernels" if fused and sp else
                             ("in-kernel s_memrealtime span over the one-in-flight timed steps"
                              if sp else "hipEvents")),
                         "launches_timed": len(sp),
                         "avg_launch_ms_events": round(float(np.mean(ev_ms)), 4) if ev_ms else None,
                         "valu": valu},
            "stage_ms_event_steps": {k2: round(v, 4) for k2, v in stages.items()},
            "step_ms_host": [round((b - a) * 1e3, 4) for a, b in zip([t0] + marks[:-1], marks)],
            "k1a_ms_steps": [round(x, 4) for x in spans],
            "k1a_ms_steps_overlapped": [round(x, 4) for x in spans2],
            "total_spikes": total_spikes,
        }
        if pr is not None:
            out["parity_ranks"] = pr
        if world == 1 and args.workload == "config2" and args.kmer_width == 64 and bases is not None:
            # (extras time the host-array and file paths from the host copy of
            # the input: none past HOST_GEN_MAX, where it is generated on the device)
            out.update(extras(args, ctr, bases, offsets, nk_rank, d_bases, d_offs, s_handle,
                              dev_idx, SpikingKmerCounter, synth))
        if side:
            out["count_ms_steps"] = [round(x, 4) for x in count_ms]
        if world == 1 and side and not args.no_side_parity:
            import bench_side
            out.update(bench_side.side_extras(args, ctr, d_bases, offsets, n_bases, nk_rank,
                                              dev_idx))
        print(json.dumps(out), flush=True)
    for c in ctrs:
        if comm is not None:
            comm.forget(c)
        c.close()
    if comm is not None and not loop:
        comm.close()
    if not loop:
        ctx.close()
    return 0


def parity_ranks(args, ctr, world, rank, dev_idx, nkdist, Counter, synth, total_kmers, ctx):
    """N > 1 (collective; the result on rank 0): rank 0 regenerates EVERY rank's
    input, counts their union in ONE process call on its own GPU, and compares
    the N-rank step's final state with it bit for bit.  The reference sums the
    per-record currents (src/spiking_hash.rs:145-154), so one call over all
    records is the N-rank answer (bit-identical currents at 1,
    2, 4 and 8 GPUs).  Pool-sliced state (config5) is gathered first."""
    import torch
    st = ctx.gather_state(ctr) if args.finish == "sliced" else None
    if rank != 0:
        return None
    k, pool = args.k, args.pool
    t0 = time.perf_counter()
    dev = torch.device("cuda", dev_idx)
    if args.workload == "config4":  # every shard of this run: [0, last shard's end)
        T = args.total_bases
        n_rec = max(1, -(-T // REC_LEN4))
        glob = np.minimum(np.arange(n_rec + 1, dtype=np.int64) * REC_LEN4, T).astype(np.uint64)
        n_shards = args.shard_of or world
        end = nkdist.shard_records(glob, n_shards, k)[world - 1][1]
        offs = np.concatenate([glob[glob < end], np.array([end], np.uint64)])
        n_all = int(end)
        d_b = torch.zeros(n_all + 16, dtype=torch.uint8, device=dev)
        synth.random_bases_torch(n_all, synth.SEED, 0, dev, out=d_b)
    else:
        parts, offl, at = [], [np.zeros(1, np.uint64)], 0
        for r in range(world):
            seed = synth.SEED ^ (r * 0x9E37)
            if args.bases <= HOST_GEN_MAX:
                b, o = synth.make_records(args.bases, RECS, seed=seed, repeats_per_mb=64,
                                          motif_len=200)
                parts.append(torch.from_numpy(b).to(dev))
            else:
                b, o = synth.make_records_torch(args.bases, RECS, seed=seed, repeats_per_mb=64,
                                                motif_len=200, device=dev, pad=0)
                parts.append(b)
            offl.append(o[1:] + np.uint64(at))
            at += args.bases
        parts.append(torch.zeros(16, dtype=torch.uint8, device=dev))
        d_b = torch.cat(parts)
        del parts
        offs = np.concatenate(offl)
        n_all = at
    gen_s = time.perf_counter() - t0
    d_o = torch.from_numpy(offs.view(np.int64)).to(dev)
    torch.cuda.synchronize()
    g = Counter(k, 1.0, 0.95, 2, 1.0, pool, True, device=dev_idx, kmer_width=args.kmer_width)
    g.process_parallel_device(d_b.data_ptr(), d_o.data_ptr(), offs.size - 1, n_all)
    if st is None:
        st = {"currents": ctr.currents(), "spike_counts": ctr.spike_counts(),
              "voltages": ctr.voltages(), "refractory": ctr.refractory()}
    one = {"currents": g.currents(), "spike_counts": g.spike_counts(),
           "voltages": g.voltages(), "refractory": g.refractory()}
    top_n, top_1 = ctr.top_abundant_neurons(20), g.top_abundant_neurons(20)
    # every step starts from a reset pool: the spike counts are the last step's
    spikes_n, spikes_1 = int(st["spike_counts"].sum(dtype=np.uint64)), g.energy.total_spikes()
    out = {"method": (f"rank 0 regenerated all {world} ranks' inputs ({n_all:,} bases, "
                      f"{offs.size - 1} records) and ran ONE process_parallel over them on its GPU; "
                      "compared with the N-rank step's final state"),
           "currents": bool(np.array_equal(st["currents"], one["currents"])),
           "spike_counts": bool(np.array_equal(st["spike_counts"], one["spike_counts"])),
           "voltages_bitwise": bool(np.array_equal(st["voltages"].view(np.uint32),
                                                   one["voltages"].view(np.uint32))),
           "refractory": bool(np.array_equal(st["refractory"], one["refractory"])),
           "top20_with_uniques": top_n == top_1,
           "total_spikes": [spikes_n, spikes_1],
           "sum_currents": [int(st["currents"].sum(dtype=np.uint64)), int(total_kmers)],
           "currents_sha1": hashlib.sha1(st["currents"].tobytes()).hexdigest()[:16],
           "seconds": round(time.perf_counter() - t0, 2), "generate_s": round(gen_s, 2)}
    out["all_equal"] = bool(out["currents"] and out["spike_counts"] and out["voltages_bitwise"]
                            and out["refractory"] and out["top20_with_uniques"]
                            and spikes_n == spikes_1
                            and out["sum_currents"][0] == out["sum_currents"][1])
    g.close()
    del d_b, d_o
    return out


def extras(args, ctr, bases, offsets, nk, d_bases, d_offs, s_handle, dev_idx, Counter, synth):
    """Rank 0 at N=1: the full-size CPU baseline with a full bit-compare, the
    end-to-end figures and the exact_counts step."""
    import torch
    out = {}
    k, pool, n_recs = args.k, args.pool, offsets.size - 1
    if not args.no_extras:
        e2e = {}
        # host records -> results (nk_process_parallel: PCIe copy of the input)
        g = Counter(k, 1.0, 0.95, 2, 1.0, pool, True, device=dev_idx)

        def host_run():
            g.reset()
            g.process_parallel_arrays(bases, offsets)
        log("end_to_end: host records")
        best, med = timed(host_run, 3)
        e2e["host_records"] = {"entry": "nk_process_parallel", "s_best": round(best, 5),
                               "s_median": round(med, 5),
                               "mkmers_per_s": round(nk / best / 1e6, 1),
                               "total_spikes": g.energy.total_spikes()}
        # file in the page cache -> results (stream_sequences + process_parallel,
        # src/main.rs:40-46; GPU FASTA ingest)
        with tempfile.TemporaryDirectory(dir="/tmp") as td:
            path = os.path.join(td, "config2.fa")
            synth.write_fasta(path, bases, offsets)
            fsize = os.path.getsize(path)

            def file_run():
                g.reset()
                g.process_file_parallel(path)
            log("end_to_end: FASTA file")
            best, med = timed(file_run, 3)
            e2e["fasta_file"] = {"entry": "nk_process_file_parallel", "file_bytes": fsize,
                                 "s_best": round(best, 5), "s_median": round(med, 5),
                                 "mkmers_per_s": round(nk / best / 1e6, 1),
                                 "gb_per_s": round(fsize / best / 1e9, 2),
                                 "total_spikes": g.energy.total_spikes(),
                                 "same_results": g.top_abundant_neurons(20) == ctr.top_abundant_neurons(20)
                                 and g.energy.total_spikes() == ctr.energy.total_spikes()}
        g.close()
        out["end_to_end"] = e2e
        # the step with the exact k-mer table (counts / get_count / full
        # kmer_per_neuron, src/spiking_hash.rs:157-172): the shim's configuration
        x = Counter(k, 1.0, 0.95, 2, 1.0, pool, True, device=dev_idx, exact_counts=True)

        def exact_step():
            x.reset(s_handle, blocking=False)
            x.process_parallel_device(d_bases.data_ptr(), d_offs.data_ptr(), n_recs, bases.size,
                                      s_handle)
        log("exact_counts step")
        exact_step()
        torch.cuda.synchronize()
        best, med = timed(exact_step, 5)
        out["exact_counts_step"] = {"ms_best": round(best * 1e3, 3), "ms_median": round(med * 1e3, 3),
                                    "mkmers_per_s": round(nk / med / 1e6, 1),
                                    "distinct_kmers": x.distinct_kmers(),
                                    "same_results": x.top_abundant_neurons(20) == ctr.top_abundant_neurons(20)}
        x.close()
        # what the exact table's keys would cost recomputed from the kept
        # records' positions instead of written by K1a<KEYS>
        if k <= 32 and args.kmer_width == 64:  # (the partitioned count's kept records)
            log("key gather diagnostic")
            g_ms, _ = ctr.diag_key_gather(reps=5)
            out["key_gather"] = {"ms_best": round(g_ms, 4), "keys": nk,
                                 "note": "every kept record's key recomputed from (tile, position) "
                                         "and the resident bases (nk_diag_key_gather_ms), no table built"}
    if not args.no_cpu_baseline:
        log("cpu_baseline: oracle process_parallel on the whole input")
        ref, dt, threads = cpu_baseline(bases, offsets, k, pool)
        log(f"cpu_baseline: {dt:.1f} s")
        out["cpu_baseline"] = {
            "value": round(nk / dt / 1e6, 4), "unit": "Mk-mers/s", "cores": threads,
            "host_cpus": os.cpu_count(), "kind": "port", "seconds": round(dt, 3),
            "sample": (f"the whole rank-0 config-2 input ({bases.size:,} bases, {nk:,} k-mers, "
                       f"{n_recs} records, pool {pool:,}, k={k}, canonical): oracle/nk_oracle.c "
                       f"process_parallel restatement, one thread per record like rayon over "
                       f"records (src/spiking_hash.rs:94-95), exact k-mer map, serial merge; the "
                       f"1000-step LIF serial over neurons, run once per distinct count among "
                       f"fresh neurons and reused (a fresh neuron's spikes are a function of its "
                       f"count, oracle/nk_oracle.c:558-592) -- the reference steps every neuron")}
        # SURVEY.md §8d's optional stronger baseline, labelled as such: the same
        # currents and spike counts by chunked threads with no exact k-mer map
        # and a memoised LIF (oracle/nk_oracle.c nko_lean_currents_lif)
        from oracle import cbind
        lt = max(1, min(16, int(os.environ.get("OMP_NUM_THREADS", "16")), os.cpu_count() or 1))
        log(f"cpu_baseline: lean variant on {lt} threads")
        t_l = time.perf_counter()
        l_cur, l_sp, l_tot = cbind.lean_currents_lif(bases, offsets, k, pool, True, 1000, lt)
        dt_l = time.perf_counter() - t_l
        out["cpu_baseline"]["lean"] = {
            "value": round(nk / dt_l / 1e6, 4), "unit": "Mk-mers/s", "cores": lt,
            "seconds": round(dt_l, 3),
            "kind": "lean (NOT the reference's structure): currents + spike counts only",
            "sample": "the same whole rank-0 input: windows split across threads, per-thread u64 "
                      "currents summed, no exact k-mer map, 1000-step LIF memoised by count",
            "same_results": bool(np.array_equal(l_cur, ref.currents())
                                 and np.array_equal(l_sp, ref.spike_counts())
                                 and l_tot == ref.total_spikes)}
        # the timed GPU run's final state (the last step) vs the restatement
        out["parity_full"] = parity(ctr, ref)
        if "exact_counts_step" in out:  # counts.len() of the exact table vs the map
            out["parity_full"]["distinct_kmers"] = [out["exact_counts_step"]["distinct_kmers"],
                                                    ref.distinct_kmers()]
        del ref
    return out


if __name__ == "__main__":
    sys.exit(main())
