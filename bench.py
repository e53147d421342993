#!/usr/bin/env python3
"""bench.py — NeuroKmer k-mer -> spike hot path on MI355X.

Metric (BASELINE.json): Mk-mers/s at k=31, pool=2M, total spikes bit-exact vs
the CPU reference restatement.  Workload = config 2: 115,000,000 synthetic
bases in 7 records per GPU (weak scaling), k=31, pool_size=2,000,000,
--canonical, in-memory semantics (process_parallel).  One step = reset the
neuron pool, then one full pass of the hot path over the resident input:
tile/record index -> K1 hash+count -> [N>1: RCCL all-reduce of the u64
currents] -> closed-form LIF -> exact top-20 -> unique-k-mer pass for the
top-20 rows [N>1: all-gather of the top k-mer keys].  Inputs are resident in
HBM before the timed region.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402  (import before the HIP library: one shared runtime)
import torch.distributed as dist  # noqa: E402

METRIC = "Mk-mers/sec at k=31, pool=2M; total-spikes bit-exact vs CPU ref"
K = 31
POOL = 2_000_000
BASES = 115_000_000
RECS = 7
HBM_PEAK = 8.0e12  # B/s, MI355X spec (MI355X_MICROARCH.md chip table)


class _CAI:
    """Wraps a raw device pointer for torch.as_tensor (no copy)."""

    def __init__(self, ptr: int, n: int, typestr: str = "<i8"):
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": typestr,
                                         "data": (ptr, False), "version": 3}


def n_kmers(offsets: np.ndarray, k: int) -> int:
    lens = np.diff(offsets.astype(np.int64))
    return int(np.clip(lens - k + 1, 0, None).sum())


# VALU issue cycles per instruction of K1a's mix: the per-k-mer loop body's
# 142 instructions cost 470 issue clocks at the measured gfx950 rates (VOP1/2
# e32 2.45 clk, v_bitop3 2.37, VOP3 4.2; tools/isabench.hip)
K1A_ISSUE_CLK_PER_INSTR = 3.31


def load_pmc():
    """The committed rocprofv3 PMC summary of K1 (profiles/pmc_count_kernel.json):
    HBM bytes per launch, VALU instructions and busy cycles per launch."""
    path = os.path.join(ROOT, "profiles", "pmc_count_kernel.json")
    try:
        with open(path) as f:
            return json.load(f)
    except Exception:
        return {}


def cpu_baseline(bases: np.ndarray, offsets: np.ndarray, per_record: int = 2_000_000,
                 pool: int = POOL):
    """The C restatement of process_parallel (oracle/nk_oracle.c, 'port') on a
    bounded sample of the same workload: the first `per_record` bases of each
    of the 7 records, parallel over records like rayon (src/spiking_hash.rs:
    94-95; 7 threads), exact k-mer map, serial merge, serial 2M-neuron LIF
    (:157-200).  About 10 s of CPU work."""
    from oracle import cbind
    per = int(min(per_record, np.diff(offsets.astype(np.int64)).min()))
    segs = [bases[int(offsets[i]):int(offsets[i]) + per] for i in range(offsets.size - 1)]
    offs = np.zeros(len(segs) + 1, np.uint64)
    np.cumsum([x.size for x in segs], out=offs[1:])
    b = np.concatenate(segs)
    threads = offsets.size - 1  # one rayon work unit per record
    ref = cbind.OracleCounter(K, 1.0, 0.95, 2, 1.0, pool, True)
    t0 = time.perf_counter()
    ref.process_parallel_arrays(b, offs, threads)
    dt = time.perf_counter() - t0
    nk = n_kmers(offs, K)
    return {"rate": nk / dt / 1e6, "seconds": dt, "kmers": nk, "bases": int(offs[-1]),
            "per_record": per, "threads": threads, "ref": ref, "sample": (b, offs)}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--bases", type=int, default=BASES)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--settle", type=float, default=0.25,
                    help="seconds of untimed steps after the warmup (GPU clock settle)")
    # side measurements only (the metric is pool 2M): e.g. config 3's 16 M pool
    ap.add_argument("--pool", type=int, default=POOL)
    ap.add_argument("--k", type=int, default=K)
    ap.add_argument("--kmer-width", type=int, default=64, choices=(64, 128))
    # test-only: rehearse the multi-rank path on a 1-GPU box (gloo, all ranks on cuda:0)
    ap.add_argument("--dist-backend", default="nccl")
    ap.add_argument("--same-device", action="store_true")
    # rehearsal: run the multi-rank step (all-reduce, key all-gather, merge)
    # in a 1-rank process group, to measure its overhead on a 1-GPU box
    ap.add_argument("--force-dist", action="store_true")
    args = ap.parse_args()
    pool = args.pool
    k = args.k

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.same_device:
        local = 0
    dist_on = world > 1 or args.force_dist
    if dist_on:
        torch.cuda.set_device(local)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(args.dist_backend)
    dev = torch.device("cuda", local)

    from neurokmer_amd import SpikingKmerCounter, synth
    from neurokmer_amd import dist as nkdist

    # ---- this rank's shard of the synthetic input (resident in HBM) --------
    bases, offsets = synth.make_records(args.bases, RECS, seed=synth.SEED ^ (rank * 0x9E37),
                                        repeats_per_mb=64, motif_len=200)
    nk = n_kmers(offsets, k)
    d_bases = torch.from_numpy(bases).to(dev)
    d_offs = torch.from_numpy(offsets.view(np.int64)).to(dev)
    torch.cuda.synchronize()

    ctr = SpikingKmerCounter(k, 1.0, 0.95, 2, 1.0, pool, True, device=local,
                             kmer_width=args.kmer_width)

    # one non-default stream for the whole run: the library's kernels, its
    # events and the collectives all go on it (a NULL stream handle would mean
    # the library's own stream)
    run_stream = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(run_stream)
    s_handle = run_stream.cuda_stream

    def step():
        s = s_handle
        ctr.reset(s, blocking=False)
        if not dist_on:
            ctr.process_parallel_device(d_bases.data_ptr(), d_offs.data_ptr(), RECS, bases.size, s)
            return
        ctr.accumulate_device(d_bases.data_ptr(), d_offs.data_ptr(), RECS, bases.size, s)
        # RCCL over xGMI: the currents as u32 (every rank's k-mers together stay
        # below 2^31), then LIF + top-N + this shard's top k-mers into a
        # fixed-size all-gather segment, the union merged on the device: one
        # host synchronisation per step
        nkdist.finalize_step(ctr, total_kmers=world * args.bases)

    per = float("inf")  # fastest warmup step (the first one allocates)
    for _ in range(max(args.warmup, 1 if args.settle > 0 else 0)):
        t_w = time.perf_counter()
        step()
        torch.cuda.synchronize()
        per = min(per, time.perf_counter() - t_w)
    # clock settle: the GPU reaches its sustained clock only after ~10-30 ms of
    # load (5 timed steps straight after 2 warmup steps run ~15% slower), so
    # untimed steps continue for about --settle seconds; every rank runs the
    # same number (the steps contain collectives).  Reported as "settle_steps".
    settle = 0
    if args.settle > 0:
        settle = min(int(args.settle / max(per, 1e-4)) + 1, 5000)
        if dist_on:
            t = torch.tensor([settle], dtype=torch.int64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            settle = int(t.item())
        for _ in range(settle):
            step()
        torch.cuda.synchronize()
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize()
    marks = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
        marks.append(time.perf_counter())  # host view: each step ends with its readback
    torch.cuda.synchronize()
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if dist_on:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())

    # K1's hipEvent times of every timed step (a ring of event pairs in the
    # library, read after the loop so no event query sits in the timed region)
    count_ms = ctr.count_history(args.steps)
    timings = ctr.last_timings()
    total_spikes = ctr.energy.total_spikes()
    top = ctr.top_abundant_neurons(20)

    if rank == 0:
        ms_step = dt / args.steps * 1e3
        value = world * nk / (dt / args.steps) / 1e6
        # roofline of the dominant kernel (K1: hash + count), algorithmic bytes
        # per launch = input bases read once + one 8-B counter update per k-mer
        c_ms = [x for x in count_ms if x is not None and x == x and x > 0]
        k1_ms = float(np.mean(c_ms)) if c_ms else timings.get("count", float("nan"))
        alg_bytes = bases.size + 8 * nk
        achieved = alg_bytes / (k1_ms * 1e-3)
        pmc = load_pmc()
        traffic, traffic_src = pmc.get("hbm_bytes_per_launch"), pmc.get("source")
        valu = None
        if pmc.get("valu_instr_per_launch") and pmc.get("sclk_ghz") and pmc.get("pmc_launch_ns"):
            # K1a is VALU-issue bound: issue cycles its instructions need per SIMD
            # (1024 SIMDs) vs the cycles the launch took (PMC GRBM_GUI_ACTIVE)
            busy = pmc["sclk_ghz"] * pmc["pmc_launch_ns"]  # cycles per launch
            need = pmc["valu_instr_per_launch"] / 1024.0 * K1A_ISSUE_CLK_PER_INSTR
            valu = {"instr_per_launch": pmc["valu_instr_per_launch"],
                    "issue_clk_per_instr": K1A_ISSUE_CLK_PER_INSTR,
                    "busy_cycles_per_launch": round(busy),
                    "issue_frac": round(need / busy, 4),
                    "sclk_ghz_live": round(busy / (k1_ms * 1e6), 3),
                    "source": traffic_src}
        out = {
            "metric": METRIC, "value": round(value, 3), "unit": "Mk-mers/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "settle_steps": settle,
            "ms_per_step": round(ms_step, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u64",
            "data": "synthetic (splitmix64 i.i.d. ACGT, seed 0x4E4B4D52^rank, 64x200-bp planted "
                    "repeats per MB)",
            "config": {"workload": (f"config 2: {bases.size:,} bases in 7 records per GPU, k={k}, "
                                    f"pool_size={pool:,}, --canonical, process_parallel"),
                       "k": k, "kmer_width": args.kmer_width, "pool_size": pool, "bases_per_gpu": int(bases.size),
                       "records_per_gpu": RECS, "kmers_per_gpu": nk,
                       "parallelism": f"dp{world}"},
            "roofline": {"bound": "hbm", "kernel": "k_part<canonical> (K1a)",
                         "achieved": round(achieved / 1e9, 2), "peak": HBM_PEAK / 1e9,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK, 4),
                         "traffic": traffic, "traffic_source": traffic_src,
                         "alg_bytes_per_launch": alg_bytes, "avg_launch_ms": round(k1_ms, 4),
                         "launches_timed": len(c_ms), "valu": valu},
            "stage_ms": {k2: round(v, 4) for k2, v in timings.items()},
            "step_ms_host": [round((b - a) * 1e3, 4) for a, b in zip([t0] + marks[:-1], marks)],
            "k1_ms_steps": [round(x, 4) for x in count_ms],
            "total_spikes": total_spikes,
        }
        if world == 1 and not args.no_cpu_baseline and k == K and args.kmer_width == 64:
            cb = cpu_baseline(bases, offsets, pool=pool)
            # parity on the same sample: GPU vs the restatement, bit-exact
            sb, so = cb["sample"]
            g = SpikingKmerCounter(K, 1.0, 0.95, 2, 1.0, pool, True, device=local)
            g.process_parallel_arrays(sb, so)
            ref = cb["ref"]
            parity = {
                "sample_bases": int(so[-1]),
                "currents": bool(np.array_equal(g.currents(), ref.currents())),
                "spike_counts": bool(np.array_equal(g.spike_counts(), ref.spike_counts())),
                "voltages_bitwise": bool(np.array_equal(g.voltages().view(np.uint32),
                                                        ref.voltages().view(np.uint32))),
                "total_spikes": [g.energy.total_spikes(), ref.total_spikes],
                "top20": g.top_abundant_neurons(20) == ref.top_abundant_neurons(20),
            }
            g.close()
            out["cpu_baseline"] = {
                "value": round(cb["rate"], 4), "unit": "Mk-mers/s", "cores": cb["threads"],
                "kind": "port",
                "sample": f"first {cb['per_record']} bases of each of the {RECS} records of "
                          f"rank 0's workload ({cb['bases']} bases, {cb['kmers']} k-mers, "
                          f"pool {pool:,}, k=31, canonical) in {cb['seconds']:.2f} s: oracle/nk_oracle.c "
                          f"process_parallel restatement (parallel over records, exact k-mer "
                          f"map, serial merge and 1000-step LIF)"}
            out["parity_on_cpu_sample"] = parity
        print(json.dumps(out), flush=True)
    ctr.close()
    if dist_on:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
