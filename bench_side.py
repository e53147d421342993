"""Side lines of bench.py: BASELINE.json configs 3-5 at their real per-GPU size.

Each line carries, besides its throughput:
  parity        full-size properties that do not need the CPU restatement
                (sum of currents = N_k, sum of spike counts = total spikes,
                determinism across handles, linearity over record halves or
                file ingest == device-resident records) plus a BIT-EXACT
                compare with the oracle (oracle/nk_oracle.c) on a 115 Mbase
                prefix of the same input;
  cpu_baseline  the oracle timed on that prefix ("prefix-timed");
  roofline      the count phase's algorithmic bytes / its hipEvent duration,
                with the PMC-measured HBM bytes of the same phase
                (profiles/pmc_<workload>.json, tools/pmc_side.py).

Reference semantics: src/spiking_hash.rs:84-201 (process_parallel), :277-486
(process_file_streaming: the LIF rule that steps zero-current neurons too).
"""
from __future__ import annotations

import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
PREFIX_BASES = 115_000_000  # the prefix the oracle checks and is timed on
PREFIX_RECS = 7
HBM_PEAK = 8.0e12
C3_POOL = 16_000_000
C3_READ = 150
C3_READS = 31_645_570  # x 316 B per FASTQ record = 10.0 GB


def log(msg: str) -> None:
    print(f"[bench_side {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def n_kmers(offsets, k: int) -> int:
    lens = np.diff(np.asarray(offsets).astype(np.int64))
    return int(np.clip(lens - k + 1, 0, None).sum())


def host_threads() -> int:
    """CPU threads this process may use (the box's share, not os.cpu_count())."""
    try:
        n = len(os.sched_getaffinity(0))
    except Exception:
        n = os.cpu_count() or 1
    cap = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return max(1, min(n, cap) if cap else n)


class _CAI:
    """A device pointer as a torch-viewable array (no copy)."""

    def __init__(self, ptr, n, typestr="<i8"):
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": typestr,
                                         "data": (ptr, False), "version": 3}


def state_of(c) -> dict:
    return {"currents": c.currents(), "spike_counts": c.spike_counts(),
            "voltages": c.voltages(), "refractory": c.refractory(),
            "total_spikes": c.energy.total_spikes(), "energy_used": c.energy_used(),
            "top20": c.top_abundant_neurons(20)}


def compare(a: dict, b_gpu=None, b_ref=None) -> dict:
    """Bit-compare a GPU state dict with another GPU state dict or with the
    oracle handle (every output the reference exposes)."""
    if b_ref is not None:
        b = {"currents": b_ref.currents(), "spike_counts": b_ref.spike_counts(),
             "voltages": b_ref.voltages(), "refractory": b_ref.refractory(),
             "total_spikes": b_ref.total_spikes, "energy_used": b_ref.energy_used(),
             "top20": b_ref.top_abundant_neurons(20)}
    else:
        b = b_gpu
    out = {
        "currents": bool(np.array_equal(a["currents"], b["currents"])),
        "spike_counts": bool(np.array_equal(a["spike_counts"], b["spike_counts"])),
        "voltages_bitwise": bool(np.array_equal(a["voltages"].view(np.uint32),
                                                b["voltages"].view(np.uint32))),
        "refractory": bool(np.array_equal(a["refractory"], b["refractory"])),
        "total_spikes": [a["total_spikes"], b["total_spikes"]],
        "energy_used": [a["energy_used"], b["energy_used"]],
        "top20_with_uniques": a["top20"] == b["top20"],
    }
    out["all_equal"] = bool(out["currents"] and out["spike_counts"] and out["voltages_bitwise"]
                            and out["refractory"] and out["top20_with_uniques"]
                            and a["total_spikes"] == b["total_spikes"]
                            and a["energy_used"] == b["energy_used"])
    return out


def equal_split(n: int, recs: int) -> np.ndarray:
    q, r = divmod(n, recs)
    lens = np.full(recs, q, np.uint64)
    lens[:r] += 1
    offs = np.zeros(recs + 1, np.uint64)
    np.cumsum(lens, out=offs[1:])
    return offs


def oracle_prefix(hb: np.ndarray, offs: np.ndarray, k: int, pool: int, width: int,
                  streaming: bool):
    """The restatement over the prefix (one thread per record like rayon's
    par_iter over records, or `threads` streaming workers), timed."""
    from oracle import cbind
    ref = cbind.OracleCounter(k, 1.0, 0.95, 2, 1.0, pool, True, width=width)
    threads = host_threads() if streaming else offs.size - 1
    t0 = time.perf_counter()
    if streaming:
        ref.process_streaming_arrays(hb, offs, threads)
    else:
        ref.process_parallel_arrays(hb, offs, threads)
    return ref, time.perf_counter() - t0, threads


# ---------------------------------------------------------------------------
# configs 4 and 5: input resident in HBM, generated on the device
# ---------------------------------------------------------------------------
def side_extras(args, ctr, d_bases, offsets, n_bases, nk, dev_idx) -> dict:
    """After the timed steps: `ctr` holds the last step's final state."""
    import torch
    from neurokmer_amd import SpikingKmerCounter, synth
    k, pool, width = args.k, args.pool, args.kmer_width
    dev = torch.device("cuda", dev_idx)
    n_recs = offsets.size - 1
    par = {}
    t_all = time.perf_counter()
    # -- full size: sums, determinism ------------------------------------
    log("side parity: full-size properties")
    st = state_of(ctr)
    par["sum_currents"] = [int(st["currents"].sum(dtype=np.uint64)), int(nk)]
    par["sum_spike_counts"] = [int(st["spike_counts"].sum(dtype=np.uint64)), st["total_spikes"]]
    par["currents_sha1"] = hashlib.sha1(st["currents"].tobytes()).hexdigest()[:16]
    d_offs = torch.from_numpy(offsets.view(np.int64)).to(dev)
    g = SpikingKmerCounter(k, 1.0, 0.95, 2, 1.0, pool, True, device=dev_idx, kmer_width=width)
    torch.cuda.synchronize()
    g.process_parallel_device(d_bases.data_ptr(), d_offs.data_ptr(), n_recs, n_bases)
    par["determinism_fresh_handle"] = compare(st, state_of(g))["all_equal"]
    # -- linearity: the records in two halves sum to the whole -----------
    m = max(1, n_recs // 2)
    whole = torch.from_numpy(st["currents"].view(np.int64)).to(dev)
    g.accumulate_device(d_bases.data_ptr(), d_offs.data_ptr(), m, int(offsets[m]))
    acc = torch.as_tensor(_CAI(g.device_currents_ptr(), pool), device=dev).clone()
    torch.cuda.synchronize()
    if m < n_recs:
        lo = int(offsets[m])
        sub = d_bases[lo:n_bases + 16]
        if sub.data_ptr() % 16:
            sub = sub.clone()
        o2 = torch.from_numpy((offsets[m:] - offsets[m]).view(np.int64)).to(dev)
        torch.cuda.synchronize()
        g.accumulate_device(sub.data_ptr(), o2.data_ptr(), n_recs - m, n_bases - lo)
        acc += torch.as_tensor(_CAI(g.device_currents_ptr(), pool), device=dev)
        torch.cuda.synchronize()
        del sub
    par["linearity_record_halves"] = bool(torch.equal(acc, whole))
    del acc, whole
    g.close()
    # -- a 115 Mbase prefix, bit-exact against the oracle ----------------
    pn = min(PREFIX_BASES, n_bases)
    p_offs = equal_split(pn, PREFIX_RECS)
    hb = d_bases[:pn].cpu().numpy()
    gen = {}
    if args.workload == "config4":
        ref_b = synth.random_bases(pn, synth.SEED, start=args.shard_lo)
        gen["source"] = f"synth.random_bases(start={args.shard_lo}) on the host"
    else:
        ref_b, _ = synth.make_records(pn, PREFIX_RECS, seed=synth.SEED, repeats_per_mb=64,
                                      motif_len=200)
        gen["source"] = "synth.make_records on the host"
    gen["device_generator_equal"] = bool(np.array_equal(ref_b, hb))
    del ref_b
    log(f"side parity: {pn:,}-base prefix on the GPU and the oracle")
    p = SpikingKmerCounter(k, 1.0, 0.95, 2, 1.0, pool, True, device=dev_idx, kmer_width=width)
    d_po = torch.from_numpy(p_offs.view(np.int64)).to(dev)
    torch.cuda.synchronize()
    p.process_parallel_device(d_bases.data_ptr(), d_po.data_ptr(), PREFIX_RECS, pn)
    ps = state_of(p)
    p.close()
    ref, dt, threads = oracle_prefix(hb, p_offs, k, pool, width, streaming=False)
    log(f"oracle prefix: {dt:.1f} s")
    pk = n_kmers(p_offs, k)
    par["prefix"] = {"bases": pn, "records": PREFIX_RECS, "kmers": pk, **gen,
                     **compare(ps, b_ref=ref)}
    del ref
    par["all_equal"] = bool(par["prefix"]["all_equal"] and gen["device_generator_equal"]
                            and par["sum_currents"][0] == par["sum_currents"][1]
                            and par["sum_spike_counts"][0] == par["sum_spike_counts"][1]
                            and par["determinism_fresh_handle"]
                            and par["linearity_record_halves"])
    par["seconds"] = round(time.perf_counter() - t_all, 1)
    cpu = {"value": round(pk / dt / 1e6, 4), "unit": "Mk-mers/s", "cores": threads,
           "host_cpus": os.cpu_count(), "kind": "port", "seconds": round(dt, 3),
           "sample": (f"prefix-timed: the first {pn:,} bases of this GPU's input as "
                      f"{PREFIX_RECS} records ({pk:,} k-mers, k={k}, kmer_width={width}, "
                      f"pool {pool:,}, canonical): oracle/nk_oracle.c process_parallel, one "
                      f"thread per record like rayon over records, exact k-mer map, 1000-step LIF")}
    return {"parity": par, "cpu_baseline": cpu}


# ---------------------------------------------------------------------------
# config 3: a 10 GB FASTQ streamed from the page cache
# ---------------------------------------------------------------------------
def config3(args) -> int:
    import torch
    sys.path.insert(0, ROOT)
    from neurokmer_amd import SpikingKmerCounter, synth

    k, pool, L = 31, C3_POOL, C3_READ
    n_reads = C3_READS
    dev = torch.device("cuda", 0)
    rec_bytes = synth.FASTQ_HDR + 2 * L + 4
    path = args.fastq or f"/dev/shm/nk_config3_{os.getpid()}.fq"
    made = False
    if not (os.path.exists(path) and os.path.getsize(path) == n_reads * rec_bytes):
        log(f"writing {n_reads:,} reads ({n_reads * rec_bytes / 1e9:.2f} GB) to {path}")
        t0 = time.perf_counter()
        synth.write_fastq_stream(path, 0, n_reads, L, synth.SEED, device=dev)
        made = True
        log(f"written in {time.perf_counter() - t0:.1f} s")
    fsize = os.path.getsize(path)
    nk = n_reads * (L - k + 1)
    try:
        return _config3_run(args, path, fsize, n_reads, nk, k, pool, L, dev, SpikingKmerCounter,
                            synth)
    finally:
        if made and not args.fastq:
            for p in (path, path + ".prefix"):
                if os.path.exists(p):
                    os.unlink(p)


def _config3_run(args, path, fsize, n_reads, nk, k, pool, L, dev, Counter, synth) -> int:
    import torch
    g = Counter(k, 1.0, 0.95, 2, 1.0, pool, True, device=0)
    log("warm-up run")
    g.process_file_streaming(path)
    ts, shas = [], []
    steps = max(1, min(args.steps, 10))
    for i in range(steps):
        g.reset()
        t0 = time.perf_counter()
        g.process_file_streaming(path)
        ts.append(time.perf_counter() - t0)
        if i in (0, steps - 1):
            shas.append(hashlib.sha1(g.currents().tobytes()).hexdigest()[:16])
        log(f"step {i}: {ts[-1] * 1e3:.1f} ms")
    t = float(np.median(ts))
    fst = state_of(g)
    g.close()

    # the same reads resident in HBM: the device-side rate (no file, no PCIe)
    log("resident reads: accumulate + finalize(streaming)")
    n_b = n_reads * L
    d_b = torch.zeros(n_b + 16, dtype=torch.uint8, device=dev)
    synth.random_bases_torch(n_b, synth.SEED, 0, dev, out=d_b)
    offs = np.arange(n_reads + 1, dtype=np.uint64) * np.uint64(L)
    d_o = torch.from_numpy(offs.view(np.int64)).to(dev)
    r = Counter(k, 1.0, 0.95, 2, 1.0, pool, True, device=0)
    # a real stream: torch's default one is handle 0, which the library reads
    # as "the handle's own stream" (the events would then bracket nothing)
    s = torch.cuda.Stream(device=dev)
    cms, tot = [], []
    for i in range(1 + steps):
        r.reset()
        e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
        torch.cuda.synchronize()
        e0.record(s)
        r.accumulate_device(d_b.data_ptr(), d_o.data_ptr(), n_reads, n_b, s.cuda_stream)
        e1.record(s)
        r.finalize(True, s.cuda_stream)
        e2.record(s)
        torch.cuda.synchronize()
        if i:
            cms.append(e0.elapsed_time(e1))
            tot.append(e0.elapsed_time(e2))
    rst = state_of(r)
    r.close()
    # PCIe: pinned host -> device copy of 1 GiB (the file path's H2D leg)
    h = torch.empty(1 << 30, dtype=torch.uint8).pin_memory()
    dd = torch.empty(1 << 30, dtype=torch.uint8, device=dev)
    dd.copy_(h, non_blocking=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        dd.copy_(h, non_blocking=True)
    torch.cuda.synchronize()
    h2d = 3 * (1 << 30) / (time.perf_counter() - t0)
    del h, dd
    # page-cache read rate of the file (one thread, 64 MiB preads)
    t0 = time.perf_counter()
    with open(path, "rb", buffering=0) as f:
        buf = bytearray(64 << 20)
        mv = memoryview(buf)
        while f.readinto(mv):
            pass
    read_gbps = fsize / (time.perf_counter() - t0) / 1e9

    par = {}
    if not args.no_side_parity:
        par["sum_currents"] = [int(fst["currents"].sum(dtype=np.uint64)), nk]
        par["sum_spike_counts"] = [int(fst["spike_counts"].sum(dtype=np.uint64)),
                                   fst["total_spikes"]]
        par["determinism_runs_sha1"] = shas
        par["file_ingest_equals_resident_records"] = compare(fst, rst)["all_equal"]
        # the first 766,667 reads (115 Mbases) as their own FASTQ, bit-exact
        pr = -(-115_000_000 // L)
        ppath = path + ".prefix"
        synth.write_fastq_stream(ppath, 0, pr, L, synth.SEED, device=dev)
        p = Counter(k, 1.0, 0.95, 2, 1.0, pool, True, device=0)
        p.process_file_streaming(ppath)
        ps = state_of(p)
        p.close()
        os.unlink(ppath)
        hb = d_b[:pr * L].cpu().numpy()
        po = offs[:pr + 1].copy()
        log("oracle: streaming restatement on the prefix reads")
        ref, dt, threads = oracle_prefix(hb, po, k, pool, 64, streaming=True)
        log(f"oracle prefix: {dt:.1f} s")
        pk = pr * (L - k + 1)
        gen_ok = bool(np.array_equal(hb[:L * 1000], synth.make_reads(1000, L)[0]))
        par["prefix"] = {"reads": pr, "bases": pr * L, "kmers": pk,
                         "host_generator_equal_first_1000_reads": gen_ok,
                         **compare(ps, b_ref=ref)}
        del ref
        par["all_equal"] = bool(par["prefix"]["all_equal"] and gen_ok
                                and par["file_ingest_equals_resident_records"]
                                and par["sum_currents"][0] == par["sum_currents"][1]
                                and par["sum_spike_counts"][0] == par["sum_spike_counts"][1]
                                and len(set(shas)) == 1)
        cpu = {"value": round(pk / dt / 1e6, 4), "unit": "Mk-mers/s", "cores": threads,
               "host_cpus": os.cpu_count(), "kind": "port", "seconds": round(dt, 3),
               "sample": (f"prefix-timed: the first {pr:,} reads ({pr * L:,} bases, {pk:,} "
                          f"k-mers) of the same FASTQ stream, k=31, pool 16,000,000, canonical: "
                          f"oracle/nk_oracle.c process_file_streaming restatement with "
                          f"{threads} workers, exact k-mer map, 1000-step LIF (streaming rule)")}
    del d_b
    cm = float(np.median(cms))
    alg = n_b + 8 * nk  # resident count: bases read once + one u64 update per k-mer
    pmc = {}
    try:
        with open(os.path.join(ROOT, "profiles", "pmc_config3.json")) as f:
            pmc = json.load(f)
        if pmc.get("shape", {}).get("reads") != n_reads:
            pmc = {}
    except Exception:
        pmc = {}
    out = {
        "metric": "Mk-mers/sec at k=31, pool=16M, 10 GB FASTQ streamed from the page cache",
        "value": round(nk / t / 1e6, 3), "unit": "Mk-mers/s", "n_gpus": 1,
        "steps": steps, "warmup": 1, "ms_per_step": round(t * 1e3, 3),
        "step_ms_all": [round(x * 1e3, 2) for x in ts],
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u64",
        "data": ("synthetic FASTQ in /dev/shm (splitmix64 i.i.d. ACGT, seed 0x4E4B4D52, "
                 "150-bp reads, @r%09d headers, constant quality 'I')"),
        "config": {"workload": (f"config 3: {fsize / 1e9:.2f} GB FASTQ ({n_reads:,} reads x {L} bp, "
                                f"{nk:,} k-mers), k=31, pool_size=16,000,000, --canonical, "
                                f"--streaming (nk_process_file_streaming: host threads read and "
                                f"parse 64 MiB windows, only sequence bytes + record ends cross "
                                f"PCIe, chunked count as they arrive, streaming LIF rule)"),
                   "k": k, "pool_size": pool, "file_bytes": fsize, "reads": n_reads,
                   "kmers": nk, "parallelism": "dp1"},
        "end_to_end": {"file_gb_per_s": round(fsize / t / 1e9, 2),
                       "pcie_h2d_pinned_gb_per_s": round(h2d / 1e9, 2),
                       "page_cache_read_1thread_gb_per_s": round(read_gbps, 2),
                       "resident_step_ms": round(float(np.median(tot)), 3),
                       "resident_mkmers_per_s": round(nk / (float(np.median(tot)) * 1e-3) / 1e6, 1),
                       # what crosses PCIe: the sequence bytes + one 8-B record end per read
                       "pcie_floor_ms": round((n_b + 8 * n_reads) / h2d * 1e3, 1),
                       "pcie_floor_whole_file_ms": round(fsize / h2d * 1e3, 1),
                       "limiter": ("the file path: three stages overlap (16 host threads pread and "
                                   "parse window w+1 of the file, the copy stream moves window w's "
                                   "sequence bytes and record ends up, the device counts them); the "
                                   "host read + parse is the slowest (NK_INGEST_PROFILE=1: the "
                                   "parse wait).  The step is %.1fx the resident count + LIF and "
                                   "%.2fx the PCIe floor of the bytes that cross PCIe (the bases "
                                   "and the record ends: the file is %.1fx the bases, the headers "
                                   "and quality lines stay on the host), so the host's read + "
                                   "parse, not PCIe, sets the step" % (
                                       t * 1e3 / float(np.median(tot)),
                                       t / ((n_b + 8 * n_reads) / h2d), fsize / n_b))},
        "roofline": {"bound": "hbm" if alg / (cm * 1e-3) / HBM_PEAK >= 0.6 else "latency",
                     "kernel": "the resident count of the reads (every batch's K1 + K1b)",
                     "achieved": round(alg / (cm * 1e-3) / 1e9, 2), "peak": HBM_PEAK / 1e9,
                     "unit": "GB/s", "frac": round(alg / (cm * 1e-3) / HBM_PEAK, 4),
                     "traffic": pmc.get("hbm_bytes_per_count"),
                     "traffic_source": pmc.get("source"),
                     "alg_bytes_per_launch": alg, "avg_launch_ms": round(cm, 3),
                     "avg_launch_source": "hipEvents around accumulate_device on its stream, median"},
        "total_spikes": fst["total_spikes"],
    }
    if par:
        out["parity"] = par
        out["cpu_baseline"] = cpu
    print(json.dumps(out), flush=True)
    return 0
