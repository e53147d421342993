#!/usr/bin/env python3
"""PMC evidence for bench.py's side lines (configs 3-5): HBM bytes and VALU
instructions of ONE step's count phase (every batch's K1 + K1b + the small
kernels between them) on the side line's own input.

    # the program rocprofv3 runs (no finish, no parity: counts only)
    python tools/pmc_side.py run  --workload config4|config5|config3 [--counts 3]
    # summary of the --pmc passes -> profiles/pmc_<workload>.json
    python tools/pmc_side.py sum  --workload config4 gpurun_out/<dir> profiles/<round dir>

`run` generates the input on the device exactly as bench.py does (config4:
shard 0 of an 8-way split of the 100 Gbase stream; config5: 12.5 Gbases, k=63,
128-bit keys, pool 256 M; config3: the 10 GB FASTQ's 31.6 M reads resident in
HBM, pool 16 M), then runs 1 + counts reset + accumulate_device calls.  `sum`
adds the counters of every nk:: kernel dispatch and divides by the number of
counts (the torch generator kernels and copies are not nk:: kernels).
FETCH_SIZE / WRITE_SIZE are KiB; the gfx950 correction (FETCH_SIZE reports
half the bytes of 16-B-per-lane streaming reads, MI355X_MICROARCH.md HBM) is
applied to every kernel, as for the headline's K1a.
"""
import argparse
import csv
import glob
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def shape_of(workload):
    if workload == "config3":
        return {"reads": 31_645_570, "read_len": 150, "k": 31, "pool": 16_000_000, "width": 64}
    if workload == "config4":
        return {"total": 100_000_000_000, "shard_of": 8, "k": 31, "pool": 2_000_000, "width": 64}
    return {"bases": 12_500_000_000, "k": 63, "pool": 256_000_000, "width": 128}


def make_input(workload, dev):
    import numpy as np
    import torch
    from neurokmer_amd import dist as nkdist, synth
    sh = shape_of(workload)
    if workload == "config3":
        n_b = sh["reads"] * sh["read_len"]
        d_b = torch.zeros(n_b + 16, dtype=torch.uint8, device=dev)
        synth.random_bases_torch(n_b, synth.SEED, 0, dev, out=d_b)
        offs = np.arange(sh["reads"] + 1, dtype=np.uint64) * np.uint64(sh["read_len"])
        return d_b, offs, n_b, sh
    if workload == "config4":
        rec = 115_000_000 // 7
        T = sh["total"]
        n_rec = -(-T // rec)
        glob_o = np.minimum(np.arange(n_rec + 1, dtype=np.int64) * rec, T).astype(np.uint64)
        lo, hi, rel, _ = nkdist.shard_records(glob_o, sh["shard_of"], sh["k"])[0]
        d_b = torch.zeros(hi - lo + 16, dtype=torch.uint8, device=dev)
        synth.random_bases_torch(hi - lo, synth.SEED, lo, dev, out=d_b)
        sh["bases"] = hi - lo
        return d_b, rel.astype(np.uint64), hi - lo, sh
    d_b, offs = synth.make_records_torch(sh["bases"], 7, seed=synth.SEED, repeats_per_mb=64,
                                         motif_len=200, device=dev)
    return d_b, offs, sh["bases"], sh


def run(a):
    import numpy as np
    import torch
    from neurokmer_amd import SpikingKmerCounter
    dev = torch.device("cuda", 0)
    d_b, offs, n_b, sh = make_input(a.workload, dev)
    d_o = torch.from_numpy(offs.view(np.int64)).to(dev)
    c = SpikingKmerCounter(sh["k"], 1.0, 0.95, 2, 1.0, sh["pool"], True, device=0,
                           kmer_width=sh["width"])
    torch.cuda.synchronize()
    for _ in range(1 + a.counts):
        c.reset()
        c.accumulate_device(d_b.data_ptr(), d_o.data_ptr(), offs.size - 1, n_b)
        torch.cuda.synchronize()
    c.close()
    print(json.dumps({"workload": a.workload, "counts": 1 + a.counts, "shape": sh}))


def summarize(a):
    sums = defaultdict(lambda: defaultdict(float))
    calls = defaultdict(lambda: defaultdict(int))
    for path in sorted(glob.glob(os.path.join(a.src, "pmc*", "*counter_collection.csv"))):
        with open(path) as f:
            for r in csv.DictReader(f):
                k = r["Kernel_Name"]
                if "nk::" not in k:
                    continue
                sums[k][r["Counter_Name"]] += float(r["Counter_Value"])
                calls[k][r["Counter_Name"]] += 1
    n = 1 + a.counts
    per = {k: {c: v / n for c, v in d.items()} for k, d in sums.items()}
    tot = defaultdict(float)
    for d in per.values():
        for c, v in d.items():
            tot[c] += v
    os.makedirs(a.dst, exist_ok=True)
    src_json = os.path.join(a.dst, f"pmc_{a.workload}_per_kernel.json")
    with open(src_json, "w") as f:
        json.dump({"per_count": per, "dispatches": {k: dict(v) for k, v in calls.items()}},
                  f, indent=1, sort_keys=True)
    sh = shape_of(a.workload)
    if a.workload == "config4":
        import numpy as np
        from neurokmer_amd import dist as nkdist
        rec = 115_000_000 // 7
        T = sh["total"]
        glob_o = np.minimum(np.arange(-(-T // rec) + 1, dtype=np.int64) * rec, T).astype(np.uint64)
        lo, hi, _, _ = nkdist.shard_records(glob_o, sh["shard_of"], sh["k"])[0]
        sh["bases"] = hi - lo
    out = {"workload": a.workload, "shape": sh, "counts_profiled": n,
           "fetch_size_bytes_raw_per_count": tot.get("FETCH_SIZE", 0.0) * 1024.0,
           "write_size_bytes_per_count": tot.get("WRITE_SIZE", 0.0) * 1024.0,
           "hbm_bytes_per_count": (2.0 * tot.get("FETCH_SIZE", 0.0) + tot.get("WRITE_SIZE", 0.0))
           * 1024.0 if "FETCH_SIZE" in tot and "WRITE_SIZE" in tot else None,
           "valu_instr_per_count": tot.get("SQ_INSTS_VALU"),
           "correction": "gfx950: FETCH_SIZE x2 for 16-B/lane streaming reads (MI355X_MICROARCH.md HBM)",
           "source": os.path.relpath(src_json, ROOT)}
    if a.workload != "config4":
        out["shape"]["bases"] = sh.get("bases", sh.get("reads", 0) * sh.get("read_len", 0))
    with open(os.path.join(ROOT, "profiles", f"pmc_{a.workload}.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=("run", "sum"))
    ap.add_argument("--workload", required=True, choices=("config3", "config4", "config5"))
    ap.add_argument("--counts", type=int, default=2)
    ap.add_argument("src", nargs="?")
    ap.add_argument("dst", nargs="?")
    a = ap.parse_intermixed_args()
    run(a) if a.mode == "run" else summarize(a)
