#!/usr/bin/env python3
"""End-to-end file throughput: FASTA / FASTQ on disk (page cache) -> result.

    python tools/ingest_bench.py [--gbases 1.0] [--reps 3]

Writes synthetic files under $TMPDIR, then times the GPU FASTX ingest
(nk_process_file_parallel / nk_process_file_streaming: chunked device parse +
count as the chunks arrive) against the host reader + nk_process_parallel of
the same records.  Prints one JSON line per case.  Not the metric (bench.py):
this is the §8f-2 path's own number.
"""
import argparse
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401  (one shared HIP runtime)

from neurokmer_amd import SpikingKmerCounter, synth  # noqa: E402
from neurokmer_amd import _lib  # noqa: E402


def n_kmers(offs, k):
    lens = np.diff(offs.astype(np.int64))
    return int(np.maximum(lens - k + 1, 0).sum())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gbases", type=float, default=1.0)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    tmp = tempfile.mkdtemp(prefix="nk_ingest_")
    nb = int(a.gbases * 1e9)
    k, pool = 31, 2_000_000
    out = []
    bases, offs = synth.make_records(nb, 7, repeats_per_mb=64, motif_len=200)
    fa = os.path.join(tmp, "in.fa")
    synth.write_fasta(fa, bases, offs, width=60)
    nk_fa = n_kmers(offs, k)
    del bases
    rb, ro = synth.make_reads(nb // 150, 150, seed=11)
    fq = os.path.join(tmp, "in.fq")
    synth.write_fastq(fq, rb, ro)
    nk_fq = n_kmers(ro, k)
    del rb
    for name, path, nk, streaming in (("fasta", fa, nk_fa, False), ("fastq", fq, nk_fq, True)):
        size = os.path.getsize(path)
        c = SpikingKmerCounter(k, 1.0, 0.95, 2, 1.0, pool, True)
        run = c.process_file_streaming if streaming else c.process_file_parallel
        run(path)  # warm-up (page cache, allocations)
        ts = []
        for _ in range(a.reps):
            c.reset()
            t0 = time.perf_counter()
            run(path)
            ts.append(time.perf_counter() - t0)
        t = min(ts)
        # host reader + host-array process_parallel (the previous path)
        recs = list(__import__("neurokmer_amd.fastx", fromlist=["x"]).stream_sequences(path)) \
            if size < (3 << 30) else None
        th = None
        if recs is not None:
            hb = np.frombuffer(b"".join(recs), np.uint8)
            ho = np.zeros(len(recs) + 1, np.uint64)
            np.cumsum([len(r) for r in recs], out=ho[1:])
            c.reset()
            t0 = time.perf_counter()
            L = _lib.load()
            import ctypes as C
            rc = L.nk_process_parallel(c._h, hb.ctypes.data_as(C.c_void_p),
                                       ho.ctypes.data_as(C.c_void_p), len(recs))
            th = time.perf_counter() - t0 if rc == 0 else None
        out.append({"case": name, "file_bytes": size, "kmers": nk,
                    "gpu_ingest_s": round(t, 4), "gpu_ingest_GBps": round(size / t / 1e9, 2),
                    "gpu_ingest_Mkmers_s": round(nk / t / 1e6, 1),
                    "host_arrays_process_s": round(th, 4) if th else None})
        print(json.dumps(out[-1]), flush=True)
    for p in (fa, fq):
        os.remove(p)


if __name__ == "__main__":
    main()
