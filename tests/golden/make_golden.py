"""Generates the committed golden fixtures under tests/golden/ from the pure-Python
restatement (oracle/pyref.py) only, so they are independent of the C oracle and
of the GPU code.  Re-run:  python tests/golden/make_golden.py

Pinning: the reference (Rust) cannot be built or imported in this image and
ships no fixtures; the SipHash core in pyref is pinned by published vectors and
by CPython's hash(bytes) (tests/test_oracle.py).  These fixtures freeze the
restatement's outputs so any later change to either oracle or to the GPU path
is caught.
"""
from __future__ import annotations

import json
import zlib
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from neurokmer_amd import synth  # noqa: E402
from oracle import pyref  # noqa: E402


def sip_kats():
    ms = [0, 1, 2, 3, 0xFF, 0x100, 0xDEADBEEF, 2**32 - 1, 2**32, 2**63, 2**64 - 1,
          0x0123456789ABCDEF, 0xAAAAAAAAAAAAAAAA]
    ms += [int(w) for w in synth.random_words(24, seed=77)]
    return [{"m": m, "sip13": pyref.sip13_u64(m)} for m in ms]


def key_cases():
    bases, offs = synth.make_records(3000, 1, seed=5, n_rate=0.01, mixed_case=True)
    seq = bases.tobytes()
    out = []
    for k in (1, 5, 21, 31, 32, 33, 63):
        for canon in (False, True):
            out.append({"k": k, "canonical": canon,
                        "keys": pyref.kmer_keys(seq[:600], k, canon)})
    return {"seq": seq[:600].decode("latin-1"), "cases": out}


def lif_table():
    rows = []
    for count in list(range(0, 1201)) + [1500, 2000, 5000, 10**4, 10**5, 10**6, 2**40]:
        v, r, sp = pyref.lif_run(count, 1000, 1.0, 0.95, 2, True)
        rows.append([count, sp, pyref.f32_bits(v), r])
    return rows


def width128():
    """--kmer-width=128 (the build's own mode): SipHash-1-3 over
    16-byte keys, key derivation cases and one small end-to-end case, all from
    oracle/pyref.py's per-window restatement."""
    ks = [0, 1, 2**64 - 1, 2**64, 2**64 + 1, 2**127, 2**128 - 1,
          0x0123456789ABCDEF_FEDCBA9876543210]
    ks += [int(a) | (int(b) << 64) for a, b in zip(synth.random_words(12, seed=78),
                                                 synth.random_words(12, seed=79))]
    kats = [{"key": str(k), "sip13": pyref.sip13_u128(k)} for k in ks]
    bases, offs = synth.make_records(2000, 1, seed=6, n_rate=0.01, mixed_case=True)
    seq = bases.tobytes()[:400]
    cases = []
    for k in (1, 21, 32, 33, 47, 63, 64):
        for canon in (False, True):
            cases.append({"k": k, "canonical": canon,
                          "keys": [str(x) for x in pyref.kmer_keys128(seq, k, canon)]})
    # end to end: currents, LIF (steps 1000), top-20 with distinct keys per neuron
    k, pool = 63, 701
    eb, eo = synth.make_records(9000, 3, seed=8, repeats_per_mb=40000, motif_len=90,
                                n_rate=0.002)
    recs = synth.records_list(eb, eo)
    cur = [0] * pool
    distinct = [set() for _ in range(pool)]
    for r in recs:
        for key in pyref.kmer_keys128(r, k, True):
            i = pyref.sip13_u128(key) % pool
            cur[i] += 1
            distinct[i].add(key)
    sc, vb, rr = [], [], []
    for c in cur:
        v, r_, sp = pyref.lif_run(c, 1000, 1.0, 0.95, 2, True)
        sc.append(sp); vb.append(pyref.f32_bits(v)); rr.append(r_)
    order = sorted(range(pool), key=lambda i: (-sc[i], i))[:20]
    e2e128 = {"k": k, "pool": pool, "canonical": True,
              "records": [x.decode("latin-1") for x in recs], "currents": cur,
              "spike_counts": sc, "voltage_bits": vb, "refractory": rr,
              "total_spikes": sum(sc),
              "top20": [[i, sc[i], len(distinct[i])] for i in order]}
    return {"sip13_u128": kats, "seq": seq.decode("latin-1"), "cases": cases, "e2e": e2e128}


CASES = [
    # name, total bases, records, k, pool, canonical, streaming, extra synth kwargs, steps
    ("noncanon_k21_p1000", 4000, 5, 21, 1000, False, False, dict(n_rate=0.01, mixed_case=True), None),
    ("canon_k31_p500_repeats", 12000, 3, 31, 500, True, False, dict(repeats_per_mb=20000, motif_len=80), None),
    ("canon_k5_p97", 3000, 4, 5, 97, True, False, dict(n_rate=0.005), None),
    ("canon_k33_p300_compat", 6000, 3, 33, 300, True, False, dict(repeats_per_mb=10000, motif_len=60), None),
    ("noncanon_k63_p100", 5000, 2, 63, 100, False, False, dict(n_rate=0.01, mixed_case=True), None),
    ("canon_k21_p400_streaming", 8000, 6, 21, 400, True, True, dict(repeats_per_mb=30000, motif_len=40), None),
    ("canon_k11_p50_steps5000", 6000, 2, 11, 50, True, False, dict(repeats_per_mb=5000, motif_len=30), 5000),
]


def e2e(name, total, nrec, k, pool, canon, streaming, kw, steps):
    bases, offs = synth.make_records(total, nrec, seed=zlib.crc32(name.encode()) & 0xFFFF, **kw)
    seqs = synth.records_list(bases, offs)
    seqs.insert(1, b"")            # empty record
    seqs.insert(2, b"ACGTN"[:max(1, min(5, k - 1))])  # record shorter than k
    c = pyref.SpikingKmerCounter(k, 1.0, 0.95, 2, 1.0, pool, canon)
    if steps is not None:
        c.steps = steps
    (c.process_streaming if streaming else c.process_parallel)(seqs)
    return {
        "name": name, "k": k, "pool": pool, "canonical": canon, "streaming": streaming,
        "steps": c.steps, "records": [s.decode("latin-1") for s in seqs],
        "currents": c.currents, "spike_counts": c.sc,
        "voltage_bits": [pyref.f32_bits(v) for v in c.v], "refractory": c.r,
        "total_spikes": c.total_spikes, "total_energy_fixed": c.total_energy,
        "top20": [list(t) for t in c.top_abundant_neurons(20)],
        "distinct_kmers": len(c.counts),
        "stdout_block": pyref.cli_result_block(c, pool, streaming),
    }


def main():
    json.dump(sip_kats(), open(os.path.join(HERE, "sip13_kat.json"), "w"))
    json.dump(key_cases(), open(os.path.join(HERE, "kmer_keys.json"), "w"))
    json.dump(lif_table(), open(os.path.join(HERE, "lif_table_default.json"), "w"))
    json.dump(width128(), open(os.path.join(HERE, "width128.json"), "w"))
    for case in CASES:
        json.dump(e2e(*case), open(os.path.join(HERE, f"e2e_{case[0]}.json"), "w"))
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    main()
