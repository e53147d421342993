"""CPU tests: pin the oracle (both restatements) and the device algorithms'
math against published vectors, CPython, golden fixtures and brute force.

Pins available for this path: the reference ships no fixtures
and cannot be built (Rust) here.  SipHash is pinned by the SipHash paper's
vectors and by CPython 3.10's hash(bytes) (SipHash-2-4, zero key under
PYTHONHASHSEED=0); SipHash-1-3 differs only in round counts.  Everything else
is pinned by the two independent restatements agreeing, and frozen by the
fixtures in tests/golden/ (tests/golden/make_golden.py).
"""
import glob
import json
import os
import random
import struct
import subprocess
import sys

import numpy as np
import pytest

from neurokmer_amd import synth
from oracle import cbind, pyref

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
K00_0F = (int.from_bytes(bytes(range(8)), "little"), int.from_bytes(bytes(range(8, 16)), "little"))


@pytest.mark.parametrize("impl", ["py", "c"])
def test_siphash24_paper_vectors(impl):
    f = pyref.siphash if impl == "py" else cbind.siphash
    assert f(2, 4, *K00_0F, b"") == 0x726FDB47DD0E0E31
    assert f(2, 4, *K00_0F, bytes(range(15))) == 0xA129CA6149BE45E5


def test_siphash24_matches_cpython_hash():
    msgs = [b"", b"a", b"abc", bytes(range(7)), bytes(range(8)), bytes(range(9)),
            bytes(range(16)), bytes(range(31)), bytes(range(64))]
    rng = random.Random(3)
    msgs += [bytes(rng.getrandbits(8) for _ in range(rng.randrange(1, 40))) for _ in range(40)]
    msgs += [m.to_bytes(8, "little") for m in (0, 1, 2**63, 2**64 - 1, 0xDEADBEEF)]
    code = ("import sys,json;ms=[bytes.fromhex(h) for h in json.load(sys.stdin)];"
            "print(json.dumps([hash(m) for m in ms]))")
    env = dict(os.environ, PYTHONHASHSEED="0")
    out = subprocess.run([sys.executable, "-c", code], input=json.dumps([m.hex() for m in msgs]),
                         capture_output=True, text=True, env=env, check=True).stdout
    for m, h in zip(msgs, json.loads(out)):
        if not m:
            continue  # CPython defines hash(b"") = 0
        want = h & (2**64 - 1)
        got_py = pyref.siphash(2, 4, 0, 0, m)
        got_c = cbind.siphash(2, 4, 0, 0, m)
        if got_py == 2**64 - 1:
            continue  # CPython maps -1 to -2
        assert got_py == want and got_c == want, m


def test_sip13_kat_golden():
    for row in json.load(open(os.path.join(GOLD, "sip13_kat.json"))):
        assert pyref.sip13_u64(row["m"]) == row["sip13"]
        assert cbind.sip13_u64(row["m"]) == row["sip13"]
    assert pyref.sip13_u64(0) == 0xBD60ACB658C79E45  # SURVEY.md §8c recorded value


def test_kmer_keys_golden():
    g = json.load(open(os.path.join(GOLD, "kmer_keys.json")))
    seq = g["seq"].encode("latin-1")
    for case in g["cases"]:
        got = cbind.kmer_keys(seq, case["k"], case["canonical"])
        assert [int(x) for x in got] == case["keys"], (case["k"], case["canonical"])
        assert pyref.kmer_keys(seq, case["k"], case["canonical"]) == case["keys"]


def test_lif_golden_table():
    for count, sp, vbits, r in json.load(open(os.path.join(GOLD, "lif_table_default.json"))):
        v, rr, s = cbind.lif(count, 1000, 1.0, 0.95, 2, True)
        assert (s, pyref.f32_bits(v), rr) == (sp, vbits, r), count
        v2, r2, s2 = lif_closed(count, 1000, 1.0, 0.95, 2, 0.0, 0)
        assert (s2, pyref.f32_bits(v2), r2) == (sp, vbits, r), count


class _View:
    """Duck-typed counter for pyref.cli_result_block from C-oracle results."""

    def __init__(self, c, top):
        self.total_spikes = c.total_spikes
        self._e = c.energy_used()
        self._top = top

    def top_abundant_neurons(self, n):
        return self._top[:n]

    def energy_used(self):
        return self._e


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLD, "e2e_*.json"))),
                         ids=lambda p: os.path.basename(p)[4:-5])
def test_e2e_golden(path):
    g = json.load(open(path))
    seqs = [s.encode("latin-1") for s in g["records"]]
    c = cbind.OracleCounter(g["k"], 1.0, 0.95, 2, 1.0, g["pool"], g["canonical"])
    c.set_steps(g["steps"])
    (c.process_streaming if g["streaming"] else c.process_parallel)(seqs, 2)
    assert [int(x) for x in c.currents()] == g["currents"]
    assert [int(x) for x in c.spike_counts()] == g["spike_counts"]
    assert [int(x) for x in c.voltages().view(np.uint32)] == g["voltage_bits"]
    assert [int(x) for x in c.refractory()] == g["refractory"]
    assert c.total_spikes == g["total_spikes"]
    assert c.total_energy_fixed == g["total_energy_fixed"]
    top = c.top_abundant_neurons(20)
    assert [list(t) for t in top] == g["top20"]
    assert c.distinct_kmers() == g["distinct_kmers"]
    assert pyref.cli_result_block(_View(c, top), g["pool"], g["streaming"]) == g["stdout_block"]


@pytest.mark.parametrize("seed", range(6))
def test_c_and_python_restatements_agree(seed):
    rng = random.Random(seed)
    k = rng.choice([1, 3, 9, 16, 21, 31, 32, 33, 47, 64])
    canon = rng.random() < 0.5
    pool = rng.choice([1, 13, 257, 3001])
    thr, leak, refr = rng.choice([(1.0, 0.95, 2), (0.3, 0.9, 0), (2.0, 1.0, 3)])
    bases, offs = synth.make_records(rng.randrange(500, 5000), rng.randrange(1, 6), seed=seed,
                                     n_rate=0.01, mixed_case=True,
                                     repeats_per_mb=rng.choice([0, 20000]), motif_len=40)
    seqs = synth.records_list(bases, offs)
    streaming = rng.random() < 0.5
    p = pyref.SpikingKmerCounter(k, thr, leak, refr, 1.0, pool, canon)
    c = cbind.OracleCounter(k, thr, leak, refr, 1.0, pool, canon)
    for _ in range(2):  # state carries across calls
        (p.process_streaming if streaming else p.process_parallel)(seqs)
        (c.process_streaming if streaming else c.process_parallel)(seqs, 3)
    assert [int(x) for x in c.currents()] == p.currents
    assert [int(x) for x in c.spike_counts()] == p.sc
    assert [int(x) for x in c.voltages().view(np.uint32)] == [pyref.f32_bits(v) for v in p.v]
    assert [int(x) for x in c.refractory()] == p.r
    assert c.total_spikes == p.total_spikes
    assert c.top_abundant_neurons(20) == p.top_abundant_neurons(20)


@pytest.mark.parametrize("seed", range(4))
def test_simulate_spikes_auto_restatements_agree(seed):
    """simulate_spikes_auto (src/spiking_hash.rs:697-714 -> :544-659) after a
    process call, repeated, with zero-current neurons stepping too; the C and
    Python restatements agree bit for bit (steps 0 leaves everything alone)."""
    rng = random.Random(100 + seed)
    k = rng.choice([5, 17, 31, 40])
    canon = rng.random() < 0.5
    pool = rng.choice([7, 257, 3001])
    thr, leak, refr = rng.choice([(1.0, 0.95, 2), (0.0, 0.9, 1), (0.02, 1.0, 0)])
    bases, offs = synth.make_records(rng.randrange(500, 4000), rng.randrange(1, 5), seed=seed,
                                     n_rate=0.01, repeats_per_mb=20000, motif_len=40)
    seqs = synth.records_list(bases, offs)
    p = pyref.SpikingKmerCounter(k, thr, leak, refr, 1.0, pool, canon)
    c = cbind.OracleCounter(k, thr, leak, refr, 1.0, pool, canon)
    for steps in (1000, 0, 37):
        p.steps = steps
        c.set_steps(steps)
        if seed % 2:
            p.process_parallel(seqs)
            c.process_parallel(seqs, 2)
        p.simulate_spikes_auto()
        c.simulate_spikes_auto()
        p.simulate_spikes_auto()
        c.simulate_spikes_auto()
        assert [int(x) for x in c.currents()] == p.currents
        assert [int(x) for x in c.spike_counts()] == p.sc
        assert [int(x) for x in c.voltages().view(np.uint32)] == [pyref.f32_bits(v) for v in p.v]
        assert [int(x) for x in c.refractory()] == p.r
        assert c.total_spikes == p.total_spikes
        assert c.top_abundant_neurons(20) == p.top_abundant_neurons(20)


# ---------------------------------------------------------------------------
# CPU models of the device algorithms (neurokmer_amd/csrc/nk_device.h)
# ---------------------------------------------------------------------------
f32 = pyref.f32


def _sip_device_model(blocks):
    """neurokmer_amd/csrc/nk_device.h's SipHash-1-3 (key 0): the message
    blocks, then the length block, two finalisation rounds and the fused last
    round, whose v0 cancels out of the output (sip_last_round_out)."""
    M = pyref.M64
    rot = pyref._rotl
    v = [0x736f6d6570736575, 0x646f72616e646f6d, 0x6c7967656e657261, 0x7465646279746573]

    def rnd():
        v[0] = (v[0] + v[1]) & M; v[1] = rot(v[1], 13) ^ v[0]; v[0] = rot(v[0], 32)
        v[2] = (v[2] + v[3]) & M; v[3] = rot(v[3], 16) ^ v[2]
        v[0] = (v[0] + v[3]) & M; v[3] = rot(v[3], 21) ^ v[0]
        v[2] = (v[2] + v[1]) & M; v[1] = rot(v[1], 17) ^ v[2]; v[2] = rot(v[2], 32)
    for m in blocks + [(8 * len(blocks)) << 56]:
        v[3] ^= m
        rnd()
        v[0] ^= m
    v[2] ^= 0xFF
    rnd()
    rnd()
    v0, v1, v2, v3 = v
    v0 = (v0 + v1) & M; v1 = rot(v1, 13) ^ v0
    v2 = (v2 + v3) & M; v3 = rot(v3, 16) ^ v2
    v3 = rot(v3, 21)
    v2 = (v2 + v1) & M; v1 = rot(v1, 17)
    x = (v2 ^ (v2 >> 32)) & 0xFFFFFFFF
    lo = (v1 ^ v3 ^ x) & 0xFFFFFFFF
    hi = ((v1 >> 32) ^ (v3 >> 32) ^ x) & 0xFFFFFFFF
    return (hi << 32) | lo


def test_sip13_last_round_model():
    """The device's fused last round equals full SipHash-1-3 (u64 and u128 keys)."""
    rng = random.Random(13)
    vals = [0, 1, M64 := (1 << 64) - 1, 1 << 63] + [rng.getrandbits(64) for _ in range(3000)]
    for m in vals:
        assert _sip_device_model([m]) == cbind.sip13_u64(m) == pyref.sip13_u64(m)
    for _ in range(1000):
        key = rng.getrandbits(126)
        assert _sip_device_model([key & M64, key >> 64]) == cbind.sip13_u128(key)


def lif_step(v, leak, c):
    return f32(f32(v * leak) + c)


def lif_closed(count, steps, thr, leak, refr, v, r):
    """Line-for-line model of nk::lif_closed (nk_device.h)."""
    thr, leak = f32(thr), f32(leak)
    c = f32(float(count) / float(steps)) if steps else float("inf")
    t = 0
    spikes = 0
    d = min(r, steps)
    r -= d
    t += d
    fired = False
    while t < steps:
        t += 1
        nv = lif_step(v, leak, c)
        if nv >= thr:
            v, r, spikes, fired = 0.0, refr, 1, True
            break
        if nv == v:
            v = nv
            t = steps
            break
        v = nv
    if not fired or t == steps:
        return v, r, spikes
    remaining = steps - t
    if remaining <= refr:
        return v, refr - remaining, spikes
    avail = remaining - refr
    x, m, fires = 0.0, 0, False
    while m < avail:
        m += 1
        nx = lif_step(x, leak, c)
        if nx >= thr:
            fires = True
            break
        if nx == x:
            x = nx
            break
        x = nx
    if not fires:
        return x, 0, spikes
    period = refr + m
    n = remaining // period
    spikes += n
    rem = remaining - n * period
    if rem <= refr:
        return 0.0, refr - rem, spikes
    y = 0.0
    for _ in range(rem - refr):
        y = lif_step(y, leak, c)
    return y, 0, spikes


def test_lif_closed_form_matches_brute_force():
    rng = random.Random(11)
    params = [(1.0, 0.95, 2), (0.5, 1.0, 0), (0.0, 0.95, 2), (1.0, 0.0, 5), (3.0, 0.99, 1),
              (1.0, 0.95, 1000), (0.7, 0.5, 3)]
    for _ in range(600):
        thr, leak, refr = rng.choice(params)
        steps = rng.choice([0, 1, 2, 7, 100, 1000, 2500])
        count = rng.choice([0, 1, 50, 51, 57, 100, 999, 1000, 1001, rng.randrange(0, 5000)])
        v0 = rng.choice([0.0, 0.0, f32(rng.random()), f32(rng.random() * 3)])
        r0 = rng.choice([0, 0, 1, 2, 7])
        want = pyref.lif_run(count, steps, thr, leak, refr, False, v0, r0, 0)
        got = lif_closed(count, steps, thr, leak, refr, v0, r0)
        assert (pyref.f32_bits(got[0]), got[1], got[2]) == \
               (pyref.f32_bits(want[0]), want[1], want[2]), (count, steps, thr, leak, refr, v0, r0)


def fastmod32(h, p):
    """Model of nk::fastmod32 (32-bit result, P < 2^30)."""
    magic = (2**64 - 1) // p
    h0, h1, m0, m1 = h & 0xFFFFFFFF, h >> 32, magic & 0xFFFFFFFF, magic >> 32
    ahi = (h0 * m0) >> 32
    mid = (h1 * m0 + ahi) & (2**64 - 1)
    mid = (h0 * m1 + mid) & (2**64 - 1)
    qlo = (h1 * m1 + (mid >> 32)) & 0xFFFFFFFF
    r = (h0 - qlo * p) & 0xFFFFFFFF
    return min(r, (r - p) & 0xFFFFFFFF)  # q = floor(h/P) - {0, 1}: one correction


def test_fastmod32_model():
    rng = random.Random(5)
    for p in (1, 2, 3, 7, 64, 100_003, 2_000_000, 8_388_608, 16_000_000, (1 << 30) - 1):
        vals = [0, 1, p - 1, p, 2**64 - 1, ((2**64 - 1) // p) * p, ((2**64 - 1) // p) * p - 1]
        vals += [rng.getrandbits(64) for _ in range(3000)]
        # near multiples of P across the range, where q's error is largest
        for _ in range(300):
            m = rng.getrandbits(64) // p
            vals += [m * p + d for d in (-1, 0, 1, p - 1) if 0 <= m * p + d < 2**64]
        for h in vals:
            assert fastmod32(h, p) == h % p, (h, p)


def _streams(seq: bytes):
    """Model of nk_tile.h conv4: forward codes MSB-first, complement codes
    LSB-first, invalid-byte bits, as Python ints over the whole sequence."""
    F = 0
    R = 0
    inv = 0
    for i, b in enumerate(seq):
        t = b | 0x20
        valid = t in (0x61, 0x63, 0x67, 0x74)
        code = ((b >> 1) ^ (b >> 2)) & 3 if valid else 0
        comp = (code ^ 3) if valid else 0
        F = (F << 2) | code
        R |= comp << (2 * i)
        inv |= (0 if valid else 1) << i
    return F, R, inv


def test_device_window_model_matches_reference():
    """The device extracts fwd/rev from the bit streams (first window) and rolls
    15 more from code words; model both against the reference's keys."""
    for seed in range(4):
        bases, _ = synth.make_records(700, 1, seed=seed, n_rate=0.02, mixed_case=True)
        seq = bases.tobytes()
        n = len(seq)
        F, R, inv = _streams(seq)
        for k in (1, 2, 5, 16, 17, 21, 31, 32):
            mask = (1 << (2 * k)) - 1
            for canon in (True, False):
                want = pyref.kmer_keys(seq, k, canon)
                for q0 in range(0, n - k + 1, 16):
                    fwd = (F >> (2 * (n - q0 - k))) & mask
                    rev = (R >> (2 * q0)) & mask
                    for j in range(16):
                        q = q0 + j
                        if q + k > n:
                            break
                        if j:
                            c = (F >> (2 * (n - (q + k - 1) - 1))) & 3
                            cc = (R >> (2 * (q + k - 1))) & 3
                            fwd = ((fwd << 2) | c) & mask
                            rev = (rev >> 2) | (cc << (2 * k - 2))
                        if canon:
                            key = min(fwd, rev)
                        elif (inv >> q) & ((1 << k) - 1):
                            key = pyref.pack_kmer(seq[q:q + k])
                        else:
                            key = fwd
                        assert key == want[q], (seed, k, canon, q)


def test_width128_oracle_matches_golden():
    """--kmer-width=128 (the build's own mode): the C
    restatement against fixtures from the independent per-window Python
    restatement (tests/golden/make_golden.py width128)."""
    d = json.load(open(os.path.join(GOLD, "width128.json")))
    for e in d["sip13_u128"]:
        assert cbind.sip13_u128(int(e["key"])) == e["sip13"]
    seq = d["seq"].encode("latin-1")
    for c in d["cases"]:
        got = cbind.kmer_keys128(seq, c["k"], c["canonical"])
        assert [str(x) for x in got] == c["keys"], (c["k"], c["canonical"])
    e = d["e2e"]
    o = cbind.OracleCounter(e["k"], 1.0, 0.95, 2, 1.0, e["pool"], True, width=128)
    o.process_parallel([r.encode("latin-1") for r in e["records"]])
    assert list(o.currents()) == e["currents"]
    assert list(o.spike_counts()) == e["spike_counts"]
    assert list(o.voltages().view(np.uint32)) == e["voltage_bits"]
    assert list(o.refractory()) == e["refractory"]
    assert o.total_spikes == e["total_spikes"]
    assert [list(t) for t in o.top_abundant_neurons(20)] == e["top20"]


def test_oracle_fast_paths_equal_the_plain_loops():
    """The oracle's test-speed shortcuts (top-N by selection instead of a full
    sort; the LIF loop run once per distinct count of fresh neurons) give the
    same rows / states as the plain forms: the sort path (n > 4096) and
    per-neuron nko_lif on each neuron."""
    bases, offs = synth.make_records(200_000, 4, seed=21, repeats_per_mb=20_000, motif_len=60)
    for streaming in (False, True):
        r = cbind.OracleCounter(19, 1.0, 0.95, 2, 1.0, 50_021, True)
        (r.process_streaming_arrays if streaming else r.process_parallel_arrays)(bases, offs)
        assert r.top_abundant_neurons(5000)[:20] == r.top_abundant_neurons(20)
        assert r.top_abundant_neurons(4097)[:300] == r.top_abundant_neurons(300)
        cur, sc, v, rr = r.currents(), r.spike_counts(), r.voltages(), r.refractory()
        for i in range(0, 50_021, 37):
            if cur[i] == 0 and not streaming:
                continue
            vv, r1, s1 = cbind.lif(int(cur[i]), 1000, 1.0, 0.95, 2, not streaming)
            assert (s1, r1) == (int(sc[i]), int(rr[i]))
            assert np.float32(vv).view(np.uint32) == v[i].view(np.uint32)


@pytest.mark.parametrize("canon,threads", [(True, 1), (True, 4), (False, 3)])
def test_lean_cpu_baseline_matches_the_restatement(canon, threads):
    """bench.py's lean CPU baseline (nko_lean_currents_lif: no exact map, chunked
    windows, memoised LIF; not the reference's structure) gives the
    restatement's currents, spike counts and total spikes."""
    from neurokmer_amd import synth
    bases, offs = synth.make_records(60_000, 5, seed=17, repeats_per_mb=20_000, motif_len=80,
                                     n_rate=0.003, mixed_case=True)
    k, pool = 21, 5_003
    cur, sp, tot = cbind.lean_currents_lif(bases, offs, k, pool, canonical=canon, n_threads=threads)
    r = cbind.OracleCounter(k, 1.0, 0.95, 2, 1.0, pool, canon)
    r.process_parallel_arrays(bases, offs)
    np.testing.assert_array_equal(cur, r.currents())
    np.testing.assert_array_equal(sp, r.spike_counts())
    assert tot == r.total_spikes
    # other LIF parameters reach the lean LIF too (they were fixed)
    cur2, sp2, tot2 = cbind.lean_currents_lif(bases, offs, k, pool, canonical=canon,
                                              n_threads=threads, steps=300, threshold=0.5,
                                              leak=0.9, refractory=3)
    r2 = cbind.OracleCounter(k, 0.5, 0.9, 3, 1.0, pool, canon)
    r2.set_steps(300)
    r2.process_parallel_arrays(bases, offs)
    np.testing.assert_array_equal(cur2, r2.currents())
    np.testing.assert_array_equal(sp2, r2.spike_counts())
    assert tot2 == r2.total_spikes
