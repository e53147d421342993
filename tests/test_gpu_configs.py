"""BASELINE.json's configurations on the HIP path (through the C ABI) against
the CPU restatement (oracle/nk_oracle.c), plus the committed golden fixtures
replayed through the HIP path with no oracle in the loop, and the fallback
count kernels.

  config 1  1,000,000 bases in 10 records, k=21, pool=100,000 (+ planted repeats
            so spikes and the top-20 are non-trivial), in-memory, both modes
  config 3  FASTQ of 150-bp reads, k=31, pool=16,000,000, --streaming:
            >= 50 MB bit-exact at two ingest chunk sizes, and a >= 1 GB
            property run (sum of currents = N_k, chunk-size invariance,
            determinism, block linearity)
  config 5  k=63, pool=256,000,000, compat (u64 release semantics) and
            --kmer-width=128, ~1 Mbase bit-exact; a multi-GB property run
  config 4  (2 ranks, records split inside with a k-1 halo): tests/test_gpu_dist.py
Reference call sites: src/spiking_hash.rs:84-201 (process_parallel),
:277-486 (process_file_streaming), src/main.rs:36-46.
"""
import contextlib
import glob
import json
import os
import subprocess

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")  # import first: one shared HIP runtime
if not torch.cuda.is_available():
    pytest.skip("no GPU", allow_module_level=True)

from neurokmer_amd import SpikingKmerCounter, synth  # noqa: E402
from neurokmer_amd import _lib  # noqa: E402
from oracle import cbind  # noqa: E402

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
THREADS = 8  # oracle record-level threads (rayon's work unit is one record)


def assert_same(gpu, ref, n=20):
    np.testing.assert_array_equal(gpu.currents(), ref.currents())
    np.testing.assert_array_equal(gpu.spike_counts(), ref.spike_counts())
    np.testing.assert_array_equal(gpu.voltages().view(np.uint32), ref.voltages().view(np.uint32))
    np.testing.assert_array_equal(gpu.refractory(), ref.refractory())
    assert gpu.energy.total_spikes() == ref.total_spikes
    assert gpu.energy_used() == ref.energy_used()
    assert gpu.top_abundant_neurons(n) == ref.top_abundant_neurons(n)


@contextlib.contextmanager
def env(**kv):
    old = {k: os.environ.get(k) for k in kv}
    os.environ.update({k: str(v) for k, v in kv.items()})
    try:
        yield
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def n_kmers(offs, k):
    return int(np.clip(np.diff(offs.astype(np.int64)) - (k - 1), 0, None).sum())


# ---- config 1 ---------------------------------------------------------------
@pytest.mark.parametrize("canon", [True, False])
def test_config1_in_memory(canon):
    bases, offs = synth.make_records(1_000_000, 10, seed=101, repeats_per_mb=400, motif_len=120)
    assert offs.size == 11 and int(offs[-1]) == 1_000_000
    g = SpikingKmerCounter(21, 1.0, 0.95, 2, 1.0, 100_000, canon)
    g.process_parallel_arrays(bases, offs)
    r = cbind.OracleCounter(21, 1.0, 0.95, 2, 1.0, 100_000, canon)
    r.process_parallel_arrays(bases, offs, THREADS)
    assert r.total_spikes > 0  # the planted repeats make the check non-vacuous
    assert int(g.currents().sum()) == n_kmers(offs, 21) == 999_800
    assert_same(g, r)


def test_config1_cli_file(tmp_path):
    """config 1 as the reference's CLI runs it: FASTA file -> in-memory path."""
    bases, offs = synth.make_records(1_000_000, 10, seed=102, repeats_per_mb=400, motif_len=120)
    p = tmp_path / "c1.fa"
    synth.write_fasta(str(p), bases, offs, width=60)
    g = SpikingKmerCounter(21, 1.0, 0.95, 2, 1.0, 100_000, True)
    g.process_file_parallel(str(p))
    r = cbind.OracleCounter(21, 1.0, 0.95, 2, 1.0, 100_000, True)
    r.process_parallel_arrays(bases, offs, THREADS)
    assert_same(g, r)
    out = subprocess.run([_lib.CLI_PATH, "-i", str(p), "-k", "21", "--pool-size", "100000",
                          "--canonical"], capture_output=True, check=True, text=True).stdout
    assert f"Total spikes fired: {r.total_spikes}\n" in out


# ---- config 3 ---------------------------------------------------------------
C3_POOL = 16_000_000


def _write_fastq_fast(path, bases, read_len, qual=ord("I")):
    """Equal-length reads -> FASTQ, vectorised: fixed-width headers @r%09d."""
    n = bases.size // read_len
    seq = bases[:n * read_len].reshape(n, read_len)
    hdr = np.frombuffer(b"".join(b"@r%09d\n" % i for i in range(n)), np.uint8).reshape(n, 12)
    nl = np.full((n, 1), ord("\n"), np.uint8)
    plus = np.frombuffer(b"+\n", np.uint8)[None, :].repeat(n, 0)
    q = np.full((n, read_len), qual, np.uint8)
    rows = np.concatenate([hdr, seq, nl, plus, q, nl], axis=1)
    with open(path, "ab") as f:
        f.write(rows.tobytes())
    return n


def test_config3_fastq_streaming_50mb(tmp_path):
    n_reads = 175_000  # 175,000 x 150 bp: 54.6 MB of FASTQ
    bases, offs = synth.make_reads(n_reads, 150, seed=103, repeats_per_mb=3000, motif_len=60,
                                   n_rate=0.0005)
    p = tmp_path / "c3.fq"
    _write_fastq_fast(str(p), bases, 150)
    assert p.stat().st_size >= 50_000_000
    r = cbind.OracleCounter(31, 1.0, 0.95, 2, 1.0, C3_POOL, True)
    r.process_streaming_arrays(bases, offs, THREADS)
    for chunk in (1 << 22, 7_000_003):  # many chunks; records cross chunk ends
        with env(NK_INGEST_CHUNK=chunk):
            g = SpikingKmerCounter(31, 1.0, 0.95, 2, 1.0, C3_POOL, True)
            g.process_file_streaming(str(p))
        assert_same(g, r)
        g.close()


def test_config3_fastq_1gb_properties(tmp_path):
    """>= 1 GB FASTQ, k=31, pool 16 M, --streaming: identical 64 MB blocks, so
    the currents must be exactly 16x one block's (linearity), their sum N_k,
    and equal across ingest chunk sizes and repeated runs (determinism)."""
    read_len, n_reads = 150, 200_000
    bases, offs = synth.make_reads(n_reads, read_len, seed=104, repeats_per_mb=200, motif_len=80)
    blk = tmp_path / "blk.fq"
    _write_fastq_fast(str(blk), bases, read_len)
    data = blk.read_bytes()
    reps = -(-(1 << 30) // len(data))  # >= 1 GiB
    big = tmp_path / "big.fq"
    with open(big, "wb") as f:
        for _ in range(reps):
            f.write(data)
    assert big.stat().st_size >= 1 << 30
    g1 = SpikingKmerCounter(31, 1.0, 0.95, 2, 1.0, C3_POOL, True)
    g1.process_file_streaming(str(blk))
    one = g1.currents()
    g1.close()
    runs = []
    for chunk in (1 << 26, 48_000_017, 1 << 26):
        with env(NK_INGEST_CHUNK=chunk):
            g = SpikingKmerCounter(31, 1.0, 0.95, 2, 1.0, C3_POOL, True)
            g.process_file_streaming(str(big))
        runs.append((g.currents(), g.spike_counts(), g.energy.total_spikes(),
                     g.top_abundant_neurons(20)))
        g.close()
    cur = runs[0][0]
    assert int(cur.sum()) == reps * n_reads * (read_len - 30)
    np.testing.assert_array_equal(cur, one * np.uint64(reps))
    for other in runs[1:]:
        np.testing.assert_array_equal(other[0], cur)
        np.testing.assert_array_equal(other[1], runs[0][1])
        assert other[2:] == runs[0][2:]
    assert int(runs[0][1].sum()) == runs[0][2]


# ---- config 5 ---------------------------------------------------------------
C5_POOL = 256_000_000


@pytest.mark.parametrize("width", [64, 128])
def test_config5_k63_pool256m(width):
    bases, offs = synth.make_records(1_000_000, 8, seed=105, repeats_per_mb=500, motif_len=150,
                                     n_rate=0.001)
    g = SpikingKmerCounter(63, 1.0, 0.95, 2, 1.0, C5_POOL, True, kmer_width=width)
    g.process_parallel_arrays(bases, offs)
    r = cbind.OracleCounter(63, 1.0, 0.95, 2, 1.0, C5_POOL, True, width=width)
    r.process_parallel_arrays(bases, offs, 2)  # 2 GB of fold currents per thread
    assert r.total_spikes > 0
    assert_same(g, r)


def _device_random_records(n_bases, n_recs, seed):
    """Uniform ACGT generated on the device (multi-GB inputs for property runs)."""
    gen = torch.Generator(device="cuda")
    gen.manual_seed(seed)
    lut = torch.tensor(list(b"ACGT"), dtype=torch.uint8, device="cuda")
    codes = torch.randint(0, 4, (n_bases + 16,), generator=gen, device="cuda", dtype=torch.uint8)
    d_b = lut[codes.long()] if n_bases < (1 << 28) else _lut_chunked(codes, lut)
    del codes
    lens = np.full(n_recs, n_bases // n_recs, np.uint64)
    lens[: n_bases % n_recs] += 1
    offs = np.zeros(n_recs + 1, np.uint64)
    np.cumsum(lens, out=offs[1:])
    return d_b, offs


def _lut_chunked(codes, lut):
    out = torch.empty_like(codes)
    step = 1 << 28
    for s in range(0, codes.numel(), step):
        out[s:s + step] = lut[codes[s:s + step].long()]
    return out


class _CAI:
    def __init__(self, ptr, n, typestr="<i8"):
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": typestr, "data": (ptr, False),
                                         "version": 3}


@pytest.mark.parametrize("width", [64, 128])
def test_config5_multi_gb_properties(width):
    """k=63, pool 256 M on 3 Gbases resident in HBM: sum of currents = N_k,
    determinism, and per-record linearity (records counted one by one sum to
    the whole), compared on the device."""
    n, recs = 3_000_000_000, 6
    d_b, offs = _device_random_records(n, recs, seed=55 + width)
    d_o = torch.from_numpy(offs.view(np.int64)).cuda()
    torch.cuda.synchronize()
    g = SpikingKmerCounter(63, 1.0, 0.95, 2, 1.0, C5_POOL, True, kmer_width=width)
    g.accumulate_device(d_b.data_ptr(), d_o.data_ptr(), recs, n)
    whole = torch.as_tensor(_CAI(g.device_currents_ptr(), C5_POOL), device="cuda").clone()
    torch.cuda.synchronize()  # the next call rewrites the library's currents
    assert int(whole.sum().item()) == n_kmers(offs, 63)
    g.accumulate_device(d_b.data_ptr(), d_o.data_ptr(), recs, n)
    again = torch.as_tensor(_CAI(g.device_currents_ptr(), C5_POOL), device="cuda")
    assert torch.equal(again, whole)
    acc = torch.zeros_like(whole)
    for i in range(recs):
        lo, hi = int(offs[i]), int(offs[i + 1])
        o = torch.from_numpy(np.array([0, hi - lo], np.int64)).cuda()
        sub = d_b[lo:hi]
        if sub.data_ptr() % 16:
            sub = sub.clone()
        torch.cuda.synchronize()
        g.accumulate_device(sub.data_ptr(), o.data_ptr(), 1, hi - lo)
        acc += torch.as_tensor(_CAI(g.device_currents_ptr(), C5_POOL), device="cuda")
        torch.cuda.synchronize()
        del sub
    assert torch.equal(acc, whole)
    g.close()


# ---- bounded arena: inputs past count_chunk() are counted batch by batch ----------
@pytest.mark.parametrize("k,pool,canon,width", [
    (31, 2_000_000, True, 64),     # Part
    (21, 100_003, False, 64),      # Part, pack_kmer keys
    (40, 50_021, True, 64),        # Gen (compat k > 32)
    (63, 20_000_003, True, 128),   # Wide, 128-bit keys
])
def test_batched_count_bit_exact(k, pool, canon, width):
    """NK_COUNT_CHUNK forces the batched count (records histogrammed and dropped
    per batch, uniques from a rescan) on a ~1.2 Mbase input: bit-exact vs the
    oracle, for host input, device input + finalize, and two steps in a row."""
    bases, offs = synth.make_records(1_200_000, 6, seed=140 + k, repeats_per_mb=4000,
                                     motif_len=100, n_rate=0.002, mixed_case=True)
    r = cbind.OracleCounter(k, 1.0, 0.95, 2, 1.0, pool, canon, width=width)
    r.process_parallel_arrays(bases, offs, THREADS)
    with env(NK_COUNT_CHUNK=200_000):  # 24 partition tiles per batch: 6 batches
        g = SpikingKmerCounter(k, 1.0, 0.95, 2, 1.0, pool, canon, kmer_width=width)
        g.process_parallel_arrays(bases, offs)
        assert_same(g, r)
        assert g.top_abundant_neurons(300) == r.top_abundant_neurons(300)  # held input
        d_b = torch.from_numpy(np.concatenate([bases, np.zeros(16, np.uint8)])).cuda()
        d_o = torch.from_numpy(offs.view(np.int64)).cuda()
        torch.cuda.synchronize()
        g.accumulate_device(d_b.data_ptr(), d_o.data_ptr(), offs.size - 1, bases.size)
        g.finalize(False)
        r.process_parallel_arrays(bases, offs, THREADS)
        assert_same(g, r)
    g.close()


def test_batched_streaming_file(tmp_path):
    """The file ingest's Part path past count_chunk(): each ingest batch is
    histogrammed and dropped (FASTQ, pool 16 M, small ingest chunks)."""
    bases, offs = synth.make_reads(20_000, 150, seed=150, repeats_per_mb=3000, motif_len=60,
                                   n_rate=0.0005)
    p = tmp_path / "b.fq"
    _write_fastq_fast(str(p), bases, 150)
    r = cbind.OracleCounter(31, 1.0, 0.95, 2, 1.0, C3_POOL, True)
    r.process_streaming_arrays(bases, offs, THREADS)
    with env(NK_COUNT_CHUNK=300_000, NK_INGEST_CHUNK=1_000_003):
        g = SpikingKmerCounter(31, 1.0, 0.95, 2, 1.0, C3_POOL, True)
        g.process_file_streaming(str(p))
    assert_same(g, r)
    g.close()


def test_part_path_past_2_32_positions():
    """k=31, pool 2M (the Part path) on 4.5 Gbases resident in HBM: past 2^32
    positions and past count_chunk(), so the count runs in bounded batches.
    The input is 5 copies of one 900 Mbase record: the currents must be exactly
    5x one copy's (counted on the keep-records path), their sum N_k, the same on
    a second run, and the top rows' uniques equal to one copy's kmer_per_neuron
    (the same distinct keys)."""
    n1, reps = 900_000_000, 5
    one, _ = _device_random_records(n1, 1, seed=77)
    d_b = torch.cat([one[:n1]] * reps + [torch.zeros(16, dtype=torch.uint8, device="cuda")])
    n = n1 * reps
    assert n > (1 << 32)
    offs = np.arange(reps + 1, dtype=np.uint64) * np.uint64(n1)
    d_o = torch.from_numpy(offs.view(np.int64)).cuda()
    o1 = torch.from_numpy(np.array([0, n1], np.int64)).cuda()
    torch.cuda.synchronize()
    g1 = SpikingKmerCounter(31, 1.0, 0.95, 2, 1.0, POOL2, True, exact_counts=True)
    g1.accumulate_device(one.data_ptr(), o1.data_ptr(), 1, n1)
    single = torch.as_tensor(_CAI(g1.device_currents_ptr(), POOL2), device="cuda").clone()
    torch.cuda.synchronize()
    kpn1 = g1.kmer_per_neuron()
    g = SpikingKmerCounter(31, 1.0, 0.95, 2, 1.0, POOL2, True)
    g.accumulate_device(d_b.data_ptr(), d_o.data_ptr(), reps, n)
    whole = torch.as_tensor(_CAI(g.device_currents_ptr(), POOL2), device="cuda").clone()
    torch.cuda.synchronize()
    assert int(whole.sum().item()) == n_kmers(offs, 31) == reps * (n1 - 30)
    assert torch.equal(whole, single * reps)
    g.accumulate_device(d_b.data_ptr(), d_o.data_ptr(), reps, n)
    g.finalize(False)
    assert torch.equal(torch.as_tensor(_CAI(g.device_currents_ptr(), POOL2), device="cuda"), whole)
    top = g.top_abundant_neurons(20)
    sc = g.spike_counts()
    assert int(sc.sum()) == g.energy.total_spikes()
    order = [int(i) for i in np.argsort(-sc.astype(np.int64), kind="stable")[:20]]
    assert [t[0] for t in top] == order
    assert [t[2] for t in top] == [int(kpn1[i]) for i in order]
    g.close()
    g1.close()


POOL2 = 2_000_000


@pytest.mark.parametrize("k,pool,canon,width,tile_list", [
    (40, 2_000_003, True, 64, None),      # Gen: dense hits (57 k-mers per neuron)
    (40, 2_000_003, True, 64, 3),         # ... list overflow -> the full rescan
    (63, 40_000_003, True, 128, None),    # Wide, 128-bit keys (lane-tagged records)
    (63, 40_000_003, True, 128, "untagged"),  # ... without lane tags: whole listed tiles
    (33, 30_000_001, True, 64, "queue1"),  # hits resolved in place (LDS hit queue of 1)
    (33, 30_000_001, False, 64, 2),       # Wide, pack_kmer keys, list overflow
    (63, C5_POOL, True, 64, None),        # config-5 pool, compat keys
    (63, C5_POOL, True, 128, "split7"),   # config 5: the split pipelined over 7 launches
    (33, 30_000_001, False, 64, "split3"),  # Wide, pack_kmer keys, 3 launches
])
def test_uniques_from_kept_records(k, pool, canon, width, tile_list):
    """Gen/Wide counts keep k_part_gen's records and segment descriptors; the
    top rows' uniques rescan only the tiles holding their records
    (k_uniq_tiles), or everything when the tile list overflows
    (NK_UNIQ_TILE_LIST): top-20 rows with uniques bit-exact vs the oracle."""
    bases, offs = synth.make_records(1_500_000, 5, seed=170 + k, repeats_per_mb=3000,
                                     motif_len=120, n_rate=0.002, mixed_case=True)
    r = cbind.OracleCounter(k, 1.0, 0.95, 2, 1.0, pool, canon, width=width)
    r.process_parallel_arrays(bases, offs, THREADS)
    kv = ({"NK_NO_LANE_TAG": 1} if tile_list == "untagged" else
          {"NK_UNIQ_HIT_QUEUE": 1} if tile_list == "queue1" else
          {"NK_SPLIT_LAUNCHES": int(tile_list[5:])} if str(tile_list).startswith("split") else
          {"NK_UNIQ_TILE_LIST": tile_list} if tile_list else {})
    with env(**kv):
        g = SpikingKmerCounter(k, 1.0, 0.95, 2, 1.0, pool, canon, kmer_width=width)
        g.process_parallel_arrays(bases, offs)
        assert_same(g, r)
        g.process_parallel_arrays(bases, offs)  # state carries over
    r.process_parallel_arrays(bases, offs, THREADS)
    assert_same(g, r)
    g.close()


@pytest.mark.parametrize("k,pool,width,top_n", [
    (40, 2_000_003, 64, 100),    # Gen, top-N not fused into the LIF (top_n > 64)
    (33, 30_000_001, 64, 20),    # Wide
    (63, 40_000_003, 128, 20),   # Wide, 128-bit keys
])
def test_k1b_fused_lif(k, pool, width, top_n):
    """The LIF from the reset state run inside the write-through K1b (Gen/Wide,
    one batch, a top-N not fused into the LIF kernel): bit-exact vs the oracle
    on a process call, a second call (state carries: the LIF kernel runs), and
    the split API (accumulate + finalize, in-memory and streaming rule), with
    the counts touched (device_currents) or the steps changed in between (the
    K1b result is dropped and the LIF kernel runs)."""
    bases, offs = synth.make_records(1_000_000, 5, seed=900 + k, repeats_per_mb=3000,
                                     motif_len=120, n_rate=0.002, mixed_case=True)
    r = cbind.OracleCounter(k, 1.0, 0.95, 2, 1.0, pool, True, width=width)
    r.process_parallel_arrays(bases, offs, THREADS)
    g = SpikingKmerCounter(k, 1.0, 0.95, 2, 1.0, pool, True, kmer_width=width, top_n=top_n)
    g.process_parallel_arrays(bases, offs)
    assert_same(g, r, n=top_n)
    g.process_parallel_arrays(bases, offs)
    r.process_parallel_arrays(bases, offs, THREADS)
    assert_same(g, r, n=top_n)
    d_b = torch.from_numpy(np.concatenate([bases, np.zeros(16, np.uint8)])).cuda()
    d_o = torch.from_numpy(offs.view(np.int64)).cuda()
    torch.cuda.synchronize()
    for streaming, between in ((False, None), (True, None), (False, "currents"), (False, "steps")):
        g.reset()
        r = cbind.OracleCounter(k, 1.0, 0.95, 2, 1.0, pool, True, width=width)
        g.accumulate_device(d_b.data_ptr(), d_o.data_ptr(), offs.size - 1, bases.size)
        if between == "currents":
            g.device_currents_ptr()
        elif between == "steps":
            g.set_steps(700)
            r.set_steps(700)
        g.finalize(streaming=streaming)
        if streaming:
            r.process_streaming_arrays(bases, offs, THREADS)
        else:
            r.process_parallel_arrays(bases, offs, THREADS)
        assert_same(g, r, n=top_n)
        g.set_steps(1000)
    g.close()


# ---- golden fixtures through the HIP path ------------------------------------
GOLDEN_E2E = sorted(glob.glob(os.path.join(GOLD, "e2e_*.json")))


@pytest.mark.parametrize("path", GOLDEN_E2E, ids=[os.path.basename(p)[4:-5] for p in GOLDEN_E2E])
def test_golden_e2e_hip(path, tmp_path):
    d = json.load(open(path))
    recs = [x.encode("latin-1") for x in d["records"]]
    g = SpikingKmerCounter(d["k"], 1.0, 0.95, 2, 1.0, d["pool"], d["canonical"])
    g.set_steps(d["steps"])
    if d["streaming"]:
        p = tmp_path / "g.fa"
        with open(p, "wb") as f:
            for i, r in enumerate(recs):
                f.write(b">g%d\n%s\n" % (i, r))
        g.process_file_streaming(str(p))
    else:
        g.process_parallel(recs)
    assert list(g.currents()) == d["currents"]
    assert list(g.spike_counts()) == d["spike_counts"]
    assert list(g.voltages().view(np.uint32)) == d["voltage_bits"]
    assert list(g.refractory()) == d["refractory"]
    assert g.energy.total_spikes() == d["total_spikes"]
    assert round(g.energy_used() * 1000) == d["total_energy_fixed"]
    assert [list(t) for t in g.top_abundant_neurons(20)] == d["top20"]
    if d["steps"] == 1000 and all(b">" not in r and b"\n" not in r for r in recs):
        # the CLI (fixed LIF constants, steps 1000) prints the same result block
        p = tmp_path / "cli.fa"
        with open(p, "wb") as f:
            for i, r in enumerate(recs):
                f.write(b">g%d\n%s\n" % (i, r))
        args = [_lib.CLI_PATH, "-i", str(p), "-k", str(d["k"]), "--pool-size", str(d["pool"])]
        if d["canonical"]:
            args.append("--canonical")
        if d["streaming"]:
            args.append("--streaming")
        out = subprocess.run(args, capture_output=True, check=True, text=True).stdout
        assert out.endswith(d["stdout_block"])


# ---- fallback count kernels ------------------------------------------------------
def _ragged(total, seed):
    bases, _ = synth.make_records(total, 1, seed=seed, n_rate=0.01, mixed_case=True,
                                  repeats_per_mb=8000, motif_len=110)
    rng = np.random.default_rng(seed)
    lens, s = [], 0
    while s < total:
        L = min(int(rng.integers(0, 3000)), total - s)
        lens.append(L)
        s += L
    offs = np.zeros(len(lens) + 1, np.uint64)
    np.cumsum(lens, out=offs[1:])
    return bases, offs


@pytest.mark.parametrize("canon", [True, False])
@pytest.mark.parametrize("k", [64, 65, 96])
def test_compat_k_past_64(k, canon):
    """Compat (u64 release-build) keys for k >= 64: k=64 runs the generic
    partition, k > 64 the direct-atomic k_kmers_compat kernel (src/models.rs:
    188-194,260-266: any k in release builds)."""
    bases, offs = _ragged(150_000, seed=500 + k)
    g = SpikingKmerCounter(k, 1.0, 0.95, 2, 1.0, 30_011, canon)
    g.process_parallel_arrays(bases, offs)
    r = cbind.OracleCounter(k, 1.0, 0.95, 2, 1.0, 30_011, canon)
    r.process_parallel_arrays(bases, offs, THREADS)
    assert_same(g, r)


@pytest.mark.parametrize("canon", [True, False])
@pytest.mark.parametrize("k,width", [(21, 64), (31, 64), (40, 64), (63, 128), (17, 128)])
def test_forced_direct_atomic_path(k, width, canon):
    """NK_FORCE_ATOMIC=1 routes a small input through the direct-atomic count
    kernels that otherwise run only past the partitions (pool > 2^31):
    k_kmers<canon, mode> (k <= 32), k_kmers_compat (k > 32), k_kmers128."""
    bases, offs = _ragged(120_000, seed=600 + k)
    with env(NK_FORCE_ATOMIC=1):
        g = SpikingKmerCounter(k, 1.0, 0.95, 2, 1.0, 100_003, canon, kmer_width=width)
        g.process_parallel_arrays(bases, offs)
    r = cbind.OracleCounter(k, 1.0, 0.95, 2, 1.0, 100_003, canon, width=width)
    r.process_parallel_arrays(bases, offs, THREADS)
    assert_same(g, r)
