"""CPU tests of the host side: the FASTA/FASTQ reader (native, via the
fastx_dump harness, and the Python mirror) and the C ABI library (loads,
exports every symbol include/neurokmer.h declares, fails loudly without a GPU).
"""
import gzip
import json
import os
import re
import subprocess

import pytest

from neurokmer_amd import _lib, synth
from neurokmer_amd.fastx import stream_sequences

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DUMP = os.path.join(ROOT, "neurokmer_amd", "bin", "fastx_dump")


def native(path, batch=1 << 20):
    out = subprocess.run([DUMP, str(path), str(batch)], capture_output=True, check=True).stdout
    d = json.loads(out)
    return d["rc"], [bytes.fromhex(h) for h in d["records"]], d["truncated"]


def both(path, batch=1 << 20):
    rc, recs, _ = native(path, batch)
    assert rc == 0
    py = list(stream_sequences(str(path)))
    assert recs == py
    return recs


@pytest.fixture(scope="module", autouse=True)
def _built():
    if not os.path.exists(DUMP):
        subprocess.run(["make", "-C", os.path.join(ROOT, "neurokmer_amd", "csrc"),
                        os.path.join("..", "bin", "fastx_dump")], check=True)


def test_fasta_multiline_crlf_blank(tmp_path):
    p = tmp_path / "a.fa"
    p.write_bytes(b">r1 desc\nACGT\r\nNNac\n\n>r2\n>r3\nTTTT\nG")
    assert both(p) == [b"ACGTNNac", b"", b"TTTTG"]


@pytest.mark.parametrize("batch", [1, 7, 1 << 20])
def test_fasta_synthetic_roundtrip(tmp_path, batch):
    bases, offs = synth.make_records(50_000, 9, n_rate=0.01, mixed_case=True)
    p = tmp_path / "s.fa"
    synth.write_fasta(str(p), bases, offs, width=61)
    assert both(p, batch) == synth.records_list(bases, offs)


def test_fastq_and_gzip(tmp_path):
    bases, offs = synth.make_reads(300, 150, seed=3)
    p = tmp_path / "r.fq"
    synth.write_fastq(str(p), bases, offs)
    assert both(p) == synth.records_list(bases, offs)
    gz = tmp_path / "r.fq.gz"
    gz.write_bytes(gzip.compress(p.read_bytes()))
    assert both(gz) == synth.records_list(bases, offs)


def test_fastq_stops_at_first_malformed_record(tmp_path):
    # src/utils.rs:16-20: a parse error ends the stream; earlier records are kept
    p = tmp_path / "bad.fq"
    p.write_bytes(b"@a\nACGT\n+\nIIII\n@b\nACG\n+\nII\n@c\nTTTT\n+\nIIII\n")
    rc, recs, truncated = native(p)
    assert rc == 0 and recs == [b"ACGT"] and truncated
    assert list(stream_sequences(str(p))) == [b"ACGT"]


def test_empty_and_unknown_format_are_errors(tmp_path):
    e = tmp_path / "empty.fa"
    e.write_bytes(b"")
    assert native(e)[0] == _lib.NK_E_PARSE
    with pytest.raises(ValueError):
        stream_sequences(str(e))
    u = tmp_path / "u.txt"
    u.write_bytes(b"ACGT\n")
    assert native(u)[0] == _lib.NK_E_PARSE
    with pytest.raises(ValueError):
        stream_sequences(str(u))
    assert native(tmp_path / "missing.fa")[0] == _lib.NK_E_IO


def header_functions():
    text = open(os.path.join(ROOT, "include", "neurokmer.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(nk_[a-z_0-9]+)\s*\(", text)))


def test_library_exports_every_header_symbol():
    L = _lib.load(share_torch=False)
    names = header_functions()
    assert len(names) >= 25
    assert sorted(_lib.EXPORTS) == names
    for n in names:
        assert hasattr(L, n), n
    nm = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True,
                        text=True, check=True).stdout
    for n in names:
        assert re.search(rf"\bT {n}$", nm, re.M), n


def test_exact_owner_matches_python_restatement():
    # the owner rank of a key (multi-GPU exact table) is pure host arithmetic:
    # the library and neurokmer_amd.dist.exact_owner must agree bit for bit
    import numpy as np
    from neurokmer_amd.dist import exact_owner
    L = _lib.load()
    rng = np.random.default_rng(5)
    keys = np.concatenate([rng.integers(0, 2**63, 2000, dtype=np.uint64) * np.uint64(2) + 1,
                           np.array([0, 1, 2**64 - 1, 2**63], np.uint64)])
    for world in (1, 2, 3, 8, 64, 4096):
        own = exact_owner(keys, world)
        assert own.min() >= 0 and own.max() < world
        assert [L.nk_exact_owner(int(x), world) for x in keys[:300]] == own[:300].tolist()
    own8 = exact_owner(keys, 8)
    assert np.bincount(own8, minlength=8).min() > 150  # spread over the ranks


def test_no_cpu_fallback_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from neurokmer_amd import SpikingKmerCounter
    with pytest.raises(_lib.NeuroKmerError) as e:
        SpikingKmerCounter(31, 1.0, 0.95, 2, 1.0, 1000, True)
    assert e.value.code == _lib.NK_E_NO_DEVICE
    assert "no CPU fallback" in str(e.value)
    L = _lib.load()
    assert L.nk_version().decode().startswith("neurokmer-mi355x")


def test_cli_rejects_bad_usage():
    cli = _lib.CLI_PATH
    r = subprocess.run([cli], capture_output=True, text=True)
    assert r.returncode == 2 and "--input" in r.stderr
    r = subprocess.run([cli, "--help"], capture_output=True, text=True)
    assert r.returncode == 0 and "--pool-size" in r.stderr
    r = subprocess.run([cli, "-i", "x.fa", "-k", "abc"], capture_output=True, text=True)
    assert r.returncode == 2


def mapped(path, window, threads, max_rec=None):
    args = [DUMP, str(path), "--mapped", str(window), str(threads)]
    if max_rec:
        args.append(str(max_rec))
    out = subprocess.run(args, capture_output=True, check=True).stdout
    d = json.loads(out)
    return d["rc"], [bytes.fromhex(h) for h in d["records"]], d["truncated"], d["fallback"]


def _random_fastq(rng, n):
    import numpy as np
    """FASTQ with the cases the ingest must get right: CRLF lines, empty
    sequences, '+' lines with text, a malformed record (header, '+' line or
    quality length), blank lines between records, blank lines at the end, a
    cut-off last record, no final newline."""
    out = []
    for i in range(n):
        eol = b"\r\n" if rng.random() < 0.2 else b"\n"
        ln = int(rng.integers(0, 40)) if rng.random() < 0.9 else 0
        seq = rng.choice(np.frombuffer(b"ACGTNacgt", np.uint8), ln).tobytes() if ln else b""
        qual = b"I" * ln
        hdr = b"@r%d" % i
        plus = b"+" if rng.random() < 0.7 else b"+r%d" % i
        kind = rng.random()
        if kind < 0.002:
            hdr = b"r%d" % i           # header without '@'
        elif kind < 0.004:
            plus = b"-"                # no '+' line
        elif kind < 0.006:
            qual = qual + b"I"         # quality length != sequence length
        elif kind < 0.008:
            out.append(b"\n")          # a blank line where a header is due
        out.append(hdr + eol + seq + eol + plus + eol + qual + eol)
    data = b"".join(out)
    tail = rng.random()
    if tail < 0.2:
        data += b"\n\n"                # blank lines end the input
    elif tail < 0.4:
        data = data.rstrip(b"\n").rstrip(b"\r")  # no final newline
    elif tail < 0.5:
        data += b"@cut\nACGT\n+\n"     # cut-off last record
    return data


@pytest.mark.parametrize("seed", range(12))
def test_mapped_fastq_extraction_matches_reader(tmp_path, seed):
    """The file ingest's host FASTQ extraction (nk_fqhost.cpp: threads over
    windows of a mapped file) takes exactly the records the sequential reader
    takes, stops where it stops, and reports a blank line between records
    (the ingest then falls back to that reader)."""
    import numpy as np
    rng = np.random.default_rng(seed)
    p = tmp_path / "f.fq"
    p.write_bytes(_random_fastq(rng, int(rng.integers(1, 400))))
    rc, recs, trunc = native(p)
    assert rc == 0
    for window, threads, max_rec in ((16, 1, None), (37, 3, None), (301, 8, None), (1 << 20, 5, None),
                                     (1 << 20, 4, 7), (5000, 2, 1)):
        mrc, mrecs, mtrunc, fb = mapped(p, window, threads, max_rec)
        assert mrc == 0
        if fb:  # only a blank line between records sends the ingest to the reader
            assert re.search(rb"\n\r?\n", p.read_bytes())
            continue
        assert mrecs == recs, (window, threads)
        assert mtrunc == trunc, (window, threads)


def test_mapped_fastq_large_synthetic(tmp_path):
    bases, offs = synth.make_reads(20_000, 150, seed=5)
    p = tmp_path / "r.fq"
    synth.write_fastq(str(p), bases, offs)
    want = synth.records_list(bases, offs)
    for window, threads in ((1 << 16, 8), (100_003, 3), (1 << 26, 16)):
        rc, recs, trunc, fb = mapped(p, window, threads)
        assert (rc, fb, trunc) == (0, False, False)
        assert recs == want


# --- a stopped input is reported ---------------------------
# The reference warns when the stream stops at a malformed record
# (`warn!("Skipping malformed record: {}", e)`, src/utils.rs:17-19); a read that
# fails (or a file that ends before its size while it is read) is an I/O error,
# not a quiet end of the input.

def _dump(*args):
    r = subprocess.run([DUMP, *map(str, args)], capture_output=True, check=True)
    return json.loads(r.stdout), r.stderr.decode()


def test_truncated_fastq_warns_once_and_keeps_earlier_records(tmp_path):
    p = tmp_path / "cut.fq"
    p.write_bytes(b"@a\nACGT\n+\nIIII\n@b\nACGTAC\n+\nIII")  # record b cut inside its quality
    for args in ((p,), (p, "--mapped", 4096, 2)):
        d, err = _dump(*args)
        assert d["rc"] == 0 and d["truncated"] and d["records"] == ["41434754"]
        lines = [ln for ln in err.splitlines() if "Skipping malformed record" in ln]
        assert len(lines) == 1 and "record 1 of" in lines[0] and str(p) in lines[0]


def test_file_ending_early_is_an_io_error(tmp_path):
    p = tmp_path / "shrinks.fq"
    bases, offs = synth.make_reads(2000, 150, seed=5)
    synth.write_fastq(str(p), bases, offs)
    d, err = _dump(p, "--mapped", 1 << 16, 4, "--shrink", 100_000)
    assert d["rc"] == _lib.NK_E_IO and "ended at byte" in d["err"]
    assert "Skipping malformed record" not in err


def test_cut_off_gzip_warns_and_stops(tmp_path):
    p = tmp_path / "cut.fq.gz"
    raw = b"".join(b"@r%d\nACGTACGT\n+\nIIIIIIII\n" % i for i in range(50_000))
    z = gzip.compress(raw)
    p.write_bytes(z[: len(z) // 2])
    d, err = _dump(p)
    assert d["rc"] == 0 and d["truncated"] and 0 < len(d["records"]) < 50_000
    assert all(r == "4143475441434754" for r in d["records"])
    assert "gzip" in err and "Skipping malformed record" in err
