"""Deterministic synthetic sequence generator.

i.i.d. uniform ACGT driven by splitmix64 in counter mode, seed 0x4E4B4D52
("NKMR"), so the same stream can be produced on the host (here, numpy), by the
C++ CLI tools, or by a device kernel for the 100 GB configs.  Base i of the
stream is ``"ACGT"[(z[i >> 5] >> (2 * (i & 31))) & 3]`` with
``z[j] = splitmix64_mix(seed + (j + 1) * 0x9E3779B97F4A7C15)``.

Options that make parity fixtures non-trivial:
  * planted repeats: ``repeats_per_mb`` copies of a ``motif_len``-bp motif in
    every 1,000,000-base block (hot neurons, saturated spikes, top-N ties);
  * ``n_rate``: fraction of bases replaced by runs of 'N' (and, with
    ``mixed_case``, lowercase bases and a few other IUPAC bytes), which
    exercise the reference's "anything else -> 0" rules (src/models.rs:231-251)
    and pack_kmer's skip rule (src/utils.rs:26-39).
"""
from __future__ import annotations

import numpy as np

SEED = 0x4E4B4D52
GAMMA = np.uint64(0x9E3779B97F4A7C15)
_ACGT = np.frombuffer(b"ACGT", dtype=np.uint8)


def _mix(z: np.ndarray) -> np.ndarray:
    z = z.astype(np.uint64, copy=True)
    with np.errstate(over="ignore"):
        z ^= z >> np.uint64(30)
        z *= np.uint64(0xBF58476D1CE4E5B9)
        z ^= z >> np.uint64(27)
        z *= np.uint64(0x94D049BB133111EB)
        z ^= z >> np.uint64(31)
    return z


def random_words(n_words: int, seed: int = SEED, start: int = 0) -> np.ndarray:
    j = np.arange(start + 1, start + n_words + 1, dtype=np.uint64)
    with np.errstate(over="ignore"):
        return _mix(np.uint64(seed & 0xFFFFFFFFFFFFFFFF) + j * GAMMA)


def random_bases(n: int, seed: int = SEED, chunk: int = 1 << 24, start: int = 0) -> np.ndarray:
    """Bases start .. start+n-1 of the splitmix64 stream as ASCII ACGT (uint8):
    any slice of a long stream (e.g. one rank's shard) without the rest."""
    out = np.empty(n, dtype=np.uint8)
    shifts = (np.arange(32, dtype=np.uint64) * np.uint64(2))
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        gs, ge = start + s, start + e
        w0, w1 = gs >> 5, (ge + 31) >> 5
        words = random_words(w1 - w0, seed, w0)
        codes = ((words[:, None] >> shifts[None, :]) & np.uint64(3)).astype(np.uint8).ravel()
        off = gs - (w0 << 5)
        out[s:e] = _ACGT[codes[off:off + (e - s)]]
    return out


def _plant_repeats(bases: np.ndarray, seed: int, per_mb: int, motif_len: int) -> None:
    block = 1_000_000
    motif = random_bases(motif_len, seed ^ 0xA5A5A5A5A5A5A5A5)
    slot = block // per_mb
    n_blocks = (bases.size + block - 1) // block
    for b in range(n_blocks):
        jit = random_words(per_mb, seed ^ 0x5EED0000 ^ b)
        for j in range(per_mb):
            # one copy per slot; when slot <= motif_len copies overlap (later wins)
            room = slot - motif_len
            pos = b * block + j * slot + (int(jit[j] % np.uint64(room)) if room > 0 else 0)
            if pos >= bases.size:
                break
            end = min(pos + motif_len, bases.size)
            bases[pos:end] = motif[:end - pos]


def _sprinkle(bases: np.ndarray, seed: int, n_rate: float, mixed_case: bool) -> None:
    n = bases.size
    if n == 0:
        return
    w = random_words(max(1, n // 64 + 1), seed ^ 0x0DDBA115)
    if n_rate > 0:
        runs = max(1, int(n * n_rate / 8))
        for t in range(runs):
            z = int(w[t % w.size]) ^ (t * 0x9E3779B97F4A7C15 & 0xFFFFFFFFFFFFFFFF)
            pos = z % n
            ln = 1 + (z >> 40) % 15
            bases[pos:pos + ln] = ord("N")
    if mixed_case:
        z = random_words(n // 16 + 1, seed ^ 0x1CA5E)
        sel = np.repeat(z, 16)[:n]
        lower = (sel & np.uint64(0xF)) == 0          # ~1/16 lowercase
        bases[lower] = bases[lower] | 0x20
        odd = (sel >> np.uint64(8) & np.uint64(0x3FF)) == 7  # ~1/1024 other bytes
        others = np.frombuffer(b"RYKMSWBDHVn.-", dtype=np.uint8)
        idx = (sel[odd] >> np.uint64(20)) % np.uint64(others.size)
        bases[odd] = others[idx.astype(np.int64)]


def make_records(total_bases: int, n_recs: int, seed: int = SEED, repeats_per_mb: int = 0,
                 motif_len: int = 200, n_rate: float = 0.0, mixed_case: bool = False):
    """-> (bases uint8[total], offsets uint64[n_recs+1]) : equal-length records,
    the first (total % n_recs) records one base longer."""
    bases = random_bases(total_bases, seed)
    if repeats_per_mb:
        _plant_repeats(bases, seed, repeats_per_mb, motif_len)
    if n_rate > 0 or mixed_case:
        _sprinkle(bases, seed, n_rate, mixed_case)
    q, r = divmod(total_bases, n_recs)
    lens = np.full(n_recs, q, dtype=np.uint64)
    lens[:r] += 1
    offsets = np.zeros(n_recs + 1, dtype=np.uint64)
    np.cumsum(lens, out=offsets[1:])
    return bases, offsets


def make_reads(n_reads: int, read_len: int = 150, seed: int = SEED, **kw):
    """FASTQ-style short reads: n_reads records of read_len bases."""
    return make_records(n_reads * read_len, n_reads, seed, **kw)


def write_fasta(path: str, bases: np.ndarray, offsets: np.ndarray, width: int = 60) -> None:
    with open(path, "wb") as f:
        for i in range(offsets.size - 1):
            s, e = int(offsets[i]), int(offsets[i + 1])
            f.write(b">s%d\n" % i)
            seq = bases[s:e].tobytes()
            for p in range(0, len(seq), width):
                f.write(seq[p:p + width])
                f.write(b"\n")


def write_fastq(path: str, bases: np.ndarray, offsets: np.ndarray, qual: int = ord("I")) -> None:
    with open(path, "wb") as f:
        for i in range(offsets.size - 1):
            s, e = int(offsets[i]), int(offsets[i + 1])
            f.write(b"@r%d\n" % i)
            f.write(bases[s:e].tobytes())
            f.write(b"\n+\n")
            f.write(bytes([qual]) * (e - s))
            f.write(b"\n")


def records_list(bases: np.ndarray, offsets: np.ndarray) -> list[bytes]:
    return [bases[int(offsets[i]):int(offsets[i + 1])].tobytes() for i in range(offsets.size - 1)]


# ---- the same streams generated on a torch device (multi-GB inputs) -------------
# torch has no uint64 arithmetic: int64 wraps the same way for +, * and ^, and a
# logical right shift is an arithmetic one masked to the bits that remain.
def _s64(x: int) -> int:
    x &= 0xFFFFFFFFFFFFFFFF
    return x - (1 << 64) if x >> 63 else x


_C1, _C2, _G = _s64(0xBF58476D1CE4E5B9), _s64(0x94D049BB133111EB), _s64(int(GAMMA))


def _mix_t(z):
    z = z ^ ((z >> 30) & ((1 << 34) - 1))
    z = z * _C1
    z = z ^ ((z >> 27) & ((1 << 37) - 1))
    z = z * _C2
    return z ^ ((z >> 31) & ((1 << 33) - 1))


def random_bases_torch(n: int, seed: int = SEED, start: int = 0, device="cuda",
                       out=None, chunk: int = 1 << 27):
    """random_bases(n, seed, start=start) as a torch uint8 tensor on `device`
    (bit-identical; written into `out[:n]` when given)."""
    import torch
    if out is None:
        out = torch.empty(n, dtype=torch.uint8, device=device)
    lut = torch.tensor(list(b"ACGT"), dtype=torch.uint8, device=out.device)
    shifts = torch.arange(0, 64, 2, dtype=torch.int64, device=out.device)
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        gs, ge = start + s, start + e
        w0, w1 = gs >> 5, (ge + 31) >> 5
        j = torch.arange(w0 + 1, w1 + 1, dtype=torch.int64, device=out.device)
        words = _mix_t(j * _G + _s64(seed))
        codes = ((words[:, None] >> shifts[None, :]) & 3).to(torch.uint8).reshape(-1)
        off = gs - (w0 << 5)
        out[s:e] = lut[codes[off:off + (e - s)].long()]
        del j, words, codes
    return out


def repeat_positions(n: int, seed: int, per_mb: int, motif_len: int) -> np.ndarray:
    """Start of every planted motif copy _plant_repeats places in n bases
    (vectorised; copies must not overlap: slot > motif_len)."""
    block = 1_000_000
    slot = block // per_mb
    room = slot - motif_len
    if room <= 0:
        raise ValueError("overlapping repeat copies: use _plant_repeats")
    n_blocks = (n + block - 1) // block
    b = np.arange(n_blocks, dtype=np.uint64)[:, None]
    j = np.arange(1, per_mb + 1, dtype=np.uint64)[None, :]
    with np.errstate(over="ignore"):
        jit = _mix((np.uint64(seed ^ 0x5EED0000) ^ b) + j * GAMMA)
    pos = (b * np.uint64(block) + (j - np.uint64(1)) * np.uint64(slot) + jit % np.uint64(room))
    pos = pos.astype(np.int64).ravel()
    return pos[pos < n]


def make_records_torch(total_bases: int, n_recs: int, seed: int = SEED, repeats_per_mb: int = 0,
                       motif_len: int = 200, device="cuda", pad: int = 16):
    """make_records(...) (no N/mixed-case sprinkling) generated on `device`:
    -> (uint8 tensor of total_bases + pad bytes, the pad zero; offsets uint64)."""
    import torch
    out = torch.zeros(total_bases + pad, dtype=torch.uint8, device=device)
    random_bases_torch(total_bases, seed, 0, device, out=out)
    if repeats_per_mb:
        motif = torch.from_numpy(random_bases(motif_len, seed ^ 0xA5A5A5A5A5A5A5A5)).to(out.device)
        pos = repeat_positions(total_bases, seed, repeats_per_mb, motif_len)
        ar = torch.arange(motif_len, dtype=torch.int64, device=out.device)
        step = 1 << 20
        for s in range(0, pos.size, step):
            p = torch.from_numpy(pos[s:s + step]).to(out.device)
            idx = (p[:, None] + ar[None, :]).reshape(-1)
            val = motif.repeat(p.numel())
            keep = idx < total_bases
            out[idx[keep]] = val[keep]
    q, r = divmod(total_bases, n_recs)
    lens = np.full(n_recs, q, dtype=np.uint64)
    lens[:r] += 1
    offsets = np.zeros(n_recs + 1, dtype=np.uint64)
    np.cumsum(lens, out=offsets[1:])
    return out, offsets


FASTQ_HDR = 12  # "@r%09d\n"


def fastq_rows_torch(first_read: int, n_reads: int, read_len: int = 150, seed: int = SEED,
                     qual: int = ord("I"), device="cuda"):
    """FASTQ records first_read .. first_read+n_reads-1 of the read stream as a
    (n_reads, 12 + 2*read_len + 4) uint8 tensor: header @r%09d, the read's bases
    = bases [read*read_len, (read+1)*read_len) of random_bases(seed), '+', a
    constant quality line (the layout of tests' _write_fastq_fast)."""
    import torch
    dev = torch.device(device)
    seq = random_bases_torch(n_reads * read_len, seed, first_read * read_len, dev)
    rows = torch.empty((n_reads, FASTQ_HDR + 2 * read_len + 4), dtype=torch.uint8, device=dev)
    rows[:, 0] = ord("@")
    rows[:, 1] = ord("r")
    idx = torch.arange(first_read, first_read + n_reads, dtype=torch.int64, device=dev)
    for d in range(9):
        rows[:, 10 - d] = (idx // (10 ** d) % 10 + 48).to(torch.uint8)
    rows[:, 11] = ord("\n")
    rows[:, FASTQ_HDR:FASTQ_HDR + read_len] = seq.view(n_reads, read_len)
    o = FASTQ_HDR + read_len
    rows[:, o] = ord("\n")
    rows[:, o + 1] = ord("+")
    rows[:, o + 2] = ord("\n")
    rows[:, o + 3:o + 3 + read_len] = qual
    rows[:, -1] = ord("\n")
    return rows


def write_fastq_stream(path: str, first_read: int, n_reads: int, read_len: int = 150,
                       seed: int = SEED, device="cuda", per_chunk: int = 1 << 20) -> int:
    """Write reads first_read .. first_read+n_reads-1 of the stream as FASTQ
    (generated on `device`, copied back chunk by chunk); returns file bytes."""
    with open(path, "wb") as f:
        for s in range(0, n_reads, per_chunk):
            m = min(per_chunk, n_reads - s)
            rows = fastq_rows_torch(first_read + s, m, read_len, seed, device=device)
            f.write(rows.cpu().numpy().tobytes())
            del rows
    return n_reads * (FASTQ_HDR + 2 * read_len + 4)
