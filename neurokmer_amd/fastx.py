"""stream_sequences — Python mirror of src/utils.rs:9-24 (needletail 0.6.3 parse).

Same rules as the native reader (neurokmer_amd/csrc/nk_fastx.cpp): format from
the first byte ('>' FASTA, '@' FASTQ), gzip transparent, FASTA sequence lines
joined with '\\r'/'\\n' removed, and the stream ENDS at the first malformed
record (the reference maps the parse error to `None`).  Raises on an empty
file or an unknown first byte, like parse_fastx_file.
"""
from __future__ import annotations

import gzip
import sys
from typing import Iterator


def _warn(path: str, record: int, why: str) -> None:
    """src/utils.rs:17-19's `warn!("Skipping malformed record: {}", e)` (stderr)."""
    print(f"[WARN  neurokmer] Skipping malformed record: {why} (record {record} of {path}); "
          "the input ends here", file=sys.stderr)


def _open(path: str):
    with open(path, "rb") as f:
        magic = f.read(2)
    return gzip.open(path, "rb") if magic == b"\x1f\x8b" else open(path, "rb")


def stream_sequences(path: str) -> Iterator[bytes]:
    f = _open(path)
    first = f.read(1)
    if not first:
        f.close()
        raise ValueError("empty file")
    if first not in (b">", b"@"):
        f.close()
        raise ValueError("unknown format: first byte is neither '>' nor '@'")
    fastq = first == b"@"

    def gen():
        with f:
            f.readline()  # rest of the first header
            if not fastq:
                seq = bytearray()
                for line in f:
                    if line.startswith(b">"):
                        yield bytes(seq)
                        seq = bytearray()
                        continue
                    seq += line.replace(b"\r", b"").replace(b"\n", b"")
                yield bytes(seq)
            else:
                header_pending = True
                n = 0
                while True:
                    if not header_pending:
                        line = f.readline()
                        while line in (b"\n", b"\r\n"):
                            line = f.readline()
                        if not line:
                            return
                        if not line.startswith(b"@"):
                            _warn(path, n, "expected '@' at the start of a FASTQ record")
                            return
                    header_pending = False
                    seq = f.readline()
                    plus = f.readline()
                    qual = f.readline()
                    if not seq or not plus.startswith(b"+") or not qual:
                        _warn(path, n, "a FASTQ record is malformed or cut off")
                        return
                    seq = seq.rstrip(b"\n").rstrip(b"\r")
                    qual = qual.rstrip(b"\n").rstrip(b"\r")
                    if len(qual) != len(seq):
                        _warn(path, n, "quality and sequence lengths differ")
                        return
                    n += 1
                    yield seq

    return gen()
