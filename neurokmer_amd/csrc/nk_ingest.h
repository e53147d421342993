// GPU FASTA/FASTQ ingest: raw file bytes, copied to the
// device in chunks, are parsed on the device into the resident input of a
// counter (bases u8 + record offsets u64), mirroring the host reader's rules
// (nk_fastx.cpp, needletail 0.6.3 semantics, src/utils.rs:9-24):
//   FASTA: a line whose first byte is '>' starts a record; every other byte
//          except '\n' and '\r' is a base.
//   FASTQ: records of four lines (header '@', sequence, '+' line, quality);
//          one trailing '\r' per line is dropped; the stream stops at the first
//          record that is malformed (header not '@', '+' line missing or
//          empty, quality length != sequence length, cut off by the end of
//          the input).  A blank line where a header is due (which the host
//          reader skips) is reported and the caller falls back to it.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace nk {

// Parser state carried across chunks (device memory; read back per chunk).
struct IngestState {
  unsigned long long data_end;   // bases in the resident buffer
  unsigned long long n_rec;      // records started (offsets[0 .. n_rec-1] written)
  // FASTA: the chunk boundary splits a line
  uint32_t at_line_start;        // the next chunk starts at a line start
  uint32_t line_is_hdr;          // else: the unfinished line is a header line
  // FASTQ (the chunk starts at a record boundary)
  unsigned long long consumed;   // bytes of the chunk covered by complete records
  uint32_t stop;                 // a malformed record ended the stream
  uint32_t blank;                // a blank line where a header was due (fall back)
};

struct IngestBufs {
  uint8_t *bases;                // resident bases, capacity cap_bases
  uint64_t *offsets;             // resident record offsets, capacity cap_recs + 1
  unsigned long long cap_bases, cap_recs;
  // scratch, sized by ingest_scratch_bytes(chunk capacity)
  void *scratch;
};

size_t ingest_scratch_bytes(size_t chunk_cap);

// Parses raw[0 .. len) (device) as the next FASTA chunk; eof: last chunk.
// Appends to bufs, updates *st (device), offsets[n_rec] = data_end afterwards.
hipError_t ingest_fasta(const uint8_t *raw, size_t len, bool eof, const IngestBufs &bufs,
                        IngestState *st, hipStream_t s);
// Parses the complete FASTQ records of raw[0 .. len) (starts at a record
// boundary); st->consumed = bytes used.  eof: the last line may lack '\n'.
hipError_t ingest_fastq(const uint8_t *raw, size_t len, bool eof, const IngestBufs &bufs,
                        IngestState *st, hipStream_t s);

}  // namespace nk
