// nk_fastx.h — host FASTA/FASTQ reader (the build's stand-in for needletail 0.6.3,
// reached through stream_sequences, src/utils.rs:9-24).
//
// Semantics kept from the reference path:
//   * format from the first byte: '>' FASTA, '@' FASTQ; anything else or an
//     empty file is an error (needletail's parse_fastx_file);
//   * gzip input is decompressed transparently (zlib);
//   * FASTA sequence = every line after the header up to the next '>' line,
//     with '\r' and '\n' removed;  FASTQ sequence = the sequence line;
//   * the first malformed record ENDS the stream (stream_sequences maps the
//     error to `None`, src/utils.rs:16-20): records before it are kept.
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

namespace nk {

class FastxReader {
 public:
  FastxReader() = default;
  ~FastxReader();
  FastxReader(const FastxReader &) = delete;
  FastxReader &operator=(const FastxReader &) = delete;

  // 0 on success, NK_E_IO / NK_E_PARSE with err set otherwise.
  int open(const char *path, std::string &err);
  // Appends whole records to bases/offsets (offsets gets one entry per record
  // end; the caller seeds offsets with {0}) until at least max_bases bases are
  // buffered or the input ends.  Returns 1 if records were appended, 0 at end.
  int next_batch(size_t max_bases, std::vector<uint8_t> &bases, std::vector<uint64_t> &offsets);
  bool truncated() const { return truncated_; }  // stopped at a malformed record
  uint64_t records() const { return n_records_; }
  // the input could not be read to its end (gzip/read error): not a malformed record
  bool io_error() const { return !io_why_.empty(); }
  const std::string &io_why() const { return io_why_; }
  void set_path(const std::string &p) { path_ = p; }

 private:
  bool fill();
  int read_byte();
  bool read_line(std::string &line, bool strip_cr);

  void *gz_ = nullptr;
  std::vector<uint8_t> buf_;
  size_t pos_ = 0, len_ = 0;
  bool eof_ = false;
  bool fastq_ = false;
  bool done_ = false;
  bool truncated_ = false;
  bool pending_header_ = false;  // FASTA: a '>' line was consumed for the next record
  uint64_t n_records_ = 0;
  std::string line_;
  std::string io_why_, path_;
  std::string damage_;  // the gzip stream is damaged or cut off (zlib's message)
};

// The reference's `warn!("Skipping malformed record: {}", e)` when the stream
// stops at a malformed record (src/utils.rs:17-19): one line on stderr naming
// the record (0-based index among the records read) and the reason.
void warn_malformed(const char *path, uint64_t record, const char *why);

// Whole-file convenience (in-memory mode, src/main.rs:44).
int read_fastx_all(const char *path, std::vector<uint8_t> &bases, std::vector<uint64_t> &offsets,
                   std::string &err);

}  // namespace nk
