// nk_fastx.cpp — see nk_fastx.h.
#include "nk_fastx.h"

#include <errno.h>
#include <stdio.h>
#include <string.h>
#include <zlib.h>

#include "neurokmer.h"

namespace nk {

static constexpr size_t kBuf = 1 << 22;

FastxReader::~FastxReader() {
  if (gz_) gzclose((gzFile)gz_);
}

void warn_malformed(const char *path, uint64_t record, const char *why) {
  fprintf(stderr, "[WARN  neurokmer] Skipping malformed record: %s (record %llu of %s); the input ends here\n",
          why, (unsigned long long)record, path ? path : "the input");
}

bool FastxReader::fill() {
  if (eof_) return false;
  if (buf_.size() < kBuf) buf_.resize(kBuf);
  int n = gzread((gzFile)gz_, buf_.data(), (unsigned)kBuf);
  if (n <= 0) {
    // an operating-system read error fails the call (NK_E_IO); a damaged or
    // cut-off gzip stream ends the input like a malformed record
    int zerr = 0;
    const char *m = gzerror((gzFile)gz_, &zerr);
    if (zerr == Z_ERRNO) io_why_ = std::string("read failed: ") + strerror(errno);
    else if (zerr != Z_OK) damage_ = std::string("gzip: ") + (m ? m : "?");
  }
  if (n <= 0) {
    eof_ = true;
    len_ = pos_ = 0;
    return false;
  }
  len_ = (size_t)n;
  pos_ = 0;
  return true;
}

int FastxReader::read_byte() {
  if (pos_ >= len_ && !fill()) return -1;
  return buf_[pos_++];
}

// Reads one line without its '\n'; false at end of input with nothing read.
bool FastxReader::read_line(std::string &line, bool strip_cr) {
  line.clear();
  bool any = false;
  for (;;) {
    if (pos_ >= len_ && !fill()) break;
    const uint8_t *s = buf_.data() + pos_;
    const uint8_t *nl = (const uint8_t *)memchr(s, '\n', len_ - pos_);
    size_t take = nl ? (size_t)(nl - s) : len_ - pos_;
    line.append((const char *)s, take);
    any = true;
    pos_ += take;
    if (nl) {
      ++pos_;
      break;
    }
  }
  if (strip_cr && !line.empty() && line.back() == '\r') line.pop_back();
  return any;
}

int FastxReader::open(const char *path, std::string &err) {
  path_ = path;
  gzFile f = gzopen(path, "rb");
  if (!f) {
    err = std::string("cannot open ") + path;
    return NK_E_IO;
  }
  gzbuffer(f, 1 << 20);
  gz_ = f;
  int c = read_byte();
  if (c < 0) {
    err = "empty file";
    return NK_E_PARSE;
  }
  if (c == '>') fastq_ = false;
  else if (c == '@') fastq_ = true;
  else {
    err = "unknown format: first byte is neither '>' nor '@'";
    return NK_E_PARSE;
  }
  // the header line of the first record
  std::string hdr;
  read_line(hdr, true);
  pending_header_ = true;
  return NK_OK;
}

int FastxReader::next_batch(size_t max_bases, std::vector<uint8_t> &bases,
                            std::vector<uint64_t> &offsets) {
  if (done_) return 0;
  const size_t start = bases.size();
  bool appended = false;
  while (!done_ && bases.size() - start < max_bases) {
    if (!fastq_) {
      if (!pending_header_) { done_ = true; break; }
      pending_header_ = false;
      // sequence lines until the next '>' at a line start
      for (;;) {
        int c = read_byte();
        if (c < 0) { done_ = true; break; }
        if (c == '>') {
          read_line(line_, true);  // header of the next record
          pending_header_ = true;
          break;
        }
        --pos_;  // put back (pos_ > 0: the byte came from the buffer)
        read_line(line_, false);
        for (char ch : line_)
          if (ch != '\r') bases.push_back((uint8_t)ch);
      }
      offsets.push_back(bases.size());
      ++n_records_;
      appended = true;
      if (done_ && !damage_.empty() && !io_error()) {  // the last record ran into a damaged stream
        truncated_ = true;
        warn_malformed(path_.c_str(), n_records_ - 1, damage_.c_str());
      }
    } else {
      // header already consumed when pending_header_ is set
      if (!pending_header_) {
        int c;
        do { c = read_byte(); } while (c == '\n' || c == '\r');
        if (c < 0) {
          done_ = true;
          if (!damage_.empty() && !io_error()) {
            truncated_ = true;
            warn_malformed(path_.c_str(), n_records_, damage_.c_str());
          }
          break;
        }
        if (c != '@') {
          truncated_ = true;
          done_ = true;
          if (!io_error()) warn_malformed(path_.c_str(), n_records_, "expected '@' at the start of a FASTQ record");
          break;
        }
        read_line(line_, true);
      }
      pending_header_ = false;
      std::string seq, plus, qual;
      const bool s_ok = read_line(seq, true), p_ok = s_ok && read_line(plus, true);
      const bool q_ok = p_ok && !plus.empty() && plus[0] == '+' && read_line(qual, true);
      if (!q_ok || qual.size() != seq.size()) {
        truncated_ = true;
        done_ = true;
        if (!io_error())
          warn_malformed(path_.c_str(), n_records_,
                         !damage_.empty() ? damage_.c_str()
                         : !s_ok || !p_ok ? "unexpected end of input inside a FASTQ record"
                         : plus.empty() || plus[0] != '+' ? "the separator line is not '+'"
                         : !q_ok ? "unexpected end of input inside a FASTQ record"
                                 : "quality and sequence lengths differ");
        break;
      }
      bases.insert(bases.end(), seq.begin(), seq.end());
      offsets.push_back(bases.size());
      ++n_records_;
      appended = true;
    }
  }
  return appended ? 1 : 0;
}

int read_fastx_all(const char *path, std::vector<uint8_t> &bases, std::vector<uint64_t> &offsets,
                   std::string &err) {
  FastxReader r;
  int rc = r.open(path, err);
  if (rc) return rc;
  bases.clear();
  offsets.assign(1, 0);
  while (r.next_batch((size_t)1 << 30, bases, offsets)) {
  }
  if (r.io_error()) {
    err = std::string(path) + ": " + r.io_why();
    return NK_E_IO;
  }
  return NK_OK;
}

}  // namespace nk
