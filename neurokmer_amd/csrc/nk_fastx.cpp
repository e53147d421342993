// nk_fastx.cpp — see nk_fastx.h.
#include "nk_fastx.h"

#include <string.h>
#include <zlib.h>

#include "neurokmer.h"

namespace nk {

static constexpr size_t kBuf = 1 << 22;

FastxReader::~FastxReader() {
  if (gz_) gzclose((gzFile)gz_);
}

bool FastxReader::fill() {
  if (eof_) return false;
  if (buf_.size() < kBuf) buf_.resize(kBuf);
  int n = gzread((gzFile)gz_, buf_.data(), (unsigned)kBuf);
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
    } else {
      // header already consumed when pending_header_ is set
      if (!pending_header_) {
        int c;
        do { c = read_byte(); } while (c == '\n' || c == '\r');
        if (c < 0) { done_ = true; break; }
        if (c != '@') { truncated_ = true; done_ = true; break; }
        read_line(line_, true);
      }
      pending_header_ = false;
      std::string seq, plus, qual;
      if (!read_line(seq, true) || !read_line(plus, true) || plus.empty() || plus[0] != '+' ||
          !read_line(qual, true) || qual.size() != seq.size()) {
        truncated_ = true;
        done_ = true;
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
  return NK_OK;
}

}  // namespace nk
