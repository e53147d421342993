// nk_reader.h — raw file chunks for the GPU FASTX ingest (nk_ingest.h).
// Plain files: parallel pread() straight into the caller's (pinned) buffer;
// gzip files: zlib's stream (host decompression).
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <string>

namespace nk {

class ChunkSource {
 public:
  ~ChunkSource();
  // 0 or an NK_E_* code (err set)
  int open(const char *path, std::string &err);
  // reads up to `want` bytes into dst; returns the bytes read (< want: end of input)
  size_t read(uint8_t *dst, size_t want);
  bool gz() const { return gz_; }
  uint64_t file_size() const { return fsize_; }
  // a read failed (errno), a plain file ended before its size, or the gzip
  // stream is corrupt: the bytes returned end early and must not be taken
  // for the end of the input
  bool failed() const { return !why_.empty(); }
  const std::string &why() const { return why_; }
  // the gzip stream is damaged or cut off: the input ends there, as at a
  // malformed record (the caller warns)
  const std::string &damage() const { return damage_; }

 private:
  int fd_ = -1;
  void *gzf_ = nullptr;
  bool gz_ = false;
  uint64_t fsize_ = 0, off_ = 0;
  std::string why_, damage_;
};

}  // namespace nk
