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

 private:
  int fd_ = -1;
  void *gzf_ = nullptr;
  bool gz_ = false;
  uint64_t fsize_ = 0, off_ = 0;
};

}  // namespace nk
