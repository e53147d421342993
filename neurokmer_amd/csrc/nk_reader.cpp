// nk_reader.cpp — see nk_reader.h.
#include "nk_reader.h"

#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>
#include <zlib.h>

#include <errno.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <thread>
#include <vector>

#include "neurokmer.h"
#include "nk_fqhost.h"

namespace nk {

ChunkSource::~ChunkSource() {
  if (gzf_) gzclose((gzFile)gzf_);
  if (fd_ >= 0) ::close(fd_);
}

int ChunkSource::open(const char *path, std::string &err) {
  fd_ = ::open(path, O_RDONLY);
  if (fd_ < 0) {
    err = std::string("cannot open ") + path;
    return NK_E_IO;
  }
  struct stat sb;
  if (fstat(fd_, &sb) == 0) fsize_ = (uint64_t)sb.st_size;
  unsigned char m[2] = {0, 0};
  gz_ = pread(fd_, m, 2, 0) == 2 && m[0] == 0x1f && m[1] == 0x8b;
  if (gz_) {
    gzFile f = gzdopen(dup(fd_), "rb");
    if (!f) {
      err = std::string("cannot open ") + path;
      return NK_E_IO;
    }
    gzbuffer(f, 1 << 20);
    gzf_ = f;
  }
  return NK_OK;
}

size_t ChunkSource::read(uint8_t *dst, size_t want) {
  if (!want) return 0;
  if (gz_) {
    size_t got = 0;
    while (got < want) {
      const int n = gzread((gzFile)gzf_, dst + got,
                           (unsigned)std::min<size_t>(want - got, (size_t)1 << 30));
      if (n <= 0) {
        int zerr = 0;
        const char *m = gzerror((gzFile)gzf_, &zerr);
        if (zerr == Z_ERRNO) why_ = std::string("read failed: ") + strerror(errno);
        else if (zerr != Z_OK) damage_ = std::string("gzip: ") + (m ? m : "?");
        break;
      }
      got += (size_t)n;
    }
    return got;
  }
  // plain file: split the read over the process's host pool (page-cache
  // copies run at the memory bandwidth of several cores, one core copies ~5-10
  // GB/s; up to 16 threads, a one-GPU box's CPU share: 8 read a 10 GB FASTQ
  // from the page cache at ~24 GB/s, profiles/r04_s2).  Parts of >= 1 MiB, so
  // a 16 MiB piece of a chunk (nk_ingest_host.cpp) still takes 16 threads;
  // the pool's threads persist (a thread per part and call cost ~15 us each).
  HostPool &pool = shared_host_pool();
  const size_t part = (size_t)1 << 20;
  const int nt = (int)std::max<size_t>(1, std::min<size_t>((size_t)pool.size(), (want + part - 1) / part));
  std::vector<size_t> got(nt, 0);
  std::atomic<int> err_no{0};
  auto work = [&](int t) {
    if (t >= nt) return;
    const size_t lo = want * t / nt, hi = want * (t + 1) / nt;
    size_t g = 0;
    while (lo + g < hi) {
      const ssize_t n = pread(fd_, dst + lo + g, hi - lo - g, (off_t)(off_ + lo + g));
      if (n < 0 && errno == EINTR) continue;
      if (n < 0) err_no = errno;
      if (n <= 0) break;
      g += (size_t)n;
    }
    got[t] = g;
  };
  if (nt <= 1) work(0);
  else pool.run(work);
  size_t total = 0;  // contiguous from the start: a short part ends the file
  for (int t = 0; t < nt; ++t) {
    total += got[t];
    if (got[t] < want * (t + 1) / nt - want * t / nt) break;
  }
  // the file's size is known: fewer bytes than it holds is a failure, not its end
  if (err_no.load())
    why_ = std::string("read failed at byte ") + std::to_string(off_ + total) + ": " + strerror(err_no.load());
  else if (total < want && off_ + total < fsize_)
    why_ = "the file ended at byte " + std::to_string(off_ + total) + " of " + std::to_string(fsize_) +
           " while it was read";
  off_ += total;
  return total;
}

}  // namespace nk
