// fqbench.cpp — host-side costs of reading a FASTQ file from the page cache
// (config 3's file path): mmap + first touch, munmap, the threaded FASTQ
// extraction (nk_fqhost.cpp) over a warm mapping, parallel pread alone, and
// the extraction reading its windows itself (threads pread, then parse: the
// ingest's form).
//   g++ -O2 -std=c++17 -I include -I neurokmer_amd/csrc tools/fqbench.cpp \
//       neurokmer_amd/csrc/nk_fqhost.cpp -lpthread -o tools/bin/fqbench
//   tools/bin/fqbench <file.fq> [threads] [window]   (writes the file if absent: 10 GB)
#include <fcntl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <chrono>
#include <string>
#include <thread>
#include <vector>

#include "nk_fqhost.h"

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static void write_fastq(const char *path, uint64_t reads, int len) {
  FILE *f = fopen(path, "wb");
  std::vector<char> buf;
  uint64_t x = 0x4E4B4D52;
  std::string rec;
  for (uint64_t r = 0; r < reads; ++r) {
    char hdr[32];
    snprintf(hdr, sizeof hdr, "@r%09llu\n", (unsigned long long)r);
    rec = hdr;
    for (int i = 0; i < len; ++i) {
      x += 0x9E3779B97F4A7C15ull;
      uint64_t z = x;
      z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
      rec.push_back("ACGT"[(z >> 62) & 3]);
    }
    rec += "\n+\n";
    rec.append(len, 'I');
    rec.push_back('\n');
    buf.insert(buf.end(), rec.begin(), rec.end());
    if (buf.size() > (64u << 20)) {
      fwrite(buf.data(), 1, buf.size(), f);
      buf.clear();
    }
  }
  fwrite(buf.data(), 1, buf.size(), f);
  fclose(f);
}

int main(int argc, char **argv) {
  const char *path = argc > 1 ? argv[1] : "/dev/shm/fqbench.fq";
  const int T = argc > 2 ? atoi(argv[2]) : 16;
  const size_t win = argc > 3 ? strtoull(argv[3], nullptr, 10) : (64u << 20);
  struct stat sb;
  if (stat(path, &sb) != 0) {
    double t = now();
    write_fastq(path, 31'600'000ull, 150);
    printf("wrote %s in %.1f s\n", path, now() - t);
    stat(path, &sb);
  }
  const size_t n = (size_t)sb.st_size;
  nk::HostPool pool(T);
  std::vector<uint8_t> hb(win + 16);
  std::vector<uint64_t> he(nk::fq_max_records(win));
  for (int rep = 0; rep < 3; ++rep) {
    // (a) fresh mapping: the extraction pays the page faults; then munmap
    int fd = open(path, O_RDONLY);
    double t0 = now();
    const uint8_t *p = (const uint8_t *)mmap(nullptr, n, PROT_READ, MAP_PRIVATE, fd, 0);
    double t1 = now();
    uint64_t pos = 0, recs = 0, bases = 0;
    while (pos < n) {
      const size_t len = std::min<size_t>(win, n - pos);
      nk::FqResult r = nk::fq_extract(const_cast<uint8_t *>(p + pos), len, pos + len >= n, hb.data(), he.data(), 0, pool);
      pos += r.consumed;
      recs += r.n_rec;
      bases += r.n_bases;
      if (r.stop || r.blank || (!r.n_rec && pos + len >= n)) break;
    }
    double t2 = now();
    // (b) the same mapping again: no faults
    pos = 0;
    while (pos < n) {
      const size_t len = std::min<size_t>(win, n - pos);
      nk::FqResult r = nk::fq_extract(const_cast<uint8_t *>(p + pos), len, pos + len >= n, hb.data(), he.data(), 0, pool);
      pos += r.consumed;
      if (r.stop || r.blank || (!r.n_rec && pos + len >= n)) break;
    }
    double t3 = now();
    munmap((void *)p, n);
    double t4 = now();
    // (c) parallel pread of the file into a 64 MB buffer, window by window
    pos = 0;
    while (pos < n) {
      const size_t len = std::min<size_t>(win, n - pos);
      pool.run([&](int t) {
        const size_t a = len * t / T, b = len * (t + 1) / T;
        size_t g = 0;
        while (a + g < b) {
          ssize_t k = pread(fd, hb.data() + a + g, b - a - g, (off_t)(pos + a + g));
          if (k <= 0) break;
          g += (size_t)k;
        }
      });
      pos += len;
    }
    double t5 = now();
    // (d) the ingest's form: each thread preads its slice, then the parse
    std::vector<uint8_t> rb(win + 64);
    pos = 0;
    while (pos < n) {
      const size_t len = std::min<size_t>(win, n - pos);
      nk::FqResult r = nk::fq_extract(rb.data(), len, pos + len >= n, hb.data(), he.data(), 0, pool, fd, pos);
      pos += r.consumed;
      if (r.stop || r.blank || (!r.n_rec && pos + len >= n)) break;
    }
    double t6 = now();
    close(fd);
    printf("rep %d: %.2f GB, %llu records, %.2f Gbases | mmap %.1f ms, extract (faulting) %.1f ms, "
           "extract (warm) %.1f ms, munmap %.1f ms, pread %.1f ms, pread+extract %.1f ms\n",
           rep, n / 1e9, (unsigned long long)recs, bases / 1e9, (t1 - t0) * 1e3, (t2 - t1) * 1e3,
           (t3 - t2) * 1e3, (t4 - t3) * 1e3, (t5 - t4) * 1e3, (t6 - t5) * 1e3);
  }
  return 0;
}
