// nk_fqhost.h — FASTQ records of a mapped file, parsed by host threads into
// sequence bytes + record ends (config 3: only the sequence lines cross PCIe).
//
// The reference's reader hands only sequence bytes to the counter
// (stream_sequences, src/utils.rs:9-24 -> src/spiking_hash.rs:408-422); the
// device FASTQ parse (nk_ingest.h) needed every file byte on the device --
// headers and quality lines are ~52 % of a 150-bp FASTQ.  Same record rules as
// nk_ingest.h / nk_fastx.cpp:
//   records of four lines (header '@', sequence, '+' line, quality); one
//   trailing '\r' per line is dropped; the stream stops at the first malformed
//   record (header not '@', '+' line missing or empty, quality length !=
//   sequence length, cut off by the end of the input); a blank line where a
//   header is due is reported (the caller falls back to the host reader, which
//   skips it), except blank lines that end the input.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <atomic>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace nk {

// A fixed set of host threads running one function on every thread at a time.
// A call hands its function over through a generation counter the threads
// spin on for a while before they block (a window of the FASTQ ingest is three
// calls ~0.3 ms apart: a condition-variable round trip per call was ~30 us).
class HostPool {
 public:
  explicit HostPool(int threads);
  ~HostPool();
  HostPool(const HostPool &) = delete;
  HostPool &operator=(const HostPool &) = delete;
  int size() const { return n_; }
  // fn(t) for t = 0 .. size()-1 (t = 0 on the calling thread); returns when all are done
  void run(const std::function<void(int)> &fn);

 private:
  void loop(int t);
  int n_;
  std::vector<std::thread> th_;
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  const std::function<void(int)> *fn_ = nullptr;
  std::mutex run_mu_;
  std::atomic<uint64_t> gen_{0};
  std::atomic<int> pending_{0};
  std::atomic<bool> quit_{false};
};

struct FqResult {
  uint64_t consumed = 0;  // input bytes of the records taken (the next call starts there)
  uint64_t n_rec = 0;     // records taken
  uint64_t n_bases = 0;   // sequence bytes written
  bool stop = false;      // a malformed record follows them: the stream ends
  bool blank = false;     // a blank line where a header is due follows them
  bool more = false;      // max_rec cut the window: records follow (call again from consumed)
  // fd >= 0: a read of the window failed or the file ended before its size
  // (nothing is taken: the caller fails with NK_E_IO instead of a silent stop)
  std::string io_error;
};

// The process's one pool (at most 16 threads: a one-GPU box's CPU share),
// shared by every handle's FASTQ ingest (a pool per handle multiplied the
// spinning threads with the handles)
HostPool &shared_host_pool();

// Records a window of `len` input bytes can hold: len / 6 + 1 (a record has
// at least 6 bytes: "@\n\n+\n\n").  A caller with less room for record ends
// passes max_rec to fq_extract.
inline size_t fq_max_records(size_t len) { return len / 6 + 1; }

// Newline positions per thread, kept between calls (allocating ~1.5 MB per
// thread per window cost more than the scan at small windows, profiles/r05_g)
struct FqScratch {
  std::vector<std::vector<uint32_t>> nl;
};

// The FASTQ records of in[0, len), which starts at a record boundary; eof: the
// input ends at len (its last line may lack '\n').  Writes every taken record's
// sequence to bases (contiguous) and ends[i] = base_off + the end of record i's
// sequence in bases.  len < 2^32.  Without eof, a record cut by the window end
// is not taken (n_rec == 0 and !stop: the caller widens the window).
// fd >= 0: in[0, len) is first read from the file at file_off, each thread its
// slice (pread straight into the buffer it then scans: the bytes are read from
// the page cache once and scanned from the thread's cache; a mapping of the
// file measured slower -- page faults, and an munmap as long as the parse,
// profiles/r05_f).
FqResult fq_extract(uint8_t *in, size_t len, bool eof, uint8_t *bases, uint64_t *ends,
                    uint64_t base_off, HostPool &pool, int fd = -1, uint64_t file_off = 0,
                    FqScratch *scratch = nullptr, uint64_t max_rec = ~0ull);

// A file opened for reading, with its size.
class HostFile {
 public:
  ~HostFile();
  int open(const char *path, std::string &err);  // 0 or an NK_E_* code
  int fd() const { return fd_; }
  uint64_t size() const { return n_; }
  const std::string &path() const { return path_; }

 private:
  int fd_ = -1;
  uint64_t n_ = 0;
  std::string path_;
};

}  // namespace nk
