// nk_fqhost.cpp — see nk_fqhost.h.
#include "nk_fqhost.h"

#if defined(__x86_64__) || defined(__i386__)
#include <emmintrin.h>
#define NK_RELAX() _mm_pause()
#else
#define NK_RELAX() std::this_thread::yield()
#endif
#include <errno.h>
#include <fcntl.h>
#include <string.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>

#include "neurokmer.h"

namespace nk {

// ---- HostPool ---------------------------------------------------------------
namespace {
constexpr int kSpin = 1 << 14;  // pause iterations before a thread blocks (~0.2-0.5 ms)
}

HostPool::HostPool(int threads) : n_(std::max(1, threads)) {
  for (int t = 1; t < n_; ++t) th_.emplace_back(&HostPool::loop, this, t);
}

HostPool::~HostPool() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    quit_.store(true);
  }
  cv_.notify_all();
  for (auto &t : th_) t.join();
}

void HostPool::loop(int t) {
  uint64_t seen = 0;
  for (;;) {
    uint64_t g = gen_.load(std::memory_order_acquire);
    for (int i = 0; g == seen && !quit_.load(std::memory_order_relaxed); ++i) {
      if (i < kSpin) {
        NK_RELAX();
      } else {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return gen_.load(std::memory_order_acquire) != seen || quit_.load(); });
      }
      g = gen_.load(std::memory_order_acquire);
    }
    if (quit_.load()) return;
    seen = g;
    (*fn_)(t);
    if (pending_.fetch_sub(1, std::memory_order_acq_rel) == 1) {
      std::lock_guard<std::mutex> lk(mu_);
      done_cv_.notify_one();
    }
  }
}

void HostPool::run(const std::function<void(int)> &fn) {
  std::lock_guard<std::mutex> one(run_mu_);  // one call at a time (handles on several host threads)
  if (n_ == 1) {
    fn(0);
    return;
  }
  fn_ = &fn;
  pending_.store(n_ - 1, std::memory_order_relaxed);
  gen_.fetch_add(1, std::memory_order_release);
  {
    std::lock_guard<std::mutex> lk(mu_);  // (a thread between its check and its wait sees gen_)
  }
  cv_.notify_all();
  fn(0);
  for (int i = 0; pending_.load(std::memory_order_acquire) != 0; ++i) {
    if (i < kSpin) {
      NK_RELAX();
    } else {
      std::unique_lock<std::mutex> lk(mu_);
      done_cv_.wait(lk, [&] { return pending_.load(std::memory_order_acquire) == 0; });
    }
  }
}

// ---- HostFile ---------------------------------------------------------------
HostFile::~HostFile() {
  if (fd_ >= 0) ::close(fd_);
}

int HostFile::open(const char *path, std::string &err) {
  path_ = path;
  fd_ = ::open(path, O_RDONLY);
  if (fd_ < 0) {
    err = std::string("cannot open ") + path;
    return NK_E_IO;
  }
  struct stat sb;
  if (fstat(fd_, &sb) != 0) {
    err = std::string("cannot stat ") + path;
    return NK_E_IO;
  }
  n_ = (uint64_t)sb.st_size;
  return NK_OK;
}

// ---- fq_extract ---------------------------------------------------------------
namespace {

// positions of '\n' in p[a, b), appended to out (64 B per step, SSE2)
void find_newlines(const uint8_t *p, size_t a, size_t b, std::vector<uint32_t> &out) {
  size_t i = a;
  while (i < b && ((uintptr_t)(p + i) & 15)) {
    if (p[i] == '\n') out.push_back((uint32_t)i);
    ++i;
  }
#if defined(__x86_64__) || defined(__i386__)
  const __m128i nl = _mm_set1_epi8('\n');
  for (; i + 64 <= b; i += 64) {
    const __m128i *q = reinterpret_cast<const __m128i *>(p + i);
    uint64_t m = (uint64_t)(uint32_t)_mm_movemask_epi8(_mm_cmpeq_epi8(_mm_load_si128(q), nl)) |
                 ((uint64_t)(uint32_t)_mm_movemask_epi8(_mm_cmpeq_epi8(_mm_load_si128(q + 1), nl)) << 16) |
                 ((uint64_t)(uint32_t)_mm_movemask_epi8(_mm_cmpeq_epi8(_mm_load_si128(q + 2), nl)) << 32) |
                 ((uint64_t)(uint32_t)_mm_movemask_epi8(_mm_cmpeq_epi8(_mm_load_si128(q + 3), nl)) << 48);
    while (m) {
      out.push_back((uint32_t)(i + (size_t)__builtin_ctzll(m)));
      m &= m - 1;
    }
  }
#else
  for (const uint8_t *q; i < b && (q = (const uint8_t *)memchr(p + i, '\n', b - i)); i = (size_t)(q - p) + 1)
    out.push_back((uint32_t)(q - p));
  i = b;
#endif
  for (; i < b; ++i)
    if (p[i] == '\n') out.push_back((uint32_t)i);
}


// the lines of the window: line i ends at the i-th '\n' (or, the extra
// unterminated last line at eof, at len) and starts after line i - 1
struct Lines {
  const std::vector<uint32_t> *nl;  // per thread
  std::vector<uint64_t> pre;        // newlines before thread t's
  int T;
  uint64_t N;                       // newlines
  uint64_t len;
  uint64_t end(uint64_t i, int &h) const {  // h: a thread hint (monotone use is O(1))
    if (i >= N) return len;
    while (h > 0 && pre[h] > i) --h;
    while (h + 1 < T && pre[h + 1] <= i) ++h;
    return nl[h][i - pre[h]];
  }
  uint64_t start(uint64_t i, int &h) const { return i ? end(i - 1, h) + 1 : 0; }
};

enum Problem : int { kNone = 0, kBad = 1, kBlank = 2 };

}  // namespace

HostPool &shared_host_pool() {
  static HostPool pool([] {  // the box's CPU share for one GPU (at most 16 threads)
    const unsigned hc = std::thread::hardware_concurrency();
    return (int)std::max<unsigned>(1, std::min<unsigned>(16, hc ? hc : 8));
  }());
  return pool;
}

FqResult fq_extract(uint8_t *in, size_t len, bool eof, uint8_t *bases, uint64_t *ends,
                    uint64_t base_off, HostPool &pool, int fd, uint64_t file_off, FqScratch *scratch,
                    uint64_t max_rec) {
  FqResult res;
  if (!len) return res;
  const int T = (int)std::min<size_t>((size_t)pool.size(), std::max<size_t>(1, len >> 16));
  // (1) every thread indexes the newlines of its slice
  FqScratch local;
  std::vector<std::vector<uint32_t>> &nl = (scratch ? scratch : &local)->nl;
  if (nl.size() < (size_t)pool.size()) nl.resize(pool.size());
  std::vector<int> rd_err(T, 0);      // errno of a failed read (-1: the file ended early)
  std::vector<uint64_t> rd_at(T, 0);  // file offset where it failed
  pool.run([&](int t) {
    if (t >= T) return;
    const size_t a = len * t / T, b = len * (t + 1) / T;
    if (fd >= 0) {  // this thread's slice, from the page cache
      size_t g = 0;
      while (a + g < b) {
        const ssize_t r = pread(fd, in + a + g, b - a - g, (off_t)(file_off + a + g));
        if (r < 0 && errno == EINTR) continue;
        if (r <= 0) {
          rd_err[t] = r < 0 ? errno : -1;
          rd_at[t] = file_off + a + g;
          break;
        }
        g += (size_t)r;
      }
      if (a + g < b) return;  // (reported below; nothing of this window is taken)
    }
    nl[t].clear();
    nl[t].reserve((b - a) / 48 + 64);
    find_newlines(in, a, b, nl[t]);
  });
  for (int t = 0; t < T; ++t)
    if (rd_err[t]) {
      res.io_error = rd_err[t] > 0 ? std::string("read failed at byte ") + std::to_string(rd_at[t]) + ": " +
                                         strerror(rd_err[t])
                                   : "the file ended at byte " + std::to_string(rd_at[t]) +
                                         " before its size while it was read";
      return res;
    }
  Lines L;
  L.nl = nl.data();
  L.T = T;
  L.len = len;
  L.pre.assign(T + 1, 0);
  for (int t = 0; t < T; ++t) L.pre[t + 1] = L.pre[t] + nl[t].size();
  L.N = L.pre[T];
  // an unterminated last line at eof (bytes after the last '\n')
  uint64_t last_nl = 0;
  bool any_nl = false;
  for (int t = T - 1; t >= 0; --t)
    if (!nl[t].empty()) {
      last_nl = nl[t].back();
      any_nl = true;
      break;
    }
  const bool tail_line = eof && (any_nl ? last_nl + 1 < len : len > 0);
  const uint64_t n_lines = L.N + (tail_line ? 1 : 0);
  const uint64_t R = n_lines / 4;
  // (2) records checked in parallel: each thread its range, its first problem
  std::vector<uint64_t> first(T, ~0ull), sum(T, 0);
  std::vector<int> kind(T, kNone);
  pool.run([&](int t) {
    if (t >= T) return;
    const uint64_t r0 = R * t / T, r1 = R * (t + 1) / T;
    int h = 0;
    uint64_t s = 0;
    for (uint64_t r = r0; r < r1; ++r) {
      const uint64_t l = 4 * r;
      const uint64_t h0 = L.start(l, h), h1 = L.end(l, h);
      const uint64_t s0 = h1 + 1, s1 = L.end(l + 1, h);
      const uint64_t p0 = s1 + 1, p1 = L.end(l + 2, h);
      const uint64_t q0 = p1 + 1, q1 = L.end(l + 3, h);
      int k = kNone;
      if (h1 == h0 || in[h0] == '\r') k = kBlank;
      else if (in[h0] != '@') k = kBad;
      else if (p1 == p0 || in[p0] != '+') k = kBad;
      else {
        const uint64_t sl = s1 - s0 - (s1 > s0 && in[s1 - 1] == '\r' ? 1 : 0);
        const uint64_t ql = q1 - q0 - (q1 > q0 && in[q1 - 1] == '\r' ? 1 : 0);
        if (sl != ql) k = kBad;
        else s += sl;
      }
      if (k != kNone) {
        first[t] = r;
        kind[t] = k;
        break;
      }
    }
    sum[t] = s;
  });
  uint64_t take = R;
  int problem = kNone;
  for (int t = 0; t < T; ++t)
    if (kind[t] != kNone) {
      take = first[t];
      problem = kind[t];
      break;
    }
  if (take > max_rec) {  // room for max_rec record ends: the rest next call
    take = max_rec;
    problem = kNone;
    res.more = true;
    // the thread holding record `take` summed past it: its bases up to take
    for (int t = 0; t < T; ++t) {
      const uint64_t r0 = R * t / T, r1 = R * (t + 1) / T;
      if (r0 < take && take < r1) {
        int h = 0;
        uint64_t sb = 0;
        for (uint64_t r = r0; r < take; ++r) {
          const uint64_t s0 = L.end(4 * r, h) + 1, s1 = L.end(4 * r + 1, h);
          sb += s1 - s0 - (s1 > s0 && in[s1 - 1] == '\r' ? 1 : 0);
        }
        sum[t] = sb;
      }
    }
  } else if (problem == kNone && eof && n_lines > 4 * R) {
    // lines after the last whole record at the end of the input: blank lines
    // end it (the host reader skips them); else a cut-off or malformed record
    int h = 0;
    bool all_blank = true;
    for (uint64_t l = 4 * R; l < n_lines && all_blank; ++l) {
      const uint64_t a = L.start(l, h), b = L.end(l, h);
      for (uint64_t i = a; i < b; ++i)
        if (in[i] != '\r') {
          all_blank = false;
          break;
        }
    }
    if (!all_blank) {
      const uint64_t a = L.start(4 * R, h), b = L.end(4 * R, h);
      problem = (b == a || in[a] == '\r') ? kBlank : kBad;
    }
  }
  // (3) the taken records' sequences, copied at their prefix offsets
  std::vector<uint64_t> off(T + 1, 0);
  for (int t = 0; t < T; ++t) {
    const uint64_t r0 = R * t / T;
    off[t + 1] = off[t] + (r0 < take ? sum[t] : 0);  // (a thread past `take` adds nothing)
  }
  pool.run([&](int t) {
    if (t >= T) return;
    const uint64_t r0 = R * t / T, r1 = std::min<uint64_t>(R * (t + 1) / T, take);
    int h = 0;
    uint64_t o = off[t];
    for (uint64_t r = r0; r < r1; ++r) {
      const uint64_t l = 4 * r;
      const uint64_t s0 = L.end(l, h) + 1, s1 = L.end(l + 1, h);
      const uint64_t sl = s1 - s0 - (s1 > s0 && in[s1 - 1] == '\r' ? 1 : 0);
      memcpy(bases + o, in + s0, sl);
      o += sl;
      ends[r] = base_off + o;
    }
  });
  int h = 0;
  res.n_rec = take;
  res.n_bases = off[T];
  res.consumed = std::min<uint64_t>(L.start(4 * take, h), len);
  res.stop = problem == kBad;
  res.blank = problem == kBlank;
  return res;
}

}  // namespace nk
