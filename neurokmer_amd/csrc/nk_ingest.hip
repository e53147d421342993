// nk_ingest.hip — GPU FASTA/FASTQ parse of one raw chunk (nk_ingest.h).
//
// FASTA (5 launches, 3 passes over the chunk, each thread one aligned 16-B
// group as the FASTQ passes read them): A per 4-KiB block: the last line
// start and the header lines that start in it; B one block: exclusive
// max-scan of the line starts and sum-scan of the headers (their totals kept
// for D); C per block: the base bytes (now that every byte's line kind is
// known); D one block: scan of the base counts, the new totals and the carried
// line state; E per block: the bases compacted in LDS and stored as one run,
// the record offsets.  (Round 6: byte loads, byte stores scattered by thread
// and D walking the chunk's last block on one thread took ~0.95 ms per 64 MB
// -- D alone 0.49 ms --, the limiter of a FASTA file's path,
// profiles/r06_ab/fasta_overlap/kernel_stats_piecewise.csv.)
//
// FASTQ (the chunk starts at a record boundary, at any address: A and C read
// aligned 16-B groups and mask the bytes outside the chunk): A newline counts;
// B scan; C newline positions; D per record: the four lines' validity and the
// sequence length, the first bad record (atomicMin) and per-1024-record sums
// of the sequence lengths; E one block: the scan of those sums, the first bad
// record's block, the new totals; G per 1024 records: the sequence offsets; F
// one wave per record: copy of the sequence bytes.  (Round 3's E was one block
// walking every record of the chunk, ~200 k per 64 MB, and A/C loaded bytes one
// at a time: the parse took ~1.3 ms per 64 MB, the limiter of a streamed 10 GB
// FASTQ, profiles/r04_s6.)
#include "nk_ingest.h"

namespace nk {

namespace {

constexpr int kIB = 256;              // threads per block
constexpr int kIPer = 16;             // bytes per thread
constexpr int kIS = kIB * kIPer;      // bytes per block
constexpr int kScanT = 1024;          // threads of the single-block scans

struct FaScratch {
  long long *ls;              // [NB] last line start in the block (-1: none)
  unsigned long long *hdr;    // [NB] header lines starting in the block
  unsigned long long *keep;   // [NB] base bytes in the block
  unsigned long long base_out, rec_base;  // resident positions of this chunk
  long long ls_all;           // the chunk's last line start (-1: none)
  unsigned long long hdr_all; // header lines starting in the chunk
};

// exclusive block scans over up to 1024 threads
template <typename T, typename Op>
__device__ T block_scan_excl(T x, T ident, Op op, T *s_w, T *total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  T incl = x;
  for (int o = 1; o < 64; o <<= 1) {
    const T y = __shfl_up(incl, o, 64);
    if (lane >= o) incl = op(incl, y);
  }
  if (lane == 63) s_w[w] = incl;
  __syncthreads();
  T pre = ident, tot = ident;
  for (int i = 0; i < nw; ++i) {
    if (i < w) pre = op(pre, s_w[i]);
    tot = op(tot, s_w[i]);
  }
  __syncthreads();
  *total = tot;
  // exclusive within the wave: shift the inclusive value by one lane
  T ex = __shfl_up(incl, 1, 64);
  if (lane == 0) ex = ident;
  return op(pre, ex);
}
struct OpAdd {
  __device__ unsigned long long operator()(unsigned long long a, unsigned long long b) const {
    return a + b;
  }
};
struct OpMax {
  __device__ long long operator()(long long a, long long b) const { return a > b ? a : b; }
};

// The newline passes read the chunk as 16-B groups aligned in memory (the
// chunk may start anywhere: a FASTQ carry is copied in front of the new data
// on the device): group g covers bytes [16 g - head, 16 g - head + 16) of the
// chunk, head = its start's offset in its 16-B line; bytes outside [0, L) are
// masked.  The buffer holds >= 16 readable bytes past the chunk.
__device__ __forceinline__ void load_group(const uint8_t *R, uint64_t L, uint32_t head, uint64_t g,
                                           uint8_t (&by)[kIPer]) {
  const uint4 v = *reinterpret_cast<const uint4 *>(R - head + 16 * g);
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int j = 0; j < kIPer; ++j) {
    const long long i = (long long)(16 * g + j) - (long long)head;
    by[j] = (i >= 0 && (uint64_t)i < L) ? (uint8_t)(w[j >> 2] >> (8 * (j & 3))) : (uint8_t)0;
  }
}

// ---- FASTA ------------------------------------------------------------------
// thread = 16-B group g = blockIdx.x * kIB + threadIdx.x (bytes 16 g - head ..
// of the chunk); prev = the byte before the group (the lane below's last one,
// or a load for lane 0), for the line-start test of its first byte
struct FaGroup {
  uint8_t by[kIPer];
  long long base;  // the chunk index of by[0]
  uint8_t prev;
};
__device__ __forceinline__ void fa_load(const uint8_t *R, uint64_t L, uint32_t head, FaGroup &x) {
  const uint64_t g = (uint64_t)blockIdx.x * kIB + threadIdx.x;
  x.base = 16 * (long long)g - (long long)head;
  if (x.base < (long long)L) {
    load_group(R, L, head, g, x.by);  // (the buffer holds 16 readable bytes past the chunk)
  } else {
#pragma unroll
    for (int j = 0; j < kIPer; ++j) x.by[j] = 0;
  }
  uint8_t p = (uint8_t)__shfl_up((int)x.by[kIPer - 1], 1, 64);  // (every lane takes part)
  if ((threadIdx.x & 63) == 0) {
    const long long i = x.base - 1;
    p = (i >= 0 && i < (long long)L) ? R[i] : (uint8_t)0;
  }
  x.prev = p;
}
__device__ __forceinline__ bool fa_in(const FaGroup &x, int j, uint64_t L) {
  const long long i = x.base + j;
  return i >= 0 && i < (long long)L;
}
// byte j (inside the chunk) starts a line
__device__ __forceinline__ bool fa_ls(const FaGroup &x, int j, uint32_t als) {
  if (x.base + j == 0) return als != 0;
  return (j ? x.by[j - 1] : x.prev) == '\n';
}

__global__ __launch_bounds__(kIB) void k_fa_a(const uint8_t *__restrict__ R, uint64_t L, uint32_t head,
                                              const IngestState *__restrict__ st, FaScratch f) {
  __shared__ long long s_l[kIB / 64];
  __shared__ unsigned long long s_h[kIB / 64];
  const uint32_t als = st->at_line_start;
  FaGroup x;
  fa_load(R, L, head, x);
  long long last = -1;
  unsigned long long h = 0;
#pragma unroll
  for (int j = 0; j < kIPer; ++j)
    if (fa_in(x, j, L) && fa_ls(x, j, als)) {
      last = x.base + j;
      h += x.by[j] == '>';
    }
  long long tl;
  unsigned long long th;
  block_scan_excl<long long>(last, -1LL, OpMax(), s_l, &tl);
  block_scan_excl<unsigned long long>(h, 0ull, OpAdd(), s_h, &th);
  if (threadIdx.x == 0) {
    f.ls[blockIdx.x] = tl;
    f.hdr[blockIdx.x] = th;
  }
}

// in-place exclusive scans of the per-block arrays (one block of kScanT)
// (up to kScanU entries per thread -- 64 MiB chunks: 16 -- held in registers,
// all loads issued together: the loop of dependent loads took B ~50 us)
constexpr int kScanU = 16;
template <typename T, typename Op>
__device__ void scan_array_excl(T *a, uint64_t n, T ident, Op op, T *s_w, T *total_out) {
  const uint64_t per = (n + kScanT - 1) / kScanT;
  const uint64_t lo = threadIdx.x * per, hi = lo + per < n ? lo + per : n;
  T tot;
  if (per <= (uint64_t)kScanU) {  // (uniform)
    T v[kScanU];
#pragma unroll
    for (int u = 0; u < kScanU; ++u) v[u] = lo + u < hi ? a[lo + u] : ident;
    T loc = ident;
#pragma unroll
    for (int u = 0; u < kScanU; ++u) loc = op(loc, v[u]);
    T run = block_scan_excl<T>(loc, ident, op, s_w, &tot);
#pragma unroll
    for (int u = 0; u < kScanU; ++u)
      if (lo + u < hi) {
        a[lo + u] = run;
        run = op(run, v[u]);
      }
  } else {
    T loc = ident;
    for (uint64_t i = lo; i < hi; ++i) loc = op(loc, a[i]);
    T run = block_scan_excl<T>(loc, ident, op, s_w, &tot);
    for (uint64_t i = lo; i < hi; ++i) {
      const T v = a[i];
      a[i] = run;
      run = op(run, v);
    }
  }
  if (total_out) *total_out = tot;
}

__global__ __launch_bounds__(kScanT) void k_fa_b(uint64_t NB, FaScratch f, FaScratch *__restrict__ fs) {
  __shared__ long long s_l[kScanT / 64];
  __shared__ unsigned long long s_h[kScanT / 64];
  long long tl;
  unsigned long long th;
  scan_array_excl<long long>(f.ls, NB, -1LL, OpMax(), s_l, &tl);
  scan_array_excl<unsigned long long>(f.hdr, NB, 0ull, OpAdd(), s_h, &th);
  if (threadIdx.x == 0) {
    fs->ls_all = tl;
    fs->hdr_all = th;
  }
}

// header kind of the line holding byte i, given the line start at or before
// it (ls >= 0) or the carried state
__device__ __forceinline__ bool line_hdr(const uint8_t *R, long long ls, const IngestState &st) {
  return ls >= 0 ? R[ls] == '>' : st.line_is_hdr != 0;
}

// the line start in effect before the group's first byte: the block's carry
// folded with the block's threads below
__device__ __forceinline__ long long fa_carry_ls(const FaGroup &x, uint64_t L, uint32_t als,
                                                 long long blk_carry, long long *s_l) {
  long long last = -1;
#pragma unroll
  for (int j = 0; j < kIPer; ++j)
    if (fa_in(x, j, L) && fa_ls(x, j, als)) last = x.base + j;
  long long tot;
  const long long ex = block_scan_excl<long long>(last, -1LL, OpMax(), s_l, &tot);
  return ex > blk_carry ? ex : blk_carry;
}

__global__ __launch_bounds__(kIB) void k_fa_c(const uint8_t *__restrict__ R, uint64_t L, uint32_t head,
                                              const IngestState *__restrict__ st, FaScratch f) {
  __shared__ long long s_l[kIB / 64];
  __shared__ unsigned long long s_k[kIB / 64];
  const IngestState S = *st;
  FaGroup x;
  fa_load(R, L, head, x);
  const long long ls = fa_carry_ls(x, L, S.at_line_start, f.ls[blockIdx.x], s_l);
  unsigned long long keep = 0;
  bool hdr = line_hdr(R, ls, S);
#pragma unroll
  for (int j = 0; j < kIPer; ++j) {
    if (!fa_in(x, j, L)) continue;
    const uint8_t c = x.by[j];
    if (fa_ls(x, j, S.at_line_start)) hdr = c == '>';
    keep += !hdr && c != '\n' && c != '\r';
  }
  unsigned long long tk;
  block_scan_excl<unsigned long long>(keep, 0ull, OpAdd(), s_k, &tk);
  if (threadIdx.x == 0) f.keep[blockIdx.x] = tk;
}

__global__ __launch_bounds__(kScanT) void k_fa_d(const uint8_t *__restrict__ R, uint64_t L,
                                                 uint64_t NB, IngestState *__restrict__ st,
                                                 FaScratch *__restrict__ fs, uint64_t *offsets) {
  __shared__ unsigned long long s_k[kScanT / 64];
  __shared__ unsigned long long s_tot;
  unsigned long long tk;
  scan_array_excl<unsigned long long>(fs->keep, NB, 0ull, OpAdd(), s_k, &tk);
  if (threadIdx.x == 0) s_tot = tk;
  __syncthreads();
  if (threadIdx.x != 0) return;
  IngestState S = *st;
  const unsigned long long nh = fs->hdr_all;  // headers in this chunk (k_fa_b's totals)
  const long long last_ls = fs->ls_all;      // the chunk's last line start
  const bool ends_nl = L > 0 && R[L - 1] == '\n';
  uint32_t hdr_after = S.line_is_hdr;
  if (!ends_nl && L > 0) hdr_after = line_hdr(R, last_ls, S) ? 1u : 0u;
  fs->base_out = S.data_end;
  fs->rec_base = S.n_rec;
  S.data_end += s_tot;
  S.n_rec += nh;
  S.at_line_start = L == 0 ? S.at_line_start : (ends_nl ? 1u : 0u);
  S.line_is_hdr = ends_nl ? 0u : hdr_after;
  *st = S;
  offsets[S.n_rec] = S.data_end;  // provisional end of the last record
}

__global__ __launch_bounds__(kIB) void k_fa_e(const uint8_t *__restrict__ R, uint64_t L, uint32_t head,
                                              const IngestState *__restrict__ st_before,
                                              const FaScratch *__restrict__ fs, FaScratch f,
                                              uint8_t *__restrict__ bases,
                                              uint64_t *__restrict__ offsets) {
  __shared__ long long s_l[kIB / 64];
  __shared__ unsigned long long s_k[kIB / 64], s_h[kIB / 64];
  __shared__ uint8_t s_out[kIS];  // the block's bases, compacted
  const IngestState S = *st_before;  // the state the chunk started from
  FaGroup x;
  fa_load(R, L, head, x);
  const long long ls = fa_carry_ls(x, L, S.at_line_start, f.ls[blockIdx.x], s_l);
  unsigned long long keep = 0, h = 0;
  bool hdr = line_hdr(R, ls, S);
#pragma unroll
  for (int j = 0; j < kIPer; ++j) {
    if (!fa_in(x, j, L)) continue;
    const uint8_t c = x.by[j];
    if (fa_ls(x, j, S.at_line_start)) {
      hdr = c == '>';
      h += hdr;
    }
    keep += !hdr && c != '\n' && c != '\r';
  }
  unsigned long long tk, th;
  unsigned long long kp = block_scan_excl<unsigned long long>(keep, 0ull, OpAdd(), s_k, &tk);
  unsigned long long hp = block_scan_excl<unsigned long long>(h, 0ull, OpAdd(), s_h, &th);
  const unsigned long long blk_out = fs->base_out + f.keep[blockIdx.x];  // the block's first base
  hp += fs->rec_base + f.hdr[blockIdx.x];
  hdr = line_hdr(R, ls, S);
#pragma unroll
  for (int j = 0; j < kIPer; ++j) {
    if (!fa_in(x, j, L)) continue;
    const uint8_t c = x.by[j];
    if (fa_ls(x, j, S.at_line_start)) {
      hdr = c == '>';
      if (hdr) offsets[hp++] = blk_out + kp;  // a record starts: bases before it
    }
    if (!hdr && c != '\n' && c != '\r') s_out[kp++] = c;
  }
  __syncthreads();
  // one run of consecutive bytes per block: consecutive lanes, consecutive bytes
  // (dword stores of the aligned middle measured equal, profiles/r06_ab/fasta_parse)
  for (uint32_t o = threadIdx.x; o < (uint32_t)tk; o += kIB) bases[blk_out + o] = s_out[o];
}

// ---- FASTQ ------------------------------------------------------------------
struct FqScratch {
  unsigned long long *nl;    // [NB] newlines per block -> exclusive prefix
  uint32_t *nlpos;           // [newlines] positions
  uint32_t *seqlen;          // [records]
  uint8_t *flag;             // [records] 0 ok, 1 bad, 2 blank header
  unsigned long long *pos;   // [records] output offset of the sequence
  unsigned long long *bsum;  // [record blocks] sum of seqlen -> exclusive prefix
  unsigned long long out_base, rec_base, n_good;
  unsigned long long first_bad;  // min index of a flagged record (~0: none)
};
constexpr int kRecBlock = 1024;  // records per block of the D/G passes

__global__ __launch_bounds__(kIB) void k_fq_a(const uint8_t *__restrict__ R, uint64_t L,
                                              uint32_t head, FqScratch f) {
  __shared__ unsigned long long s_n[kIB / 64];
  const uint64_t g = (uint64_t)blockIdx.x * kIB + threadIdx.x;
  unsigned long long n = 0;
  if (16 * g < L + head) {
    uint8_t by[kIPer];
    load_group(R, L, head, g, by);
#pragma unroll
    for (int j = 0; j < kIPer; ++j) n += by[j] == '\n';
  }
  unsigned long long tn;
  block_scan_excl<unsigned long long>(n, 0ull, OpAdd(), s_n, &tn);
  if (threadIdx.x == 0) f.nl[blockIdx.x] = tn;
}

__global__ __launch_bounds__(kScanT) void k_fq_b(uint64_t NB, FqScratch f,
                                                 unsigned long long *total) {
  __shared__ unsigned long long s_n[kScanT / 64];
  unsigned long long tn;
  scan_array_excl<unsigned long long>(f.nl, NB, 0ull, OpAdd(), s_n, &tn);
  if (threadIdx.x == 0) *total = tn;
}

__global__ __launch_bounds__(kIB) void k_fq_c(const uint8_t *__restrict__ R, uint64_t L,
                                              uint32_t head, FqScratch f) {
  __shared__ unsigned long long s_n[kIB / 64];
  const uint64_t g = (uint64_t)blockIdx.x * kIB + threadIdx.x;
  uint8_t by[kIPer];
  if (16 * g < L + head) {
    load_group(R, L, head, g, by);
  } else {
#pragma unroll
    for (int j = 0; j < kIPer; ++j) by[j] = 0;
  }
  unsigned long long n = 0;
#pragma unroll
  for (int j = 0; j < kIPer; ++j) n += by[j] == '\n';
  unsigned long long tn;
  unsigned long long at = block_scan_excl<unsigned long long>(n, 0ull, OpAdd(), s_n, &tn);
  at += f.nl[blockIdx.x];
#pragma unroll
  for (int j = 0; j < kIPer; ++j)
    if (by[j] == '\n') f.nlpos[at++] = (uint32_t)(16 * g + j - head);
}

// line l of the chunk: [start, end) without its '\n'
__device__ __forceinline__ void fq_line(const FqScratch &f, uint64_t l, uint64_t nl_total,
                                        uint64_t L, uint64_t *s, uint64_t *e) {
  *s = l == 0 ? 0 : (uint64_t)f.nlpos[l - 1] + 1;
  *e = l < nl_total ? (uint64_t)f.nlpos[l] : L;
}

// one thread per record: validity, sequence length; per block of kRecBlock
// records the sum of the lengths (bsum) and the first flagged record
__global__ __launch_bounds__(kRecBlock) void k_fq_d(const uint8_t *__restrict__ R, uint64_t L,
                                                    uint64_t n_rec,
                                                    const unsigned long long *__restrict__ nl_total_p,
                                                    FqScratch *__restrict__ fs, FqScratch f) {
  __shared__ unsigned long long s_w[kRecBlock / 64];
  const uint64_t nl_total = *nl_total_p;
  const uint64_t r = (uint64_t)blockIdx.x * kRecBlock + threadIdx.x;
  uint32_t len = 0;
  if (r < n_rec) {
    uint64_t s[4], e[4];
    for (int q = 0; q < 4; ++q) {
      fq_line(f, 4 * r + q, nl_total, L, &s[q], &e[q]);
      if (e[q] > s[q] && R[e[q] - 1] == '\r') --e[q];  // read_line strips one trailing '\r'
    }
    uint8_t fl = 0;
    if (e[0] == s[0] || R[s[0]] == '\r') fl = 2;            // blank line: the host skips it
    else if (R[s[0]] != '@') fl = 1;                       // not a header
    else if (e[2] == s[2] || R[s[2]] != '+') fl = 1;       // '+' line missing or empty
    else if (e[3] - s[3] != e[1] - s[1]) fl = 1;           // quality length != sequence
    f.flag[r] = fl;
    len = (uint32_t)(e[1] - s[1]);
    f.seqlen[r] = len;
    if (fl) atomicMin(&fs->first_bad, (unsigned long long)r);
  }
  unsigned long long tot;
  block_scan_excl<unsigned long long>((unsigned long long)len, 0ull, OpAdd(), s_w, &tot);
  if (threadIdx.x == 0) f.bsum[blockIdx.x] = tot;
}

// one block: the first bad record fixes the good prefix; the record blocks'
// length sums scanned; the totals of the chunk's good records
__global__ __launch_bounds__(kScanT) void k_fq_e(uint64_t n_rec, uint64_t L,
                                                 const unsigned long long *__restrict__ nl_total_p,
                                                 IngestState *__restrict__ st,
                                                 FqScratch *__restrict__ fs,
                                                 uint64_t *__restrict__ offsets) {
  __shared__ unsigned long long s_w[kScanT / 64];
  const FqScratch f = *fs;
  const uint64_t ng = f.first_bad < n_rec ? f.first_bad : n_rec;
  const uint64_t nrb = (n_rec + kRecBlock - 1) / kRecBlock;
  unsigned long long tn;
  scan_array_excl<unsigned long long>(f.bsum, nrb, 0ull, OpAdd(), s_w, &tn);
  // the good records' total: the blocks before ng's, plus ng's block up to ng
  const uint64_t gb = ng / kRecBlock;
  unsigned long long part = 0;
  for (uint64_t r = gb * kRecBlock + threadIdx.x; r < ng; r += kScanT) part += f.seqlen[r];
  unsigned long long ptot;
  block_scan_excl<unsigned long long>(part, 0ull, OpAdd(), s_w, &ptot);
  if (threadIdx.x != 0) return;
  const unsigned long long tot = (gb < nrb ? f.bsum[gb] : tn) + ptot;
  IngestState S = *st;
  const uint64_t nl_total = *nl_total_p;
  fs->out_base = S.data_end;
  fs->rec_base = S.n_rec;
  fs->n_good = ng;
  if (ng < n_rec) {
    if (f.flag[ng] == 2) S.blank = 1;  // fall back to the host reader
    else S.stop = 1;                   // truncated stream: drop the rest
  }
  S.data_end += tot;
  S.n_rec += ng;
  // bytes used by the complete records (4 lines each, '\n'-terminated)
  const uint64_t last_nl = 4 * ng;
  S.consumed = ng == 0 ? 0 : (last_nl <= nl_total ? (uint64_t)f.nlpos[last_nl - 1] + 1 : L);
  *st = S;
  offsets[S.n_rec] = S.data_end;
}

// per block of kRecBlock records: the good records' output offsets
__global__ __launch_bounds__(kRecBlock) void k_fq_g(uint64_t n_rec, const FqScratch *__restrict__ fs,
                                                    uint64_t *__restrict__ offsets) {
  __shared__ unsigned long long s_w[kRecBlock / 64];
  const FqScratch f = *fs;
  const uint64_t r = (uint64_t)blockIdx.x * kRecBlock + threadIdx.x;
  const uint64_t ng = f.n_good;
  if ((uint64_t)blockIdx.x * kRecBlock >= ng) return;  // uniform
  const unsigned long long len = r < ng ? f.seqlen[r] : 0ull;
  unsigned long long tot;
  const unsigned long long at = block_scan_excl<unsigned long long>(len, 0ull, OpAdd(), s_w, &tot) +
                                f.bsum[blockIdx.x] + f.out_base;
  if (r < ng) {
    f.pos[r] = at;
    offsets[f.rec_base + r] = at;
  }
}

// one wave per record: the sequence bytes to their resident offset
__global__ void k_fq_f(const uint8_t *__restrict__ R, uint64_t L,
                       const unsigned long long *__restrict__ nl_total_p,
                       const FqScratch *__restrict__ fs, uint8_t *__restrict__ bases) {
  const FqScratch f = *fs;
  const uint64_t nl_total = *nl_total_p;
  const int lane = threadIdx.x & 63;
  for (uint64_t r = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; r < f.n_good;
       r += ((uint64_t)gridDim.x * blockDim.x) >> 6) {
    uint64_t s, e;
    fq_line(f, 4 * r + 1, nl_total, L, &s, &e);
    const uint32_t n = f.seqlen[r];
    const uint64_t dst = f.pos[r];
    for (uint32_t i = lane; i < n; i += 64) bases[dst + i] = R[s + i];
  }
}

unsigned blocks_for(uint64_t L) { return (unsigned)((L + kIS - 1) / kIS); }

}  // namespace

size_t ingest_scratch_bytes(size_t chunk_cap) {
  const size_t NB = (chunk_cap + 16 + kIS - 1) / kIS + 1;
  const size_t fa = NB * (8 + 8 + 8) + sizeof(FaScratch);
  const size_t recs = chunk_cap / 4 + 2;
  const size_t fq = NB * 8 + (chunk_cap + 1) * 4 + recs * (4 + 1 + 8) + (recs / kRecBlock + 2) * 8 +
                    sizeof(FqScratch) + 64 + 64;
  return (fa > fq ? fa : fq) + 1024;
}

// scratch layout: [struct][arrays...]
hipError_t ingest_fasta(const uint8_t *raw, size_t len, bool eof, const IngestBufs &bufs,
                        IngestState *st, hipStream_t s) {
  (void)eof;
  const uint32_t head = (uint32_t)((uintptr_t)raw & 15);
  const uint64_t NB = blocks_for(len + head ? len + head : 1);
  uint8_t *p = (uint8_t *)bufs.scratch;
  FaScratch *fs = (FaScratch *)p;
  p += 256;
  FaScratch f{};
  f.ls = (long long *)p;
  p += NB * 8;
  f.hdr = (unsigned long long *)p;
  p += NB * 8;
  f.keep = (unsigned long long *)p;
  // the state the chunk starts from is needed by pass E after D updates it
  IngestState *before = (IngestState *)(p + NB * 8);
  hipError_t e = hipMemcpyAsync(fs, &f, sizeof f, hipMemcpyHostToDevice, s);
  if (e != hipSuccess) return e;
  e = hipMemcpyAsync(before, st, sizeof(IngestState), hipMemcpyDeviceToDevice, s);
  if (e != hipSuccess) return e;
  if (!len) return hipSuccess;
  hipLaunchKernelGGL(k_fa_a, dim3((unsigned)NB), dim3(kIB), 0, s, raw, (uint64_t)len, head, st, f);
  hipLaunchKernelGGL(k_fa_b, dim3(1), dim3(kScanT), 0, s, NB, f, fs);
  hipLaunchKernelGGL(k_fa_c, dim3((unsigned)NB), dim3(kIB), 0, s, raw, (uint64_t)len, head, st, f);
  hipLaunchKernelGGL(k_fa_d, dim3(1), dim3(kScanT), 0, s, raw, (uint64_t)len, NB, st, fs,
                     bufs.offsets);
  hipLaunchKernelGGL(k_fa_e, dim3((unsigned)NB), dim3(kIB), 0, s, raw, (uint64_t)len, head, before, fs,
                     f, bufs.bases, bufs.offsets);
  return hipGetLastError();
}

hipError_t ingest_fastq(const uint8_t *raw, size_t len, bool eof, const IngestBufs &bufs,
                        IngestState *st, hipStream_t s) {
  const uint32_t head = (uint32_t)((uintptr_t)raw & 15);
  const uint64_t NB = blocks_for(len + head ? len + head : 1);
  uint8_t *p = (uint8_t *)bufs.scratch;
  FqScratch *fs = (FqScratch *)p;
  p += 256;
  unsigned long long *nl_total = (unsigned long long *)p;
  p += 64;
  FqScratch f{};
  f.nl = (unsigned long long *)p;
  p += NB * 8;
  f.nlpos = (uint32_t *)p;
  p += (len + 1) * 4;
  p = (uint8_t *)(((uintptr_t)p + 15) & ~(uintptr_t)15);
  const uint64_t max_rec = len / 4 + 2;
  f.pos = (unsigned long long *)p;
  p += max_rec * 8;
  f.bsum = (unsigned long long *)p;
  p += (max_rec / kRecBlock + 2) * 8;
  f.seqlen = (uint32_t *)p;
  p += max_rec * 4;
  f.flag = (uint8_t *)p;
  f.first_bad = ~0ull;
  hipError_t e = hipMemcpyAsync(fs, &f, sizeof f, hipMemcpyHostToDevice, s);
  if (e != hipSuccess) return e;
  // newline count first: the number of candidate records follows from it
  hipLaunchKernelGGL(k_fq_a, dim3((unsigned)NB), dim3(kIB), 0, s, raw, (uint64_t)len, head, f);
  hipLaunchKernelGGL(k_fq_b, dim3(1), dim3(kScanT), 0, s, NB, f, nl_total);
  unsigned long long nl = 0;
  e = hipMemcpyAsync(&nl, nl_total, 8, hipMemcpyDeviceToHost, s);
  if (e != hipSuccess) return e;
  e = hipStreamSynchronize(s);
  if (e != hipSuccess) return e;
  // lines: '\n'-terminated ones, plus an unterminated last line at the end of input
  uint64_t lines = nl;
  if (eof && len) {
    uint8_t last = 0;
    e = hipMemcpy(&last, raw + len - 1, 1, hipMemcpyDeviceToHost);
    if (e != hipSuccess) return e;
    if (last != '\n') ++lines;
  }
  const uint64_t n_rec = lines / 4;  // complete 4-line records
  hipLaunchKernelGGL(k_fq_c, dim3((unsigned)NB), dim3(kIB), 0, s, raw, (uint64_t)len, head, f);
  const uint64_t nrb = (n_rec + kRecBlock - 1) / kRecBlock;
  if (n_rec)
    hipLaunchKernelGGL(k_fq_d, dim3((unsigned)nrb), dim3(kRecBlock), 0, s, raw, (uint64_t)len, n_rec,
                       nl_total, fs, f);
  hipLaunchKernelGGL(k_fq_e, dim3(1), dim3(kScanT), 0, s, n_rec, (uint64_t)len, nl_total, st, fs,
                     bufs.offsets);
  if (n_rec) {
    hipLaunchKernelGGL(k_fq_g, dim3((unsigned)nrb), dim3(kRecBlock), 0, s, n_rec, fs, bufs.offsets);
    const uint64_t waves = n_rec < 65536 ? n_rec : 65536;
    hipLaunchKernelGGL(k_fq_f, dim3((unsigned)((waves * 64 + 255) / 256)), dim3(256), 0, s, raw,
                       (uint64_t)len, nl_total, fs, bufs.bases);
  }
  return hipGetLastError();
}

}  // namespace nk
