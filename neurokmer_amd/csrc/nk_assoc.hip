// nk_assoc.hip — the reference's associative memory on the
// device: WillshawNetwork (src/associative.rs:12-62) with a bit-packed weight
// matrix, and KmerAssociativeMemory (:64-139) whose k-mer patterns come from
// BLAKE3 (the blake3 crate's hash of the key's 8 LE bytes) computed on the
// device.
//
// Layout: weights W[i] = row i as ceil(n/32) u32 words (n = pattern size;
// 128 KiB at n = 1024).  store(pattern) ORs bit j into row i for every pair
// (i, j) of the pattern's set bits (one atomicOr per pair: patterns are
// sparse, ~1 % of n).  recall runs synchronous steps state' = (W state > 0)
// as "row i intersects state" on packed words until the state repeats.
// find_similar scores every distinct stored k-mer by the Hamming distance of
// its pattern to the recalled state from the pattern's (<= n/100) set bits.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <unordered_set>
#include <vector>

#include "neurokmer.h"

int nk_fail_msg(int code, const char *msg);  // nk_counter.cpp: nk_last_error() text

namespace nk {
namespace {

// ---- BLAKE3 of one 8-byte input (one chunk, one block, the root) -------------
__device__ __constant__ uint32_t kB3IV[8] = {0x6A09E667u, 0xBB67AE85u, 0x3C6EF372u, 0xA54FF53Au,
                                             0x510E527Fu, 0x9B05688Cu, 0x1F83D9ABu, 0x5BE0CD19u};

__device__ __forceinline__ uint32_t rotr32(uint32_t x, int r) {
  return __builtin_amdgcn_alignbit(x, x, r);
}

#define NK_B3G(a, b, c, d, mx, my)   \
  do {                               \
    v[a] = v[a] + v[b] + (mx);       \
    v[d] = rotr32(v[d] ^ v[a], 16);  \
    v[c] = v[c] + v[d];              \
    v[b] = rotr32(v[b] ^ v[c], 12);  \
    v[a] = v[a] + v[b] + (my);       \
    v[d] = rotr32(v[d] ^ v[a], 8);   \
    v[c] = v[c] + v[d];              \
    v[b] = rotr32(v[b] ^ v[c], 7);   \
  } while (0)

// digest words 0..7 (little-endian bytes) of BLAKE3(8 LE bytes of key)
__device__ void blake3_u64(uint64_t key, uint32_t out[8]) {
  uint32_t m[16] = {(uint32_t)key, (uint32_t)(key >> 32), 0, 0, 0, 0, 0, 0,
                    0, 0, 0, 0, 0, 0, 0, 0};
  uint32_t v[16];
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = kB3IV[i];
#pragma unroll
  for (int i = 0; i < 4; ++i) v[8 + i] = kB3IV[i];
  v[12] = 0;   // chunk counter
  v[13] = 0;
  v[14] = 8;   // block length
  v[15] = 11;  // CHUNK_START | CHUNK_END | ROOT
  constexpr int P[16] = {2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8};
#pragma unroll
  for (int r = 0; r < 7; ++r) {
    NK_B3G(0, 4, 8, 12, m[0], m[1]);
    NK_B3G(1, 5, 9, 13, m[2], m[3]);
    NK_B3G(2, 6, 10, 14, m[4], m[5]);
    NK_B3G(3, 7, 11, 15, m[6], m[7]);
    NK_B3G(0, 5, 10, 15, m[8], m[9]);
    NK_B3G(1, 6, 11, 12, m[10], m[11]);
    NK_B3G(2, 7, 8, 13, m[12], m[13]);
    NK_B3G(3, 4, 9, 14, m[14], m[15]);
    uint32_t t[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) t[i] = m[P[i]];
#pragma unroll
    for (int i = 0; i < 16; ++i) m[i] = t[i];
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) out[i] = v[i] ^ v[i + 8];
}

constexpr int kMaxBits = 32;  // n / 100 set bits at most here: n <= 3299 is
                              // what KmerAssociativeMemory builds (n <= 1024)

// the set bits of pattern(kmer) (src/associative.rs:84-96): byte i % 32 of
// the digest, modulo n, for i < n / 100; duplicates removed.  -> count
__device__ int kmer_bits(uint64_t kmer, uint32_t n, uint32_t *bits) {
  uint32_t d[8];
  blake3_u64(kmer, d);
  const uint32_t nb = n / 100;
  int m = 0;
  for (uint32_t i = 0; i < nb && i < (uint32_t)kMaxBits; ++i) {
    const uint32_t byte = (d[(i % 32) >> 2] >> (8 * (i & 3))) & 0xFFu;
    const uint32_t b = byte % n;
    bool dup = false;
    for (int j = 0; j < m; ++j) dup |= bits[j] == b;
    if (!dup) bits[m++] = b;
  }
  return m;
}

// store: W[a] |= bit b for every pair of the listed bits (grid-stride: a dense
// pattern of n = 2^20 bits has 2^40 pairs, more than a 32-bit grid holds)
__global__ void k_ws_store_bits(uint32_t *__restrict__ W, uint32_t words,
                                const uint32_t *__restrict__ idx, uint32_t m) {
  const uint64_t pairs = (uint64_t)m * m;
  for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < pairs;
       t += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t a = idx[t / m], b = idx[t % m];
    atomicOr(&W[(uint64_t)a * words + (b >> 5)], 1u << (b & 31));
  }
}

// store_kmer of a batch: each thread one k-mer's pattern pairs
__global__ void k_assoc_store(uint32_t *__restrict__ W, uint32_t words, uint32_t n,
                              const uint64_t *__restrict__ kmers, uint64_t count) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= count) return;
  uint32_t bits[kMaxBits];
  const int m = kmer_bits(kmers[t], n, bits);
  for (int i = 0; i < m; ++i)
    for (int j = 0; j < m; ++j)
      atomicOr(&W[(uint64_t)bits[i] * words + (bits[j] >> 5)], 1u << (bits[j] & 31));
}

// one recall step: out bit i = row i intersects `in`; *changed |= out != in.
// A wave per row: lanes stride over the row's words, a ballot combines.
__global__ void k_ws_recall_step(const uint32_t *__restrict__ W, uint32_t words, uint32_t n,
                                 const uint32_t *__restrict__ in, uint32_t *__restrict__ out,
                                 uint32_t *__restrict__ changed) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t row = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (row >= n) return;
  const uint32_t *r = W + row * words;
  uint32_t hit = 0;
  for (uint32_t w = lane; w < words; w += 64) hit |= r[w] & in[w];
  const bool on = __ballot(hit != 0) != 0;
  if (lane == 0) {
    const bool was = (in[row >> 5] >> (row & 31)) & 1u;
    if (on) atomicOr(&out[row >> 5], 1u << (row & 31));
    if (on != was) atomicOr(changed, 1u);
  }
}

__global__ void k_assoc_query_bits(uint64_t kmer, uint32_t n, uint32_t *__restrict__ state) {
  if (threadIdx.x != 0) return;
  uint32_t bits[kMaxBits];
  const int m = kmer_bits(kmer, n, bits);
  for (int i = 0; i < m; ++i) state[bits[i] >> 5] |= 1u << (bits[i] & 31);
}

// Hamming distance of each stored k-mer's pattern to the recalled state:
// |R| + |P| - 2 |R & P| from P's set bits; within max_d -> (index, d) out
__global__ void k_assoc_distance(const uint64_t *__restrict__ kmers, uint64_t count, uint32_t n,
                                 const uint32_t *__restrict__ rec, uint32_t pop_rec,
                                 uint64_t max_d, uint64_t *__restrict__ out,
                                 unsigned long long *__restrict__ n_out) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= count) return;
  uint32_t bits[kMaxBits];
  const int m = kmer_bits(kmers[t], n, bits);
  uint32_t both = 0;
  for (int i = 0; i < m; ++i) both += (rec[bits[i] >> 5] >> (bits[i] & 31)) & 1u;
  const uint64_t d = (uint64_t)pop_rec + (uint64_t)m - 2ull * both;
  if (d <= max_d) {
    const unsigned long long at = atomicAdd(n_out, 1ull);
    out[2 * at] = t;
    out[2 * at + 1] = d;
  }
}

unsigned grid_of(uint64_t threads, unsigned block) {
  return (unsigned)std::max<uint64_t>(1, (threads + block - 1) / block);
}

}  // namespace
}  // namespace nk

using namespace nk;

#define AS_CHK(expr)                                                              \
  do {                                                                            \
    hipError_t e_ = (expr);                                                       \
    if (e_ != hipSuccess) return nk_fail_msg(NK_E_DEVICE, hipGetErrorString(e_)); \
  } while (0)

struct nk_willshaw {
  int device = 0;
  uint32_t n = 0, words = 0;
  uint32_t *W = nullptr;         // n x words
  uint32_t *state = nullptr;     // 2 x words (double buffer)
  uint32_t *flag = nullptr;      // changed
  uint32_t *idx = nullptr;       // store: set bits of one pattern (n entries)
  hipStream_t s = nullptr;
  uint64_t stored = 0;
};

namespace {

int ws_init(nk_willshaw *w, size_t n, int device) {
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev)
    return nk_fail_msg(NK_E_NO_DEVICE, "no such HIP device (this library has no CPU fallback)");
  if (n > (1u << 20)) return nk_fail_msg(NK_E_INVALID, "pattern size above 2^20");
  w->device = device;
  w->n = (uint32_t)n;
  w->words = (uint32_t)((n + 31) / 32);
  AS_CHK(hipSetDevice(device));
  AS_CHK(hipStreamCreateWithFlags(&w->s, hipStreamNonBlocking));
  const size_t wb = std::max<size_t>((size_t)w->n * w->words, 1) * 4;
  AS_CHK(hipMalloc((void **)&w->W, wb));
  AS_CHK(hipMalloc((void **)&w->state, std::max<size_t>(2 * w->words, 1) * 4));
  AS_CHK(hipMalloc((void **)&w->flag, 4));
  AS_CHK(hipMalloc((void **)&w->idx, std::max<size_t>(n, 1) * 4));
  AS_CHK(hipMemsetAsync(w->W, 0, wb, w->s));
  AS_CHK(hipStreamSynchronize(w->s));
  return NK_OK;
}

void ws_release(nk_willshaw *w) {
  if (w->s) (void)hipStreamSynchronize(w->s);
  if (w->W) (void)hipFree(w->W);
  if (w->state) (void)hipFree(w->state);
  if (w->flag) (void)hipFree(w->flag);
  if (w->idx) (void)hipFree(w->idx);
  if (w->s) (void)hipStreamDestroy(w->s);
}

// steps of synchronous recall from the state in buffer 0; -> the buffer
// holding the final state (one flag readback per step: it stops early when
// the state repeats, src/associative.rs:58)
int ws_recall_dev(nk_willshaw *w, size_t steps, uint32_t **final_state) {
  uint32_t *cur = w->state, *nxt = w->state + w->words;
  for (size_t st = 0; st < steps && w->n; ++st) {
    AS_CHK(hipMemsetAsync(nxt, 0, w->words * 4, w->s));
    AS_CHK(hipMemsetAsync(w->flag, 0, 4, w->s));
    hipLaunchKernelGGL(k_ws_recall_step, dim3(grid_of((uint64_t)w->n * 64, 256)), dim3(256), 0,
                       w->s, w->W, w->words, w->n, cur, nxt, w->flag);
    AS_CHK(hipGetLastError());
    uint32_t changed = 0;
    AS_CHK(hipMemcpyAsync(&changed, w->flag, 4, hipMemcpyDeviceToHost, w->s));
    AS_CHK(hipStreamSynchronize(w->s));
    if (!changed) break;
    std::swap(cur, nxt);
  }
  *final_state = cur;
  return NK_OK;
}

}  // namespace

struct nk_assoc {
  nk_willshaw net;
  std::unordered_set<uint64_t> seen;  // distinct stored k-mers (pattern_to_kmers members)
  uint64_t *kmers = nullptr;          // device copy of them, in store order
  size_t nk = 0, cap = 0;
  uint64_t *batch = nullptr;          // store batch staging
  size_t batch_cap = 0;
  uint64_t *res = nullptr;            // find_similar: (index, distance) pairs
  unsigned long long *n_res = nullptr;
};

extern "C" {

nk_willshaw *nk_willshaw_new(size_t pattern_size, int device) {
  nk_willshaw *w = new nk_willshaw();
  if (ws_init(w, pattern_size, device)) {
    ws_release(w);
    delete w;
    return nullptr;
  }
  return w;
}

void nk_willshaw_free(nk_willshaw *w) {
  if (!w) return;
  (void)hipSetDevice(w->device);
  ws_release(w);
  delete w;
}

int nk_willshaw_store(nk_willshaw *w, const uint8_t *pattern, size_t len) {
  if (!w || (len && !pattern)) return nk_fail_msg(NK_E_INVALID, "null argument");
  if (len != w->n) return nk_fail_msg(NK_E_INVALID, "Pattern size mismatch");
  std::vector<uint32_t> on;
  for (size_t i = 0; i < len; ++i)
    if (pattern[i] > 0) on.push_back((uint32_t)i);
  AS_CHK(hipSetDevice(w->device));
  if (!on.empty()) {
    AS_CHK(hipMemcpyAsync(w->idx, on.data(), on.size() * 4, hipMemcpyHostToDevice, w->s));
    const uint64_t pairs = (uint64_t)on.size() * on.size();
    const unsigned grid = (unsigned)std::min<uint64_t>((pairs + 255) / 256, 1u << 20);
    hipLaunchKernelGGL(k_ws_store_bits, dim3(grid), dim3(256), 0, w->s, w->W,
                       w->words, w->idx, (uint32_t)on.size());
    AS_CHK(hipGetLastError());
    AS_CHK(hipStreamSynchronize(w->s));  // `on` is host memory the copy reads
  }
  w->stored++;
  return NK_OK;
}

int nk_willshaw_recall(nk_willshaw *w, const uint8_t *noisy, size_t len, size_t steps,
                       uint8_t *out) {
  if (!w || (len && (!noisy || !out))) return nk_fail_msg(NK_E_INVALID, "null argument");
  if (len != w->n) return nk_fail_msg(NK_E_INVALID, "Noisy pattern size mismatch");
  std::vector<uint32_t> st(std::max<uint32_t>(w->words, 1), 0);
  for (size_t i = 0; i < len; ++i)
    if (noisy[i] > 0) st[i >> 5] |= 1u << (i & 31);
  AS_CHK(hipSetDevice(w->device));
  if (w->words) AS_CHK(hipMemcpyAsync(w->state, st.data(), w->words * 4, hipMemcpyHostToDevice, w->s));
  uint32_t *fin = nullptr;
  int rc = ws_recall_dev(w, steps, &fin);
  if (rc) return rc;
  if (w->words) AS_CHK(hipMemcpyAsync(st.data(), fin, w->words * 4, hipMemcpyDeviceToHost, w->s));
  AS_CHK(hipStreamSynchronize(w->s));
  for (size_t i = 0; i < len; ++i) out[i] = ((st[i >> 5] >> (i & 31)) & 1u) ? 255 : 0;
  return NK_OK;
}

uint64_t nk_willshaw_stored(const nk_willshaw *w) { return w ? w->stored : 0; }

nk_assoc *nk_assoc_new(size_t k, int device) {
  if (k == 0) {
    nk_fail_msg(NK_E_INVALID, "k must be >= 1");
    return nullptr;
  }
  nk_assoc *a = new nk_assoc();
  const size_t n = k <= 10 ? ((size_t)1 << k) : 1024;  // src/associative.rs:73
  if (ws_init(&a->net, n, device) ||
      hipMalloc((void **)&a->n_res, sizeof(unsigned long long)) != hipSuccess) {
    ws_release(&a->net);
    delete a;
    return nullptr;
  }
  return a;
}

void nk_assoc_free(nk_assoc *a) {
  if (!a) return;
  (void)hipSetDevice(a->net.device);
  ws_release(&a->net);
  if (a->kmers) (void)hipFree(a->kmers);
  if (a->batch) (void)hipFree(a->batch);
  if (a->res) (void)hipFree(a->res);
  if (a->n_res) (void)hipFree(a->n_res);
  delete a;
}

size_t nk_assoc_pattern_size(const nk_assoc *a) { return a ? a->net.n : 0; }

int nk_assoc_store_kmers(nk_assoc *a, const uint64_t *kmers, const uint32_t *counts, size_t n) {
  (void)counts;  // store_kmer's count is not used by the reference (:99-110)
  if (!a || (n && !kmers)) return nk_fail_msg(NK_E_INVALID, "null argument");
  if (!n) return NK_OK;
  nk_willshaw &w = a->net;
  AS_CHK(hipSetDevice(w.device));
  if (n > a->batch_cap) {
    if (a->batch) AS_CHK(hipFree(a->batch));
    a->batch = nullptr;
    a->batch_cap = 0;
    AS_CHK(hipMalloc((void **)&a->batch, n * 8));
    a->batch_cap = n;
  }
  AS_CHK(hipMemcpyAsync(a->batch, kmers, n * 8, hipMemcpyHostToDevice, w.s));
  hipLaunchKernelGGL(k_assoc_store, dim3(grid_of(n, 256)), dim3(256), 0, w.s, w.W, w.words, w.n,
                     a->batch, (uint64_t)n);
  AS_CHK(hipGetLastError());
  // the distinct k-mers in store order (kmer_to_pattern / pattern_to_kmers)
  std::vector<uint64_t> fresh;
  for (size_t i = 0; i < n; ++i)
    if (a->seen.insert(kmers[i]).second) fresh.push_back(kmers[i]);
  if (a->nk + fresh.size() > a->cap) {
    size_t nc = std::max<size_t>(2 * a->cap, a->nk + fresh.size());
    uint64_t *nb = nullptr;
    AS_CHK(hipMalloc((void **)&nb, nc * 8));
    if (a->nk) AS_CHK(hipMemcpyAsync(nb, a->kmers, a->nk * 8, hipMemcpyDeviceToDevice, w.s));
    AS_CHK(hipStreamSynchronize(w.s));
    if (a->kmers) AS_CHK(hipFree(a->kmers));
    a->kmers = nb;
    a->cap = nc;
    if (a->res) AS_CHK(hipFree(a->res));
    a->res = nullptr;
    AS_CHK(hipMalloc((void **)&a->res, nc * 16));
  }
  if (!fresh.empty())
    AS_CHK(hipMemcpyAsync(a->kmers + a->nk, fresh.data(), fresh.size() * 8, hipMemcpyHostToDevice,
                          w.s));
  AS_CHK(hipStreamSynchronize(w.s));  // kmers / fresh are host memory the copies read
  a->nk += fresh.size();
  w.stored += n;
  return NK_OK;
}

long nk_assoc_find_similar(nk_assoc *a, uint64_t query, size_t max_distance, uint64_t *kmers,
                           float *sim, size_t cap) {
  if (!a || (cap && (!kmers || !sim))) return nk_fail_msg(NK_E_INVALID, "null argument");
  nk_willshaw &w = a->net;
  AS_CHK(hipSetDevice(w.device));
  // the query's pattern, recalled over 10 steps (:115-118)
  if (w.words) AS_CHK(hipMemsetAsync(w.state, 0, w.words * 4, w.s));
  hipLaunchKernelGGL(k_assoc_query_bits, dim3(1), dim3(64), 0, w.s, query, w.n, w.state);
  AS_CHK(hipGetLastError());
  uint32_t *rec = nullptr;
  int rc = ws_recall_dev(&w, 10, &rec);
  if (rc) return rc;
  std::vector<uint32_t> r(std::max<uint32_t>(w.words, 1), 0);
  if (w.words) AS_CHK(hipMemcpyAsync(r.data(), rec, w.words * 4, hipMemcpyDeviceToHost, w.s));
  AS_CHK(hipMemsetAsync(a->n_res, 0, 8, w.s));
  AS_CHK(hipStreamSynchronize(w.s));
  uint32_t pop = 0;
  for (uint32_t x : r) pop += (uint32_t)__builtin_popcount(x);
  if (a->nk) {
    hipLaunchKernelGGL(k_assoc_distance, dim3(grid_of(a->nk, 256)), dim3(256), 0, w.s, a->kmers,
                       (uint64_t)a->nk, w.n, rec, pop, (uint64_t)max_distance, a->res, a->n_res);
    AS_CHK(hipGetLastError());
  }
  unsigned long long m = 0;
  AS_CHK(hipMemcpyAsync(&m, a->n_res, 8, hipMemcpyDeviceToHost, w.s));
  AS_CHK(hipStreamSynchronize(w.s));
  std::vector<uint64_t> res(2 * m), km(a->nk);
  if (m) {
    AS_CHK(hipMemcpyAsync(res.data(), a->res, m * 16, hipMemcpyDeviceToHost, w.s));
    AS_CHK(hipMemcpyAsync(km.data(), a->kmers, a->nk * 8, hipMemcpyDeviceToHost, w.s));
    AS_CHK(hipStreamSynchronize(w.s));
  }
  // similarity descending (:130); equal similarities by k-mer ascending (the
  // reference's order there follows HashMap iteration, which is unspecified)
  std::vector<std::pair<uint64_t, uint64_t>> out(m);  // (distance, kmer)
  for (unsigned long long i = 0; i < m; ++i) out[i] = {res[2 * i + 1], km[res[2 * i]]};
  std::sort(out.begin(), out.end());
  for (size_t i = 0; i < out.size() && i < cap; ++i) {
    kmers[i] = out[i].second;
    sim[i] = 1.0f - (float)out[i].first / (float)w.n;
  }
  return (long)m;
}

}  // extern "C"
