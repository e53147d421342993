/* nk_assoc_oracle.c — TEST INFRASTRUCTURE ONLY: CPU restatement of the
 * reference's associative memory (src/associative.rs) used as the parity
 * checker of the device implementation (neurokmer_amd/csrc/nk_assoc.hip).
 * Nothing in the product path links or calls this file.
 *
 *   WillshawNetwork       src/associative.rs:12-62  (dense u8 weights, i32 sums,
 *                                                    exactly as the reference)
 *   KmerAssociativeMemory src/associative.rs:64-139
 *   blake3::hash          the blake3 crate (Cargo.lock: blake3; not vendored in
 *                         /root/reference): the published BLAKE3 algorithm for
 *                         one chunk (<= 1024 bytes), pinned against the
 *                         published digests of "" and "abc"
 *                         (tests/test_assoc_oracle.py).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* ---- BLAKE3, one chunk ----------------------------------------------------- */
static const uint32_t B3_IV[8] = {0x6A09E667u, 0xBB67AE85u, 0x3C6EF372u, 0xA54FF53Au,
                                  0x510E527Fu, 0x9B05688Cu, 0x1F83D9ABu, 0x5BE0CD19u};
static const uint8_t B3_PERM[16] = {2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8};
enum { B3_CHUNK_START = 1, B3_CHUNK_END = 2, B3_ROOT = 8 };

static uint32_t rotr32(uint32_t x, int r) { return (x >> r) | (x << (32 - r)); }

static void b3_g(uint32_t *v, int a, int b, int c, int d, uint32_t mx, uint32_t my) {
  v[a] = v[a] + v[b] + mx;
  v[d] = rotr32(v[d] ^ v[a], 16);
  v[c] = v[c] + v[d];
  v[b] = rotr32(v[b] ^ v[c], 12);
  v[a] = v[a] + v[b] + my;
  v[d] = rotr32(v[d] ^ v[a], 8);
  v[c] = v[c] + v[d];
  v[b] = rotr32(v[b] ^ v[c], 7);
}

/* the compression function; out16 = the full 16-word state after the
 * feed-forward of the chaining value (words 0..7 are the next cv / digest) */
static void b3_compress(const uint32_t cv[8], const uint32_t block[16], uint64_t counter,
                        uint32_t block_len, uint32_t flags, uint32_t out16[16]) {
  uint32_t v[16], m[16], t[16];
  memcpy(v, cv, 32);
  memcpy(v + 8, B3_IV, 16);
  v[12] = (uint32_t)counter;
  v[13] = (uint32_t)(counter >> 32);
  v[14] = block_len;
  v[15] = flags;
  memcpy(m, block, 64);
  for (int r = 0; r < 7; ++r) {
    b3_g(v, 0, 4, 8, 12, m[0], m[1]);
    b3_g(v, 1, 5, 9, 13, m[2], m[3]);
    b3_g(v, 2, 6, 10, 14, m[4], m[5]);
    b3_g(v, 3, 7, 11, 15, m[6], m[7]);
    b3_g(v, 0, 5, 10, 15, m[8], m[9]);
    b3_g(v, 1, 6, 11, 12, m[10], m[11]);
    b3_g(v, 2, 7, 8, 13, m[12], m[13]);
    b3_g(v, 3, 4, 9, 14, m[14], m[15]);
    for (int i = 0; i < 16; ++i) t[i] = m[B3_PERM[i]];
    memcpy(m, t, 64);
  }
  for (int i = 0; i < 8; ++i) {
    out16[i] = v[i] ^ v[i + 8];
    out16[i + 8] = v[i + 8] ^ cv[i];
  }
}

/* BLAKE3 of len <= 1024 bytes (one chunk, the root), 32-byte digest.
 * Returns -1 for longer inputs (not needed: the keys are 8 bytes). */
int nko_blake3(const uint8_t *in, size_t len, uint8_t out[32]) {
  if (len > 1024) return -1;
  uint32_t cv[8], st[16], block[16];
  memcpy(cv, B3_IV, 32);
  size_t nblk = len ? (len + 63) / 64 : 1;
  for (size_t b = 0; b < nblk; ++b) {
    uint8_t buf[64] = {0};
    size_t off = b * 64, n = len - off < 64 ? len - off : 64;
    if (len) memcpy(buf, in + off, n);
    else n = 0;
    for (int i = 0; i < 16; ++i)
      block[i] = (uint32_t)buf[4 * i] | ((uint32_t)buf[4 * i + 1] << 8) |
                 ((uint32_t)buf[4 * i + 2] << 16) | ((uint32_t)buf[4 * i + 3] << 24);
    uint32_t flags = (b == 0 ? B3_CHUNK_START : 0) | (b == nblk - 1 ? B3_CHUNK_END | B3_ROOT : 0);
    b3_compress(cv, block, 0, (uint32_t)n, flags, st);
    memcpy(cv, st, 32);
  }
  for (int i = 0; i < 8; ++i) {
    out[4 * i] = (uint8_t)cv[i];
    out[4 * i + 1] = (uint8_t)(cv[i] >> 8);
    out[4 * i + 2] = (uint8_t)(cv[i] >> 16);
    out[4 * i + 3] = (uint8_t)(cv[i] >> 24);
  }
  return 0;
}

/* ---- WillshawNetwork (src/associative.rs:12-62) ---------------------------- */
typedef struct nko_willshaw {
  uint8_t *w;  /* pattern_size x pattern_size, 0/1 */
  size_t n;
  uint64_t stored;
} nko_willshaw;

nko_willshaw *nko_willshaw_new(size_t n) {
  nko_willshaw *h = (nko_willshaw *)calloc(1, sizeof *h);
  if (!h) return NULL;
  h->n = n;
  const size_t nn = n * n;
  h->w = (uint8_t *)calloc(nn > 0 ? nn : 1, 1);
  if (!h->w) { free(h); return NULL; }
  return h;
}

void nko_willshaw_free(nko_willshaw *h) {
  if (!h) return;
  free(h->w);
  free(h);
}

/* :29-42  every (i, j) with both bits set gets weight 1 */
int nko_willshaw_store(nko_willshaw *h, const uint8_t *p, size_t len) {
  if (len != h->n) return -1; /* "Pattern size mismatch" */
  for (size_t i = 0; i < h->n; ++i)
    for (size_t j = 0; j < h->n; ++j)
      if (p[i] > 0 && p[j] > 0) h->w[i * h->n + j] = 1;
  h->stored++;
  return 0;
}

/* :45-61  synchronous updates, state' = (W . state > 0), stop when unchanged */
int nko_willshaw_recall(const nko_willshaw *h, const uint8_t *noisy, size_t len, size_t steps,
                        uint8_t *out) {
  if (len != h->n) return -1;
  size_t n = h->n;
  int8_t *s = (int8_t *)malloc(n ? n : 1), *t = (int8_t *)malloc(n ? n : 1);
  for (size_t i = 0; i < n; ++i) s[i] = noisy[i] > 0 ? 1 : 0;
  for (size_t step = 0; step < steps; ++step) {
    int same = 1;
    for (size_t i = 0; i < n; ++i) {
      int32_t sum = 0;
      for (size_t j = 0; j < n; ++j) sum += (int32_t)h->w[i * n + j] * (int32_t)s[j];
      t[i] = sum > 0 ? 1 : 0;
      if (t[i] != s[i]) same = 0;
    }
    if (same) break;
    memcpy(s, t, n);
  }
  for (size_t i = 0; i < n; ++i) out[i] = s[i] > 0 ? 255 : 0;
  free(s);
  free(t);
  return 0;
}

uint64_t nko_willshaw_stored(const nko_willshaw *h) { return h->stored; }

/* ---- KmerAssociativeMemory (src/associative.rs:64-139) --------------------- */
typedef struct nko_assoc {
  nko_willshaw *net;
  size_t n;         /* pattern size */
  uint64_t *kmers;  /* distinct stored k-mers (pattern_to_kmers' members) */
  size_t nk, cap;
} nko_assoc;

size_t nko_assoc_pattern_size(size_t k) { return k <= 10 ? ((size_t)1 << k) : 1024; } /* :73 */

/* :84-96  ~1% of the bits from the BLAKE3 digest of the key's 8 LE bytes */
void nko_assoc_kmer_pattern(size_t n, uint64_t kmer, uint8_t *p) {
  uint8_t le[8], d[32];
  for (int i = 0; i < 8; ++i) le[i] = (uint8_t)(kmer >> (8 * i));
  nko_blake3(le, 8, d);
  memset(p, 0, n);
  for (size_t i = 0; i < n / 100; ++i) p[d[i % 32] % n] = 255;
}

nko_assoc *nko_assoc_new(size_t k) {
  nko_assoc *a = (nko_assoc *)calloc(1, sizeof *a);
  if (!a) return NULL;
  a->n = nko_assoc_pattern_size(k);
  a->net = nko_willshaw_new(a->n);
  return a;
}

void nko_assoc_free(nko_assoc *a) {
  if (!a) return;
  nko_willshaw_free(a->net);
  free(a->kmers);
  free(a);
}

/* :99-110 (the count is not used by the reference) */
int nko_assoc_store(nko_assoc *a, uint64_t kmer, uint32_t count) {
  (void)count;
  uint8_t *p = (uint8_t *)malloc(a->n);
  nko_assoc_kmer_pattern(a->n, kmer, p);
  int rc = nko_willshaw_store(a->net, p, a->n);
  free(p);
  if (rc) return rc;
  for (size_t i = 0; i < a->nk; ++i)
    if (a->kmers[i] == kmer) return 0;
  if (a->nk == a->cap) {
    a->cap = a->cap ? 2 * a->cap : 64;
    a->kmers = (uint64_t *)realloc(a->kmers, a->cap * 8);
  }
  a->kmers[a->nk++] = kmer;
  return 0;
}

static int res_cmp(const void *x, const void *y) {
  const uint64_t *a = (const uint64_t *)x, *b = (const uint64_t *)y; /* [distance, kmer] */
  if (a[0] != b[0]) return a[0] < b[0] ? -1 : 1;
  return a[1] < b[1] ? -1 : (a[1] > b[1]);
}

/* :113-134  recall(query pattern, 10 steps), then every stored k-mer whose
 * pattern is within max_distance (Hamming, nonzero bits) of the recalled one,
 * similarity = 1 - d / n as f32, by similarity descending.  The reference's
 * order among equal similarities follows HashMap/HashSet iteration (not
 * specified); this restatement and the device take k-mer ascending. */
size_t nko_assoc_find_similar(const nko_assoc *a, uint64_t query, size_t max_distance,
                              uint64_t *kmers, float *sim, size_t cap) {
  size_t n = a->n;
  uint8_t *q = (uint8_t *)malloc(n ? n : 1), *r = (uint8_t *)malloc(n ? n : 1),
          *p = (uint8_t *)malloc(n ? n : 1);
  nko_assoc_kmer_pattern(n, query, q);
  nko_willshaw_recall(a->net, q, n, 10, r);
  uint64_t *res = (uint64_t *)malloc(2 * 8 * (a->nk ? a->nk : 1));
  size_t m = 0;
  for (size_t i = 0; i < a->nk; ++i) {
    nko_assoc_kmer_pattern(n, a->kmers[i], p);
    size_t d = 0;
    for (size_t j = 0; j < n; ++j) d += (r[j] > 0) != (p[j] > 0);
    if (d <= max_distance) {
      res[2 * m] = d;
      res[2 * m + 1] = a->kmers[i];
      ++m;
    }
  }
  qsort(res, m, 16, res_cmp);
  for (size_t i = 0; i < m && i < cap; ++i) {
    kmers[i] = res[2 * i + 1];
    sim[i] = 1.0f - (float)res[2 * i] / (float)n;
  }
  free(q);
  free(r);
  free(p);
  free(res);
  return m;
}
