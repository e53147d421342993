/*
 * nk_oracle.c — CPU restatement of NeuroKmer's hot path (TEST INFRASTRUCTURE).
 *
 * See nk_oracle.h for scope and the pinning statement.  Build with
 * -ffp-contract=off: the reference computes `v*leak + c` as two rounded f32
 * operations (Rust never contracts), src/models.rs:41.
 *
 * The code follows the reference's control flow on purpose (per-record local
 * maps merged serially, serial kmer_per_neuron rebuild, serial LIF loop) so it
 * can double as the "port" CPU baseline timed by bench.py.
 */
#include "nk_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------ */
/* SipHash (siphasher 1.0.2, Cargo.lock:1520-1522; call site                */
/* src/spiking_hash.rs:78-82)                                               */
/* ------------------------------------------------------------------------ */
static inline uint64_t rotl64(uint64_t x, int b) { return (x << b) | (x >> (64 - b)); }

#define SIPROUND                                                              \
  do {                                                                        \
    v0 += v1; v1 = rotl64(v1, 13); v1 ^= v0; v0 = rotl64(v0, 32);             \
    v2 += v3; v3 = rotl64(v3, 16); v3 ^= v2;                                  \
    v0 += v3; v3 = rotl64(v3, 21); v3 ^= v0;                                  \
    v2 += v1; v1 = rotl64(v1, 17); v1 ^= v2; v2 = rotl64(v2, 32);             \
  } while (0)

uint64_t nko_siphash(int c_rounds, int d_rounds, uint64_t k0, uint64_t k1,
                     const uint8_t *msg, size_t len) {
  uint64_t v0 = 0x736f6d6570736575ULL ^ k0;
  uint64_t v1 = 0x646f72616e646f6dULL ^ k1;
  uint64_t v2 = 0x6c7967656e657261ULL ^ k0;
  uint64_t v3 = 0x7465646279746573ULL ^ k1;
  size_t full = len & ~(size_t)7;
  for (size_t i = 0; i < full; i += 8) {
    uint64_t m = 0;
    for (int j = 0; j < 8; ++j) m |= (uint64_t)msg[i + j] << (8 * j);
    v3 ^= m;
    for (int r = 0; r < c_rounds; ++r) SIPROUND;
    v0 ^= m;
  }
  uint64_t b = ((uint64_t)(len & 0xff)) << 56;
  for (size_t j = 0; j < (len & 7); ++j) b |= (uint64_t)msg[full + j] << (8 * j);
  v3 ^= b;
  for (int r = 0; r < c_rounds; ++r) SIPROUND;
  v0 ^= b;
  v2 ^= 0xff;
  for (int r = 0; r < d_rounds; ++r) SIPROUND;
  return v0 ^ v1 ^ v2 ^ v3;
}

uint64_t nko_sip13_u64(uint64_t m) {
  uint8_t le[8];
  for (int j = 0; j < 8; ++j) le[j] = (uint8_t)(m >> (8 * j));
  return nko_siphash(1, 3, 0, 0, le, 8);
}

uint64_t nko_map_kmer(uint64_t kmer, uint64_t pool) { return nko_sip13_u64(kmer) % pool; }

/* ------------------------------------------------------------------------ */
/* RollingKmerHash, src/models.rs:175-299.  Release-build semantics: the     */
/* `<<` at :265 masks its shift amount to 6 bits (k>32), `power` becomes 0   */
/* for k>=33 (:192-194), `mask` = !0 for k>=32 (:188).                       */
/* ------------------------------------------------------------------------ */
typedef struct {
  size_t k;
  uint64_t fwd, rev, mask, power;
} roll_t;

static inline uint64_t base_to_bits(uint8_t b) { /* models.rs:231-239 */
  switch (b) {
    case 'A': case 'a': return 0;
    case 'C': case 'c': return 1;
    case 'G': case 'g': return 2;
    case 'T': case 't': return 3;
    default: return 0;
  }
}
static inline uint64_t base_to_comp_bits(uint8_t b) { /* models.rs:243-251 */
  switch (b) {
    case 'A': case 'a': return 3;
    case 'C': case 'c': return 2;
    case 'G': case 'g': return 1;
    case 'T': case 't': return 0;
    default: return 0;
  }
}

static void roll_new(roll_t *h, size_t k) { /* models.rs:186-203 */
  h->k = k;
  h->mask = k < 32 ? ((1ULL << (2 * k)) - 1) : ~0ULL;
  uint64_t p = 1;
  for (size_t i = 0; i + 1 < k; ++i) p = (p << 2) & h->mask;
  h->power = p;
  h->fwd = 0;
  h->rev = 0;
}
static void roll_init(roll_t *h, const uint8_t *first_k) { /* models.rs:206-227 */
  h->fwd = 0;
  for (size_t i = 0; i < h->k; ++i) h->fwd = ((h->fwd << 2) & h->mask) | base_to_bits(first_k[i]);
  h->rev = 0;
  for (size_t i = h->k; i-- > 0;) h->rev = ((h->rev << 2) & h->mask) | base_to_comp_bits(first_k[i]);
}
static inline void roll_slide(roll_t *h, uint8_t next, uint8_t prev) { /* models.rs:254-269 */
  uint64_t pb = base_to_bits(prev), nb = base_to_bits(next);
  h->fwd = h->fwd - pb * h->power; /* wrapping_sub, wrapping mul in release */
  h->fwd = ((h->fwd << 2) | nb) & h->mask;
  uint64_t cn = base_to_comp_bits(next);
  unsigned sh = (unsigned)((2 * (h->k - 1)) & 63); /* release-mode shl masks to 6 bits */
  h->rev = (h->rev >> 2) | (cn << sh);
  h->rev &= h->mask;
}

uint64_t nko_pack_kmer(const uint8_t *w, size_t k) { /* utils.rs:26-39 */
  uint64_t packed = 0;
  for (size_t i = 0; i < k; ++i) {
    uint64_t bits;
    switch (w[i]) {
      case 'A': case 'a': bits = 0; break;
      case 'C': case 'c': bits = 1; break;
      case 'G': case 'g': bits = 2; break;
      case 'T': case 't': bits = 3; break;
      default: continue; /* skip N/ambiguous */
    }
    packed = (packed << 2) | bits;
  }
  return packed;
}

/* Calls emit(key, ctx) for every k-mer of one record in the reference's order
 * (src/spiking_hash.rs:102-138; identical loop at :326-352). */
typedef void (*emit_fn)(uint64_t key, void *ctx);
static void record_kmers(const uint8_t *seq, size_t len, size_t k, int canonical,
                         emit_fn emit, void *ctx) {
  if (canonical && len >= k) {
    roll_t h;
    roll_new(&h, k);
    roll_init(&h, seq);
    emit(h.fwd < h.rev ? h.fwd : h.rev, ctx);
    for (size_t i = 1; i + k <= len; ++i) {
      roll_slide(&h, seq[i + k - 1], seq[i - 1]);
      emit(h.fwd < h.rev ? h.fwd : h.rev, ctx);
    }
  } else {
    if (len < k) return; /* seq.windows(k) yields nothing */
    for (size_t i = 0; i + k <= len; ++i) emit(nko_pack_kmer(seq + i, k), ctx);
  }
}

typedef struct { uint64_t *out; size_t n; } collect_ctx;
static void collect_emit(uint64_t key, void *ctx) {
  collect_ctx *c = (collect_ctx *)ctx;
  c->out[c->n++] = key;
}
size_t nko_kmer_keys(const uint8_t *seq, size_t len, size_t k, int canonical, uint64_t *out) {
  collect_ctx c = {out, 0};
  if (k == 0) return 0;
  record_kmers(seq, len, k, canonical, collect_emit, &c);
  return c.n;
}

/* ------------------------------------------------------------------------ */
/* --kmer-width=128: the build's true k<=64 mode.  Not in  */
/* the reference; defined here and restated on the device:                   */
/*   canonical: fwd = sum code(b_i) << 2(k-1-i), rev = sum comp(b_i) << 2i    */
/*     over the window (A1 codes: other bytes -> 0 on both strands),         */
/*     key = min(fwd, rev) as u128;                                          */
/*   non-canonical: pack_kmer in u128 (skips non-ACGT, keeps the last 64);   */
/*   neuron = SipHash-1-3(key 0) over the key's 16 LE bytes (what u128::hash */
/*     feeds SipHasher13: Hasher::write_u128 -> to_ne_bytes) % pool.         */
/* ------------------------------------------------------------------------ */
uint64_t nko_sip13_u128(uint64_t lo, uint64_t hi) {
  uint8_t le[16];
  for (int i = 0; i < 8; ++i) le[i] = (uint8_t)(lo >> (8 * i));
  for (int i = 0; i < 8; ++i) le[8 + i] = (uint8_t)(hi >> (8 * i));
  return nko_siphash(1, 3, 0, 0, le, 16);
}

typedef unsigned __int128 u128;
typedef void (*emit128_fn)(u128 key, void *ctx);
static void record_kmers128(const uint8_t *seq, size_t len, size_t k, int canonical,
                            emit128_fn emit, void *ctx) {
  if (len < k) return;
  const u128 mask = k >= 64 ? ~(u128)0 : (((u128)1 << (2 * k)) - 1);
  if (canonical) {
    u128 fwd = 0, rev = 0;
    for (size_t i = 0; i < k; ++i) fwd = ((fwd << 2) | base_to_bits(seq[i])) & mask;
    for (size_t i = k; i-- > 0;) rev = ((rev << 2) | base_to_comp_bits(seq[i])) & mask;
    emit(fwd < rev ? fwd : rev, ctx);
    for (size_t i = 1; i + k <= len; ++i) {
      const uint8_t nx = seq[i + k - 1];
      fwd = ((fwd << 2) | base_to_bits(nx)) & mask;
      rev = (rev >> 2) | ((u128)base_to_comp_bits(nx) << (2 * (k - 1)));
      emit(fwd < rev ? fwd : rev, ctx);
    }
  } else {
    for (size_t i = 0; i + k <= len; ++i) {
      u128 packed = 0;
      for (size_t j = 0; j < k; ++j) {
        const uint8_t b = seq[i + j];
        if (b == 'A' || b == 'a' || b == 'C' || b == 'c' || b == 'G' || b == 'g' || b == 'T' ||
            b == 't')
          packed = (packed << 2) | base_to_bits(b);
      }
      emit(packed, ctx);
    }
  }
}

typedef struct { uint64_t *out; size_t n; } collect128_ctx;
static void collect128_emit(u128 key, void *ctx) {
  collect128_ctx *c = (collect128_ctx *)ctx;
  c->out[2 * c->n] = (uint64_t)key;
  c->out[2 * c->n + 1] = (uint64_t)(key >> 64);
  c->n++;
}
size_t nko_kmer_keys128(const uint8_t *seq, size_t len, size_t k, int canonical, uint64_t *out) {
  collect128_ctx c = {out, 0};
  if (k == 0 || k > 64) return 0;
  record_kmers128(seq, len, k, canonical, collect128_emit, &c);
  return c.n;
}
static uint64_t map128(u128 key, uint64_t pool) {
  return nko_sip13_u128((uint64_t)key, (uint64_t)(key >> 64)) % pool;
}

/* ------------------------------------------------------------------------ */
/* Exact k-mer map (the reference's HashMap<u64,u32> / DashMap<u64,AtomicU32>)*/
/* Open addressing, linear probing; counts wrap at 2^32 like the AtomicU32.   */
/* ------------------------------------------------------------------------ */
typedef struct {
  uint64_t *keys;
  uint32_t *vals;
  uint8_t *used;
  size_t cap, n;
} kmap_t;

static inline uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}
static void kmap_init(kmap_t *m, size_t cap_hint) {
  size_t cap = 64;
  while (cap < cap_hint * 2) cap <<= 1;
  m->cap = cap;
  m->n = 0;
  m->keys = (uint64_t *)malloc(cap * sizeof(uint64_t));
  m->vals = (uint32_t *)malloc(cap * sizeof(uint32_t));
  m->used = (uint8_t *)calloc(cap, 1);
}
static void kmap_free(kmap_t *m) {
  free(m->keys); free(m->vals); free(m->used);
  memset(m, 0, sizeof(*m));
}
static void kmap_add(kmap_t *m, uint64_t key, uint32_t v);
static void kmap_grow(kmap_t *m) {
  kmap_t nm;
  kmap_init(&nm, m->cap);
  for (size_t i = 0; i < m->cap; ++i)
    if (m->used[i]) kmap_add(&nm, m->keys[i], m->vals[i]);
  kmap_free(m);
  *m = nm;
}
static void kmap_add(kmap_t *m, uint64_t key, uint32_t v) {
  if ((m->n + 1) * 2 > m->cap) kmap_grow(m);
  size_t msk = m->cap - 1, i = mix64(key) & msk;
  while (m->used[i]) {
    if (m->keys[i] == key) { m->vals[i] += v; return; }
    i = (i + 1) & msk;
  }
  m->used[i] = 1;
  m->keys[i] = key;
  m->vals[i] = v;
  m->n++;
}
static int kmap_get(const kmap_t *m, uint64_t key, uint32_t *out) {
  if (!m->cap) return 0;
  size_t msk = m->cap - 1, i = mix64(key) & msk;
  while (m->used[i]) {
    if (m->keys[i] == key) { *out = m->vals[i]; return 1; }
    i = (i + 1) & msk;
  }
  return 0;
}

/* the same map over u128 keys (--kmer-width=128) */
typedef struct {
  u128 *keys;
  uint32_t *vals;
  uint8_t *used;
  size_t cap, n;
} kmap128_t;
static inline uint64_t mix128(u128 k) { return mix64((uint64_t)k ^ mix64((uint64_t)(k >> 64))); }
static void kmap128_init(kmap128_t *m, size_t cap_hint) {
  size_t cap = 64;
  while (cap < cap_hint * 2) cap <<= 1;
  m->cap = cap;
  m->n = 0;
  m->keys = (u128 *)malloc(cap * sizeof(u128));
  m->vals = (uint32_t *)malloc(cap * sizeof(uint32_t));
  m->used = (uint8_t *)calloc(cap, 1);
}
static void kmap128_free(kmap128_t *m) {
  free(m->keys); free(m->vals); free(m->used);
  memset(m, 0, sizeof(*m));
}
static void kmap128_add(kmap128_t *m, u128 key, uint32_t v);
static void kmap128_grow(kmap128_t *m) {
  kmap128_t nm;
  kmap128_init(&nm, m->cap);
  for (size_t i = 0; i < m->cap; ++i)
    if (m->used[i]) kmap128_add(&nm, m->keys[i], m->vals[i]);
  kmap128_free(m);
  *m = nm;
}
static void kmap128_add(kmap128_t *m, u128 key, uint32_t v) {
  if ((m->n + 1) * 2 > m->cap) kmap128_grow(m);
  size_t msk = m->cap - 1, i = mix128(key) & msk;
  while (m->used[i]) {
    if (m->keys[i] == key) { m->vals[i] += v; return; }
    i = (i + 1) & msk;
  }
  m->used[i] = 1;
  m->keys[i] = key;
  m->vals[i] = v;
  m->n++;
}
static int kmap128_get(const kmap128_t *m, u128 key, uint32_t *out) {
  if (!m->cap) return 0;
  size_t msk = m->cap - 1, i = mix128(key) & msk;
  while (m->used[i]) {
    if (m->keys[i] == key) { *out = m->vals[i]; return 1; }
    i = (i + 1) & msk;
  }
  return 0;
}

/* ------------------------------------------------------------------------ */
/* LifNeuron (src/models.rs:9-51) and EnergyTracker (:145-173)               */
/* ------------------------------------------------------------------------ */
static inline int lif_update(float *v, uint32_t *r, uint64_t *sc, float thr, float leak,
                             uint32_t refr, float c) {
  if (*r > 0) { *r -= 1; return 0; }
  float t = *v * leak; /* two roundings, never fused (-ffp-contract=off) */
  *v = t + c;
  if (*v >= thr) { *v = 0.0f; *r = refr; *sc += 1; return 1; }
  return 0;
}

/* Rust `f64 as u64`: saturating, NaN -> 0 */
static uint64_t f64_as_u64(double x) {
  if (!(x > 0.0)) return 0;
  if (x >= 18446744073709551616.0) return UINT64_MAX;
  return (uint64_t)x;
}

void nko_lif(uint64_t count, uint64_t steps, float thr, float leak, uint32_t refr,
             int skip_zero, float *v, uint32_t *r, uint64_t *spikes) {
  double total = (double)count;
  if (skip_zero && total == 0.0) return;
  float c = (float)(total / (double)steps);
  for (uint64_t s = 0; s < steps; ++s) lif_update(v, r, spikes, thr, leak, refr, c);
}

/* ------------------------------------------------------------------------ */
/* SpikingKmerCounter (src/spiking_hash.rs:16-77)                            */
/* ------------------------------------------------------------------------ */
struct nko_counter {
  size_t k, pool;
  float thr, leak;
  uint32_t refr;
  double cost;
  int canonical;
  uint64_t steps;
  /* neurons */
  float *v;
  uint32_t *r;
  uint64_t *sc;
  /* neuron_currents, kmer_per_neuron, counts */
  uint64_t *currents;
  uint32_t *kpn;
  kmap_t counts;
  int width;           /* 64: the reference's u64 keys; 128: --kmer-width=128 */
  kmap128_t counts128; /* counts when width == 128 */
  /* energy */
  uint64_t total_spikes, total_energy;
};

nko_counter *nko_new_w(size_t k, float threshold, float leak, uint32_t refractory,
                       double spike_cost, size_t pool_size, int use_canonical, int width) {
  if (width != 64 && width != 128) return NULL;
  if (width == 128 && (k == 0 || k > 64)) return NULL;
  nko_counter *c = (nko_counter *)calloc(1, sizeof(*c));
  c->width = width;
  kmap128_init(&c->counts128, 16);
  c->k = k; c->pool = pool_size; c->thr = threshold; c->leak = leak;
  c->refr = refractory; c->cost = spike_cost; c->canonical = use_canonical;
  c->steps = 1000; /* src/spiking_hash.rs:70 */
  size_t P = pool_size ? pool_size : 1;
  c->v = (float *)calloc(P, sizeof(float));
  c->r = (uint32_t *)calloc(P, sizeof(uint32_t));
  c->sc = (uint64_t *)calloc(P, sizeof(uint64_t));
  c->currents = (uint64_t *)calloc(P, sizeof(uint64_t));
  c->kpn = (uint32_t *)calloc(P, sizeof(uint32_t));
  kmap_init(&c->counts, 16);
  return c;
}

nko_counter *nko_new(size_t k, float threshold, float leak, uint32_t refractory,
                     double spike_cost, size_t pool_size, int use_canonical) {
  return nko_new_w(k, threshold, leak, refractory, spike_cost, pool_size, use_canonical, 64);
}

void nko_free(nko_counter *c) {
  if (!c) return;
  free(c->v); free(c->r); free(c->sc); free(c->currents); free(c->kpn);
  kmap_free(&c->counts);
  kmap128_free(&c->counts128);
  free(c);
}

static inline void add_spikes(nko_counter *c, uint64_t n) { /* models.rs:159-164 */
  c->total_spikes += n;
  c->total_energy += n * f64_as_u64(c->cost * 1000.0);
}

/* ---- fold/reduce over records (spiking_hash.rs:94-154) -------------------- */
typedef struct {
  nko_counter *c;
  const uint8_t *bases;
  const uint64_t *offsets;
  size_t n_recs;
  size_t next; /* record work queue: rayon's work unit is one record (:94-95) */
  pthread_mutex_t mu;
  kmap_t *maps; /* one map per record, like `maps.push(local_counts)` (:141) */
  kmap128_t *maps128; /* width 128 */
} fold_shared;

typedef struct {
  fold_shared *s;
  uint64_t *currents; /* per-split `vec![0u64; pool_size]` (:97) */
} fold_arg;

typedef struct { uint64_t *currents; kmap128_t *map; uint64_t pool; } rec128_ctx;
static void rec128_emit(u128 key, void *vctx) {
  rec128_ctx *x = (rec128_ctx *)vctx;
  kmap128_add(x->map, key, 1);
  x->currents[map128(key, x->pool)] += 1;
}

typedef struct { uint64_t *currents; kmap_t *map; uint8_t *unique; uint64_t pool; } rec_ctx;
static void rec_emit(uint64_t key, void *vctx) {
  rec_ctx *x = (rec_ctx *)vctx;
  kmap_add(x->map, key, 1);                  /* :110,124,133 */
  uint64_t idx = nko_map_kmer(key, x->pool); /* :111,125,135 */
  x->currents[idx] += 1;                     /* :112,126,136 */
  x->unique[idx] = 1;                        /* :113,127,137 (never read) */
}

static void *fold_worker(void *p) {
  fold_arg *a = (fold_arg *)p;
  fold_shared *s = a->s;
  nko_counter *c = s->c;
  for (;;) {
    pthread_mutex_lock(&s->mu);
    size_t i = s->next++;
    pthread_mutex_unlock(&s->mu);
    if (i >= s->n_recs) break;
    const uint8_t *seq = s->bases + s->offsets[i];
    size_t len = (size_t)(s->offsets[i + 1] - s->offsets[i]);
    if (c->width == 128) {
      kmap128_init(&s->maps128[i], 16);
      rec128_ctx x = {a->currents, &s->maps128[i], c->pool};
      record_kmers128(seq, len, c->k, c->canonical, rec128_emit, &x);
      continue;
    }
    uint8_t *unique = (uint8_t *)calloc(c->pool ? c->pool : 1, 1); /* :100 */
    kmap_init(&s->maps[i], 16);
    rec_ctx x = {a->currents, &s->maps[i], unique, c->pool};
    record_kmers(seq, len, c->k, c->canonical, rec_emit, &x);
    free(unique);
  }
  return NULL;
}

static int has_kmers(const nko_counter *c, const uint64_t *offsets, size_t n_recs) {
  for (size_t i = 0; i < n_recs; ++i)
    if (offsets[i + 1] - offsets[i] >= c->k) return 1;
  return 0;
}

/* Shared accumulate phase of process_parallel / process_file_streaming. */
static int accumulate(nko_counter *c, const uint8_t *bases, const uint64_t *offsets,
                      size_t n_recs, int n_threads) {
  if (c->k == 0) return -1;                                      /* reference panics */
  if (c->pool == 0 && has_kmers(c, offsets, n_recs)) return -1;  /* `% 0` panics */
  if (n_threads < 1) n_threads = 1;
  size_t P = c->pool ? c->pool : 1;
  fold_shared s;
  s.c = c; s.bases = bases; s.offsets = offsets; s.n_recs = n_recs; s.next = 0;
  pthread_mutex_init(&s.mu, NULL);
  s.maps = (kmap_t *)calloc(n_recs ? n_recs : 1, sizeof(kmap_t));
  s.maps128 = (kmap128_t *)calloc(n_recs ? n_recs : 1, sizeof(kmap128_t));
  fold_arg *args = (fold_arg *)calloc((size_t)n_threads, sizeof(fold_arg));
  pthread_t *th = (pthread_t *)calloc((size_t)n_threads, sizeof(pthread_t));
  for (int t = 0; t < n_threads; ++t) {
    args[t].s = &s;
    args[t].currents = (uint64_t *)calloc(P, sizeof(uint64_t));
  }
  if (n_threads == 1) fold_worker(&args[0]);
  else {
    /* the workers pull records from s.next: a thread that cannot be created
       has its (empty or partial) share run on the calling thread */
    int *made = (int *)calloc((size_t)n_threads, sizeof(int));
    for (int t = 0; t < n_threads; ++t)
      made[t] = pthread_create(&th[t], NULL, fold_worker, &args[t]) == 0;
    for (int t = 0; t < n_threads; ++t) {
      if (made[t]) pthread_join(th[t], NULL);
      else fold_worker(&args[t]);
    }
    free(made);
  }
  /* reduce: elementwise u64 sum (:145-154) */
  memset(c->currents, 0, P * sizeof(uint64_t));
  for (int t = 0; t < n_threads; ++t) {
    for (size_t i = 0; i < c->pool; ++i) c->currents[i] += args[t].currents[i];
    free(args[t].currents);
  }
  /* counts.clear(); merge the local maps serially (:157-165) */
  memset(c->kpn, 0, P * sizeof(uint32_t));
  if (c->width == 128) {
    kmap128_free(&c->counts128);
    kmap128_init(&c->counts128, 16);
    for (size_t i = 0; i < n_recs; ++i) {
      kmap128_t *m = &s.maps128[i];
      for (size_t j = 0; j < m->cap; ++j)
        if (m->used[j]) kmap128_add(&c->counts128, m->keys[j], m->vals[j]);
      kmap128_free(m);
    }
    for (size_t j = 0; j < c->counts128.cap; ++j)
      if (c->counts128.used[j]) c->kpn[map128(c->counts128.keys[j], c->pool)] += 1;
  } else {
    kmap_free(&c->counts);
    kmap_init(&c->counts, 16);
    for (size_t i = 0; i < n_recs; ++i) {
      kmap_t *m = &s.maps[i];
      for (size_t j = 0; j < m->cap; ++j)
        if (m->used[j]) kmap_add(&c->counts, m->keys[j], m->vals[j]);
      kmap_free(m);
    }
    /* kmer_per_neuron rebuild (:167-172) */
    for (size_t j = 0; j < c->counts.cap; ++j)
      if (c->counts.used[j]) c->kpn[nko_map_kmer(c->counts.keys[j], c->pool)] += 1;
  }
  pthread_mutex_destroy(&s.mu);
  free(s.maps); free(s.maps128); free(args); free(th);
  return 0;
}

/* Test-speed memo for the LIF loop (oracle only): a neuron that enters the
 * 1000-step loop in the fresh state (v = +0.0, r = 0) ends in a state that
 * depends on its count alone, so the reference loop runs ONCE per distinct
 * count among fresh neurons and the result is reused for the others
 * (pool = 16 M streaming / 256 M in-memory parity cases).  Neurons in any
 * other state always run the loop. */
#define LIF_MEMO_BITS 16
typedef struct { uint64_t count; uint64_t spikes; float v; uint32_t r; int used; } lif_memo_t;
static void lif_neuron(nko_counter *c, lif_memo_t *memo, size_t i, int skip_zero) {
  uint32_t vb;
  memcpy(&vb, &c->v[i], 4);
  if (memo && vb == 0 && c->r[i] == 0) {
    uint64_t cnt = c->currents[i];
    lif_memo_t *m = &memo[(cnt * 0x9E3779B97F4A7C15ULL) >> (64 - LIF_MEMO_BITS)];
    if (!(m->used && m->count == cnt)) {
      float v = 0.0f; uint32_t r = 0; uint64_t sp = 0;
      nko_lif(cnt, c->steps, c->thr, c->leak, c->refr, skip_zero, &v, &r, &sp);
      m->count = cnt; m->spikes = sp; m->v = v; m->r = r; m->used = 1;
    }
    c->v[i] = m->v; c->r[i] = m->r; c->sc[i] += m->spikes;
    return;
  }
  nko_lif(c->currents[i], c->steps, c->thr, c->leak, c->refr, skip_zero, &c->v[i], &c->r[i], &c->sc[i]);
}

int nko_process_parallel(nko_counter *c, const uint8_t *bases, const uint64_t *offsets,
                         size_t n_recs, int n_threads) {
  if (accumulate(c, bases, offsets, n_recs, n_threads)) return -1;
  /* Spike simulation, serial (:186-200) */
  lif_memo_t *memo = (lif_memo_t *)calloc((size_t)1 << LIF_MEMO_BITS, sizeof(lif_memo_t));
  for (size_t i = 0; i < c->pool; ++i) {
    uint64_t before = c->sc[i];
    lif_neuron(c, memo, i, 1);
    add_spikes(c, c->sc[i] - before);
  }
  free(memo);
  return 0;
}

/* simulate_spikes_simd (src/spiking_hash.rs:544-659) — what
 * simulate_spikes_auto (:697-714) runs on x86-64 with AVX2: `steps` updates of
 * every neuron from neuron_currents (zero currents included), per 8-lane batch
 * v' = active ? v*leak + c : v (two roundings), spike where active and
 * v' >= thr (the blend puts f32::MAX in the threshold of refractory lanes; a
 * refractory neuron's v is the 0 its spike left, so none spikes), r counted
 * down / set to refractory exactly as LifNeuron::update (src/models.rs:34-51);
 * total spikes and energy added once.  steps == 0 returns before touching
 * anything (:549-551). */
void nko_simulate_spikes_auto(nko_counter *c) {
  if (c->steps == 0) return;
  uint64_t total = 0;
  lif_memo_t *memo = (lif_memo_t *)calloc((size_t)1 << LIF_MEMO_BITS, sizeof(lif_memo_t));
  for (size_t i = 0; i < c->pool; ++i) {
    uint64_t before = c->sc[i];
    lif_neuron(c, memo, i, 0);
    total += c->sc[i] - before;
  }
  free(memo);
  add_spikes(c, total);
}

int nko_process_streaming(nko_counter *c, const uint8_t *bases, const uint64_t *offsets,
                          size_t n_recs, int n_threads) {
  if (accumulate(c, bases, offsets, n_recs, n_threads)) return -1;
  nko_simulate_spikes_auto(c); /* :482 */
  return 0;
}

/* process_sequence (src/spiking_hash.rs:203-273) */
typedef struct { nko_counter *c; uint8_t *unique; } seq_ctx;
static void seq_emit(uint64_t key, void *vctx) {
  seq_ctx *x = (seq_ctx *)vctx;
  uint64_t idx = nko_map_kmer(key, x->c->pool);
  kmap_add(&x->c->counts, key, 1);
  x->c->currents[idx] += 1;
  x->unique[idx] = 1;
}
static void seq128_emit(u128 key, void *vctx) {
  seq_ctx *x = (seq_ctx *)vctx;
  uint64_t idx = map128(key, x->c->pool);
  kmap128_add(&x->c->counts128, key, 1);
  x->c->currents[idx] += 1;
  x->unique[idx] = 1;
}
int nko_process_sequence(nko_counter *c, const uint8_t *seq, size_t len) {
  if (c->k == 0) return -1;
  if (len < c->k) return 0;
  if (c->pool == 0) return -1;
  uint8_t *unique = (uint8_t *)calloc(c->pool, 1);
  seq_ctx x = {c, unique};
  if (c->width == 128)
    record_kmers128(seq, len, c->k, c->canonical, seq128_emit, &x);
  else
    record_kmers(seq, len, c->k, c->canonical, seq_emit, &x);
  for (size_t i = 0; i < c->pool; ++i)
    if (unique[i]) c->kpn[i] += 1;
  for (size_t i = 0; i < c->pool; ++i) {
    double cur = (double)c->currents[i];
    if (cur > 0.0 && lif_update(&c->v[i], &c->r[i], &c->sc[i], c->thr, c->leak, c->refr, (float)cur))
      add_spikes(c, 1);
    c->currents[i] = 0;
  }
  free(unique);
  return 0;
}

const uint64_t *nko_currents(const nko_counter *c) { return c->currents; }
const float *nko_voltages(const nko_counter *c) { return c->v; }
const uint32_t *nko_refractory(const nko_counter *c) { return c->r; }
const uint64_t *nko_spike_counts(const nko_counter *c) { return c->sc; }
const uint32_t *nko_kmer_per_neuron(const nko_counter *c) { return c->kpn; }
uint64_t nko_total_spikes(const nko_counter *c) { return c->total_spikes; }
uint64_t nko_total_energy_fixed(const nko_counter *c) { return c->total_energy; }
double nko_energy_used(const nko_counter *c) { return (double)c->total_energy / 1000.0; }
size_t nko_distinct_kmers(const nko_counter *c) {
  return c->width == 128 ? c->counts128.n : c->counts.n;
}
void nko_set_steps(nko_counter *c, uint64_t steps) { c->steps = steps; }
uint64_t nko_get_steps(const nko_counter *c) { return c->steps; }

/* top_abundant_neurons (src/spiking_hash.rs:661-673): stable sort by spike
 * count descending; equal counts keep ascending index order. */
typedef struct { uint64_t idx, sc; } top_t;
static int top_cmp(const void *a, const void *b) {
  const top_t *x = (const top_t *)a, *y = (const top_t *)b;
  if (x->sc != y->sc) return x->sc > y->sc ? -1 : 1;
  return x->idx < y->idx ? -1 : (x->idx > y->idx);
}
size_t nko_top_abundant(const nko_counter *c, size_t n, uint64_t *idx, uint64_t *spikes,
                        uint32_t *uniques) {
  size_t P = c->pool;
  if (n <= 4096 && P > 8 * n) {
    /* same order as the sort below, by selection: scan in index order and keep
     * the best m rows sorted (sc desc, idx asc); a later index never beats an
     * equal count, so only strictly larger counts enter (test speed at 256 M) */
    size_t m = n, have = 0;
    top_t *b = (top_t *)malloc((m ? m : 1) * sizeof(top_t));
    for (size_t i = 0; i < P; ++i) {
      uint64_t sc = c->sc[i];
      if (have == m && (m == 0 || sc <= b[m - 1].sc)) continue;
      size_t j = have < m ? have++ : m - 1;
      while (j > 0 && b[j - 1].sc < sc) { b[j] = b[j - 1]; --j; }
      b[j].idx = i; b[j].sc = sc;
    }
    for (size_t i = 0; i < have; ++i) {
      idx[i] = b[i].idx; spikes[i] = b[i].sc; uniques[i] = c->kpn[b[i].idx];
    }
    free(b);
    return have;
  }
  top_t *t = (top_t *)malloc((P ? P : 1) * sizeof(top_t));
  for (size_t i = 0; i < P; ++i) { t[i].idx = i; t[i].sc = c->sc[i]; }
  qsort(t, P, sizeof(top_t), top_cmp); /* (sc desc, idx asc) == stable sort */
  size_t m = n < P ? n : P;
  for (size_t i = 0; i < m; ++i) {
    idx[i] = t[i].idx;
    spikes[i] = t[i].sc;
    uniques[i] = c->kpn[t[i].idx];
  }
  free(t);
  return m;
}

int nko_get_count128(const nko_counter *c, uint64_t lo, uint64_t hi, uint32_t *out) {
  return kmap128_get(&c->counts128, ((u128)hi << 64) | lo, out);
}

int nko_get_count(const nko_counter *c, uint64_t kmer, uint32_t *out) {
  return kmap_get(&c->counts, kmer, out);
}

/* ------------------------------------------------------------------------ */
/* Lean CPU baseline (not the reference's structure; see nk_oracle.h)        */
/* ------------------------------------------------------------------------ */
typedef struct {
  const uint8_t *bases;
  const uint64_t *offsets;
  size_t n_recs, k;
  int canonical;
  uint64_t pool, steps, w_lo, w_hi; /* this thread's windows [w_lo, w_hi) of all windows */
  float thr, leak;                  /* LIF parameters (src/models.rs:20-51) */
  uint32_t refr;
  uint64_t *cur;                    /* this thread's currents (pool) */
  uint64_t *cur_all, *spikes, n_lo, n_hi, total; /* the LIF phase: neurons [n_lo, n_hi) */
  int nthreads, idx;
  void *all;
} lean_ctx;

static void *lean_count(void *p) {
  lean_ctx *t = (lean_ctx *)p;
  uint64_t w0 = 0; /* windows before record r */
  for (size_t r = 0; r < t->n_recs; ++r) {
    const uint64_t s0 = t->offsets[r], len = t->offsets[r + 1] - s0;
    const uint64_t nw = len >= t->k ? len - t->k + 1 : 0;
    const uint64_t a = t->w_lo > w0 ? t->w_lo - w0 : 0, b = t->w_hi < w0 + nw ? t->w_hi - w0 : nw;
    if (a < b) {
      const uint8_t *seq = t->bases + s0;
      if (t->canonical) {
        roll_t h;
        roll_new(&h, t->k);
        roll_init(&h, seq + a);
        t->cur[nko_sip13_u64(h.fwd < h.rev ? h.fwd : h.rev) % t->pool] += 1;
        for (uint64_t i = a + 1; i < b; ++i) {
          roll_slide(&h, seq[i + t->k - 1], seq[i - 1]);
          t->cur[nko_sip13_u64(h.fwd < h.rev ? h.fwd : h.rev) % t->pool] += 1;
        }
      } else {
        for (uint64_t i = a; i < b; ++i) t->cur[nko_sip13_u64(nko_pack_kmer(seq + i, t->k)) % t->pool] += 1;
      }
    }
    w0 += nw;
    if (w0 >= t->w_hi) break;
  }
  return NULL;
}

static void *lean_lif(void *p) {
  lean_ctx *t = (lean_ctx *)p;
  lean_ctx *all = (lean_ctx *)t->all;
  uint64_t tot = 0;
  enum { kMemo = 4096 };  /* spikes depend on the count alone (fresh state): memoised */
  uint64_t memo[kMemo];
  for (int i = 0; i < kMemo; ++i) memo[i] = UINT64_MAX;
  for (uint64_t i = t->n_lo; i < t->n_hi; ++i) {
    uint64_t c = 0;
    for (int j = 0; j < t->nthreads; ++j) c += all[j].cur[i];
    t->cur_all[i] = c;
    uint64_t sp;
    if (c < kMemo && memo[c] != UINT64_MAX) {
      sp = memo[c];
    } else {
      float v = 0.0f;
      uint32_t r = 0;
      sp = 0;
      nko_lif(c, t->steps, t->thr, t->leak, t->refr, 0, &v, &r, &sp);
      if (c < kMemo) memo[c] = sp;
    }
    t->spikes[i] = sp;
    tot += sp;
  }
  t->total = tot;
  return NULL;
}

/* fn(ctx[j]) on n threads; a thread that cannot be created runs its share
   on the calling thread */
static void run_threads(void *(*fn)(void *), lean_ctx *t, pthread_t *th, int n) {
  int *made = (int *)calloc((size_t)n, sizeof(int));
  for (int j = 0; j < n; ++j) made[j] = made && pthread_create(&th[j], NULL, fn, &t[j]) == 0;
  for (int j = 0; j < n; ++j) {
    if (made && made[j]) pthread_join(th[j], NULL);
    else fn(&t[j]);
  }
  free(made);
}

int nko_lean_currents_lif(const uint8_t *bases, const uint64_t *offsets, size_t n_recs, size_t k,
                          int canonical, uint64_t pool, uint64_t steps, float thr, float leak,
                          uint32_t refr, int n_threads,
                          uint64_t *currents, uint64_t *spikes, uint64_t *total_spikes) {
  if (!pool || k < 1 || k > 32 || n_threads < 1) return -1;
  uint64_t nw = 0;
  for (size_t r = 0; r < n_recs; ++r) {
    const uint64_t len = offsets[r + 1] - offsets[r];
    nw += len >= k ? len - k + 1 : 0;
  }
  lean_ctx *t = (lean_ctx *)calloc((size_t)n_threads, sizeof(lean_ctx));
  pthread_t *th = (pthread_t *)calloc((size_t)n_threads, sizeof(pthread_t));
  if (!t || !th) { free(t); free(th); return -1; }
  int rc = 0;
  for (int j = 0; j < n_threads; ++j) {
    t[j].bases = bases; t[j].offsets = offsets; t[j].n_recs = n_recs; t[j].k = k;
    t[j].canonical = canonical; t[j].pool = pool; t[j].steps = steps;
    t[j].thr = thr; t[j].leak = leak; t[j].refr = refr;
    t[j].w_lo = nw * (uint64_t)j / (uint64_t)n_threads;
    t[j].w_hi = nw * (uint64_t)(j + 1) / (uint64_t)n_threads;
    t[j].cur = (uint64_t *)calloc(pool, sizeof(uint64_t));
    t[j].cur_all = currents; t[j].spikes = spikes;
    t[j].n_lo = pool * (uint64_t)j / (uint64_t)n_threads;
    t[j].n_hi = pool * (uint64_t)(j + 1) / (uint64_t)n_threads;
    t[j].nthreads = n_threads; t[j].idx = j; t[j].all = t;
    if (!t[j].cur) rc = -1;
  }
  if (!rc) {
    run_threads(lean_count, t, th, n_threads);
    run_threads(lean_lif, t, th, n_threads);  /* (after every count: the LIF sums them) */
    uint64_t tot = 0;
    for (int j = 0; j < n_threads; ++j) tot += t[j].total;
    *total_spikes = tot;
  }
  for (int j = 0; j < n_threads; ++j) free(t[j].cur);
  free(t);
  free(th);
  return rc;
}
