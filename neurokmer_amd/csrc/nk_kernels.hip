// nk_kernels.hip — gfx950 kernels of the NeuroKmer k-mer -> spike hot path.
//
//   K1 k_kmers<CANON,MODE>  one workgroup = one tile of 4096 k-mer start
//       positions.  Coalesced 16-B loads of the tile (+64-base halo) are
//       converted once into three LDS bit streams: forward 2-bit codes
//       (MSB-first), complement codes (LSB-first) and an invalid-byte mask.
//       Each lane then extracts its window's forward and reverse-complement
//       values with two funnel shifts (no per-k-mer rolling), takes the
//       canonical min (src/models.rs:284-286), hashes with SipHash-1-3 and
//       reduces % pool exactly.  MODE 0 adds 1 to the neuron's u64 current
//       (src/spiking_hash.rs:112,126); MODE 1 (second pass) keeps only k-mers
//       of the top-N neurons and inserts them into a device hash set, which
//       gives "unique k-mers colliding" (src/spiking_hash.rs:157-172,661-673).
//   K1c k_kmers_compat<CANON,MODE>  k > 32: the reference's release-build u64
//       semantics (src/models.rs:188-194,260-266), one lane per position.
//   K3 k_lif_apply  closed-form LIF per neuron + spike histogram + totals.
//   K4 k_topn_*     exact top-N by (spikes desc, index asc).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "nk_device.h"
#include "nk_kernels.h"

namespace nk {

constexpr int kHalo = 64;                       // bases staged past the tile
constexpr int kStage = kTile + kHalo;           // 4160 bytes
constexpr int kChunks = kStage / 16;            // 260 16-B chunks
constexpr int kPerThread = kTile / kBlock;      // 16 positions per lane
constexpr unsigned long long kEmpty = ~0ULL;

// ---------------------------------------------------------------------------
// byte -> 2-bit code conversion (4 bytes at a time).  A/a 0, C/c 1, G/g 2,
// T/t 3, anything else 0 on BOTH strands (src/models.rs:231-251).
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t eq_bytes(uint32_t t, uint32_t c) {
  uint32_t z = t ^ c;
  return ~(((z & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | z) & 0x80808080u;  // 0x80 where byte == c
}

struct Conv4 {
  uint32_t fnib;  // 4 forward codes, first base in bits 7:6
  uint32_t rnib;  // 4 complement codes, first base in bits 1:0
  uint32_t inv;   // 4 invalid-byte bits, first base in bit 0
};

__device__ __forceinline__ Conv4 conv4(uint32_t x) {
  uint32_t t = x | 0x20202020u;
  uint32_t valid = eq_bytes(t, 0x61616161u) | eq_bytes(t, 0x63636363u) |
                   eq_bytes(t, 0x67676767u) | eq_bytes(t, 0x74747474u);
  uint32_t vm = valid >> 7;  // 0x01 per valid byte
  uint32_t vm3 = vm * 3u;
  uint32_t code = ((x >> 1) ^ (x >> 2)) & 0x03030303u & vm3;
  uint32_t comp = (code ^ 0x03030303u) & vm3;
  Conv4 o;
  o.fnib = ((code << 6) & 0xC0u) | ((code >> 4) & 0x30u) | ((code >> 14) & 0x0Cu) |
           ((code >> 24) & 0x03u);
  o.rnib = (comp & 0x03u) | ((comp >> 6) & 0x0Cu) | ((comp >> 12) & 0x30u) |
           ((comp >> 18) & 0xC0u);
  uint32_t m = ~vm & 0x01010101u;
  o.inv = (m & 1u) | ((m >> 7) & 2u) | ((m >> 14) & 4u) | ((m >> 21) & 8u);
  return o;
}

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}

__device__ __forceinline__ uint32_t code_of(uint8_t b) {
  uint32_t t = b | 0x20u;
  bool v = (t == 'a') | (t == 'c') | (t == 'g') | (t == 't');
  return v ? (((uint32_t)b >> 1) ^ ((uint32_t)b >> 2)) & 3u : 0u;
}
__device__ __forceinline__ uint32_t comp_of(uint8_t b) {
  uint32_t t = b | 0x20u;
  bool v = (t == 'a') | (t == 'c') | (t == 'g') | (t == 't');
  return v ? ((((uint32_t)b >> 1) ^ ((uint32_t)b >> 2)) & 3u) ^ 3u : 0u;
}
__device__ __forceinline__ bool valid_byte(uint8_t b) {
  uint32_t t = b | 0x20u;
  return (t == 'a') | (t == 'c') | (t == 'g') | (t == 't');
}

// ---------------------------------------------------------------------------
// first record of each tile: largest r < n_recs with offsets[r] <= tile start
// ---------------------------------------------------------------------------
__global__ void k_tile_rec(const uint64_t *__restrict__ offsets, uint64_t n_recs,
                           uint64_t n_tiles, uint32_t *__restrict__ tile_rec) {
  uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n_tiles) return;
  uint64_t pos = t * (uint64_t)kTile;
  uint64_t lo = 0, hi = n_recs;  // invariant: offsets[lo] <= pos, answer in [lo, hi)
  while (hi - lo > 1) {
    uint64_t mid = (lo + hi) >> 1;
    if (offsets[mid] <= pos) lo = mid;
    else hi = mid;
  }
  tile_rec[t] = (uint32_t)lo;
}

// ---------------------------------------------------------------------------
// top-N membership table in LDS (MODE 1)
// ---------------------------------------------------------------------------
__device__ __forceinline__ void set_insert(const UniqArgs &u, uint32_t slot, uint64_t key) {
  if (key == kEmpty) {
    if (atomicCAS(&u.special[slot], 0u, 1u) == 0u) atomicAdd(&u.uniq[slot], 1u);
    return;
  }
  uint64_t h = mix64(key) & u.set_mask;
  for (;;) {
    unsigned long long prev = atomicCAS(&u.set_keys[h], kEmpty, (unsigned long long)key);
    if (prev == kEmpty) {
      atomicAdd(&u.uniq[slot], 1u);
      return;
    }
    if (prev == key) return;
    h = (h + 1) & u.set_mask;
  }
}

__device__ __forceinline__ int probe_top(const uint64_t *tbl_idx, const uint32_t *tbl_slot,
                                         uint32_t tbl_mask, uint64_t idx) {
  uint32_t h = (uint32_t)idx & tbl_mask;
  for (;;) {
    uint64_t e = tbl_idx[h];
    if (e == idx) return (int)tbl_slot[h];
    if (e == kEmpty) return -1;
    h = (h + 1) & tbl_mask;
  }
}

__device__ void build_top_tbl(const UniqArgs &u, uint64_t *tbl_idx, uint32_t *tbl_slot) {
  for (uint32_t i = threadIdx.x; i < u.tbl_size; i += blockDim.x) tbl_idx[i] = kEmpty;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t mask = u.tbl_size - 1;
    for (uint32_t s = 0; s < u.n_top; ++s) {
      uint64_t idx = u.top[s].idx;
      uint32_t h = (uint32_t)idx & mask;
      while (tbl_idx[h] != kEmpty) h = (h + 1) & mask;
      tbl_idx[h] = idx;
      tbl_slot[h] = s;
    }
  }
  __syncthreads();
}

// ---------------------------------------------------------------------------
// K1: k <= 32
// ---------------------------------------------------------------------------
template <bool CANON, int MODE>
__global__ __launch_bounds__(kBlock) void k_kmers(KmerInput in, int k, FastMod fm,
                                                  unsigned long long *__restrict__ currents,
                                                  UniqArgs u) {
  __shared__ uint32_t sF[kChunks + 2];
  __shared__ uint32_t sR[kChunks + 2];
  __shared__ uint16_t sINV[kChunks + 4];
  __shared__ uint32_t sWIN[kTile / 32];
  __shared__ uint4 sRAW[CANON ? 1 : kChunks];
  extern __shared__ uint64_t dyn[];  // MODE 1: probe table

  const int tid = threadIdx.x;
  const uint64_t T0 = (uint64_t)blockIdx.x * kTile;
  const uint64_t n_bases = in.n_bases;

  // 1. stage the tile: coalesced 16-B loads -> bit streams
  for (int c = tid; c < kChunks; c += kBlock) {
    uint64_t g = T0 + 16ull * c;
    uint4 v;
    if (g + 16 <= n_bases) {
      v = *reinterpret_cast<const uint4 *>(in.bases + g);
    } else {
      uint32_t w[4] = {0, 0, 0, 0};
      for (int j = 0; j < 16; ++j)
        if (g + j < n_bases) w[j >> 2] |= (uint32_t)in.bases[g + j] << (8 * (j & 3));
      v = make_uint4(w[0], w[1], w[2], w[3]);
    }
    Conv4 a = conv4(v.x), b = conv4(v.y), cc = conv4(v.z), d = conv4(v.w);
    sF[c] = (a.fnib << 24) | (b.fnib << 16) | (cc.fnib << 8) | d.fnib;
    sR[c] = a.rnib | (b.rnib << 8) | (cc.rnib << 16) | (d.rnib << 24);
    sINV[c] = (uint16_t)(a.inv | (b.inv << 4) | (cc.inv << 8) | (d.inv << 12));
    if (!CANON) sRAW[c] = v;
  }
  if (tid < 2) { sF[kChunks + tid] = 0; sR[kChunks + tid] = 0; }
  if (tid < 4) sINV[kChunks + tid] = 0;
  for (int i = tid; i < kTile / 32; i += kBlock) sWIN[i] = 0;

  uint64_t *tbl_idx = dyn;
  uint32_t *tbl_slot = reinterpret_cast<uint32_t *>(dyn + (MODE == 1 ? u.tbl_size : 0));
  if (MODE == 1) build_top_tbl(u, tbl_idx, tbl_slot);  // contains __syncthreads
  __syncthreads();

  // 2. windows crossing a record boundary (or running past the end) are not k-mers
  {
    const uint64_t limit = T0 + kTile + (uint64_t)k - 1;
    const uint64_t r0 = in.tile_rec[blockIdx.x];
    for (uint64_t r = r0 + 1 + tid; r <= in.n_recs; r += kBlock) {
      uint64_t b = in.offsets[r];
      if (b >= limit) break;
      uint64_t lo = (b + 1 > (uint64_t)k) ? b + 1 - (uint64_t)k : 0;
      if (lo < T0) lo = T0;
      uint64_t hi = b < T0 + kTile ? b : T0 + kTile;
      for (uint64_t q = lo - T0; q < hi - T0;) {  // <= 2 words for k <= 32
        uint32_t w = (uint32_t)(q >> 5), s = (uint32_t)(q & 31);
        uint32_t nb = (uint32_t)((hi - T0) - q);
        uint32_t take = nb < 32 - s ? nb : 32 - s;
        uint32_t bits = (take == 32 ? 0xFFFFFFFFu : ((1u << take) - 1u)) << s;
        atomicOr(&sWIN[w], bits);
        q += take;
      }
    }
  }
  __syncthreads();

  const int twok = 2 * k;
  const uint64_t mask2k = (k >= 32) ? ~0ULL : ((1ULL << twok) - 1ULL);
  const uint32_t kmask = (k >= 32) ? 0xFFFFFFFFu : ((1u << k) - 1u);

#pragma unroll 4
  for (int j = 0; j < kPerThread; ++j) {
    const int q = j * kBlock + tid;
    const uint64_t p = T0 + (uint64_t)q;
    if (p + (uint64_t)k > n_bases) break;
    if ((sWIN[q >> 5] >> (q & 31)) & 1u) continue;
    const int w = q >> 4;
    const int s = 2 * (q & 15);
    uint64_t hi64 = ((uint64_t)sF[w] << 32) | sF[w + 1];
    uint64_t x = (hi64 << s) | (((uint64_t)sF[w + 2] << s) >> 32);
    uint64_t fwd = x >> (64 - twok);
    uint64_t key;
    if (CANON) {
      uint64_t lo64 = ((uint64_t)sR[w + 1] << 32) | sR[w];
      uint64_t y = (lo64 >> s) | (((uint64_t)sR[w + 2] << 32) << (32 - s));
      uint64_t rev = y & mask2k;
      key = fwd < rev ? fwd : rev;
    } else {
      // pack_kmer skips non-ACGT bytes (src/utils.rs:26-39)
      const int iw = q >> 4;  // 16 bits per sINV entry
      const int is = q & 15;
      uint64_t z = ((uint64_t)sINV[iw] | ((uint64_t)sINV[iw + 1] << 16) |
                    ((uint64_t)sINV[iw + 2] << 32) | ((uint64_t)sINV[iw + 3] << 48)) >> is;
      if ((uint32_t)z & kmask) {
        const uint8_t *raw = reinterpret_cast<const uint8_t *>(sRAW);
        uint64_t pk = 0;
        for (int i = 0; i < k; ++i) {
          uint8_t bb = raw[q + i];
          if (valid_byte(bb)) pk = (pk << 2) | code_of(bb);
        }
        key = pk;
      } else {
        key = fwd;
      }
    }
    const uint64_t idx = fastmod(sip13_u64(key), fm);
    if (MODE == 0) {
      atomicAdd(&currents[idx], 1ULL);
    } else {
      int slot = probe_top(tbl_idx, tbl_slot, u.tbl_size - 1, idx);
      if (slot >= 0) set_insert(u, (uint32_t)slot, key);
    }
  }
}

// ---------------------------------------------------------------------------
// K1c: k > 32, the reference's release-build u64 semantics, lane per position.
//   forward  = last 32 bases of the window (mask !0, power 0: models.rs:188,192)
//   reverse  = (rev_init >> 2j) | OR_{u<=min(j-1, sh/2)} comp(b[p+k-1-u]) << (sh-2u)
//              with j = p - record_start, sh = (2(k-1)) & 63 (masked shl, :265)
//              and rev_init = complement codes of the record's first 32 bases.
// ---------------------------------------------------------------------------
template <bool CANON, int MODE>
__global__ __launch_bounds__(kBlock) void k_kmers_compat(KmerInput in, int k, FastMod fm,
                                                         unsigned long long *__restrict__ currents,
                                                         UniqArgs u) {
  extern __shared__ uint64_t dyn[];
  uint64_t *tbl_idx = dyn;
  uint32_t *tbl_slot = reinterpret_cast<uint32_t *>(dyn + (MODE == 1 ? u.tbl_size : 0));
  if (MODE == 1) build_top_tbl(u, tbl_idx, tbl_slot);

  const uint64_t T0 = (uint64_t)blockIdx.x * kTile;
  const uint32_t sh = (uint32_t)((2 * (k - 1)) & 63);
  uint64_t r = in.tile_rec[blockIdx.x];
  for (int j = 0; j < kPerThread; ++j) {
    const uint64_t p = T0 + (uint64_t)j * kBlock + threadIdx.x;
    if (p >= in.n_bases) break;
    while (r + 1 < in.n_recs && in.offsets[r + 1] <= p) ++r;
    const uint64_t s0 = in.offsets[r], e0 = in.offsets[r + 1];
    if (p < s0 || p + (uint64_t)k > e0) continue;
    const uint8_t *b = in.bases;
    uint64_t key;
    if (CANON) {
      uint64_t fwd = 0;
      for (int i = 0; i < 32; ++i) fwd = (fwd << 2) | code_of(b[p + k - 32 + i]);
      const uint64_t jj = p - s0;
      uint64_t rev = 0;
      if (jj < 32) {
        uint64_t ri = 0;
        for (int i = 31; i >= 0; --i) ri = (ri << 2) | comp_of(b[s0 + i]);
        rev = ri >> (2 * jj);
      }
      uint64_t umax = sh / 2;
      if (jj >= 1 && jj - 1 < umax) umax = jj - 1;
      if (jj >= 1)
        for (uint64_t uu = 0; uu <= umax; ++uu)
          rev |= (uint64_t)comp_of(b[p + k - 1 - uu]) << (sh - 2 * uu);
      key = fwd < rev ? fwd : rev;
    } else {
      uint64_t pk = 0;
      for (int i = 0; i < k; ++i) {
        uint8_t bb = b[p + i];
        if (valid_byte(bb)) pk = (pk << 2) | code_of(bb);
      }
      key = pk;
    }
    const uint64_t idx = fastmod(sip13_u64(key), fm);
    if (MODE == 0) {
      atomicAdd(&currents[idx], 1ULL);
    } else {
      int slot = probe_top(tbl_idx, tbl_slot, u.tbl_size - 1, idx);
      if (slot >= 0) set_insert(u, (uint32_t)slot, key);
    }
  }
}

// ---------------------------------------------------------------------------
// K3: LIF
// ---------------------------------------------------------------------------
__global__ void k_lif_table(LifEntry *__restrict__ tbl, int n, LifParams lp) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float v = 0.0f;
  uint32_t r = 0;
  float c = lif_current((uint64_t)i, lp.steps);
  uint64_t sp = lif_closed(c, lp.steps, lp.thr, lp.leak, lp.refr, v, r);
  tbl[i].spikes = sp;
  tbl[i].v = v;
  tbl[i].r = r;
}

constexpr int kLifPerThread = 8;

__global__ __launch_bounds__(kBlock) void k_lif_apply(const uint64_t *__restrict__ currents,
                                                      float *__restrict__ V,
                                                      uint32_t *__restrict__ R,
                                                      uint64_t *__restrict__ SC, uint64_t pool,
                                                      LifParams lp,
                                                      const LifEntry *__restrict__ tbl, int tbl_n,
                                                      uint32_t *__restrict__ hist,
                                                      unsigned long long *__restrict__ stats) {
  __shared__ uint32_t sh[kHistBins];
  __shared__ unsigned long long s_sp[kBlock / 64];
  __shared__ unsigned long long s_mx[kBlock / 64];
  for (int i = threadIdx.x; i < kHistBins; i += kBlock) sh[i] = 0;
  __syncthreads();
  const uint64_t base = (uint64_t)blockIdx.x * kBlock * kLifPerThread;
  unsigned long long my_sp = 0, my_mx = 0;
  for (int j = 0; j < kLifPerThread; ++j) {
    uint64_t i = base + (uint64_t)j * kBlock + threadIdx.x;
    if (i >= pool) break;
    uint64_t cnt = currents[i];
    uint64_t sc = SC[i];
    if (!(lp.skip_zero && cnt == 0) && lp.steps != 0) {
      float v = V[i];
      uint32_t r = R[i];
      uint64_t sp;
      if (v == 0.0f && r == 0 && cnt < (uint64_t)tbl_n) {
        const LifEntry e = tbl[cnt];
        sp = e.spikes;
        v = e.v;
        r = e.r;
      } else {
        sp = lif_closed(lif_current(cnt, lp.steps), lp.steps, lp.thr, lp.leak, lp.refr, v, r);
      }
      V[i] = v;
      R[i] = r;
      sc += sp;
      SC[i] = sc;
      my_sp += sp;
    }
    my_mx = sc > my_mx ? sc : my_mx;
    atomicAdd(&sh[sc < (uint64_t)(kHistBins - 1) ? (uint32_t)sc : (uint32_t)(kHistBins - 1)], 1u);
  }
  // wave reductions
  for (int o = 32; o > 0; o >>= 1) {
    my_sp += __shfl_down(my_sp, o, 64);
    unsigned long long om = __shfl_down(my_mx, o, 64);
    my_mx = om > my_mx ? om : my_mx;
  }
  if ((threadIdx.x & 63) == 0) { s_sp[threadIdx.x >> 6] = my_sp; s_mx[threadIdx.x >> 6] = my_mx; }
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long a = 0, m = 0;
    for (int w = 0; w < kBlock / 64; ++w) { a += s_sp[w]; m = s_mx[w] > m ? s_mx[w] : m; }
    if (a) atomicAdd(&stats[0], a);
    atomicMax(&stats[1], m);
  }
  for (int i = threadIdx.x; i < kHistBins; i += kBlock)
    if (sh[i]) atomicAdd(&hist[i], sh[i]);
}

// ---------------------------------------------------------------------------
// K4: top-N
// ---------------------------------------------------------------------------
// Finds T = spike count of the N-th row from the 4096-bin histogram
// (bin = min(spikes, 4095)).  One block of 1024 threads, 4 bins each.
__global__ __launch_bounds__(1024) void k_topn_threshold(const uint32_t *__restrict__ hist,
                                                         uint64_t n, uint64_t pool,
                                                         TopState *__restrict__ st) {
  __shared__ unsigned long long part[1024];
  const int t = threadIdx.x;
  // thread t owns bins [4095-4t-3, 4095-4t] i.e. counting from the top
  unsigned long long loc = 0;
  for (int j = 0; j < 4; ++j) loc += hist[kHistBins - 1 - (4 * t + j)];
  part[t] = loc;
  __syncthreads();
  // inclusive scan over threads (Hillis-Steele; 10 steps)
  for (int o = 1; o < 1024; o <<= 1) {
    unsigned long long v = t >= o ? part[t - o] : 0ull;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  const unsigned long long want = n < pool ? n : pool;
  unsigned long long before = t ? part[t - 1] : 0ull;  // rows in higher bins
  if (want == 0) {
    if (t == 0) { st->T = ~0ULL; st->n_above = 0; st->need = 0; st->emit_above = 0; st->refine = 0; }
    return;
  }
  if (before < want && part[t] >= want) {
    unsigned long long cum = before;
    for (int j = 0; j < 4; ++j) {
      int bin = kHistBins - 1 - (4 * t + j);
      unsigned long long h = hist[bin];
      if (cum + h >= want) {
        st->T = (uint64_t)bin;
        st->n_above = cum;
        st->need = want - cum;
        st->emit_above = 0;
        st->refine = (bin == kHistBins - 1) ? 1u : 0u;
        break;
      }
      cum += h;
    }
  }
}

// 256-bin histogram of digit (sc >> shift) & 255 over neurons whose higher bits
// equal `prefix` (radix refine for spike counts >= 4095; rare path).
__global__ __launch_bounds__(kBlock) void k_radix_hist(const uint64_t *__restrict__ sc, uint64_t pool,
                                                       int shift, uint64_t prefix,
                                                       uint32_t *__restrict__ h256) {
  __shared__ uint32_t sh[256];
  sh[threadIdx.x] = 0;
  __syncthreads();
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < pool;
       i += (uint64_t)gridDim.x * kBlock) {
    uint64_t v = sc[i];
    uint64_t hi = (shift + 8 >= 64) ? 0 : (v >> (shift + 8));
    if (hi == prefix) atomicAdd(&sh[(v >> shift) & 255], 1u);
  }
  __syncthreads();
  if (sh[threadIdx.x]) atomicAdd(&h256[threadIdx.x], sh[threadIdx.x]);
}

constexpr int kTopChunk = kBlock * 8;  // neurons per block in count/emit

__global__ __launch_bounds__(kBlock) void k_topn_count(const uint64_t *__restrict__ sc,
                                                       uint64_t pool,
                                                       const TopState *__restrict__ st,
                                                       uint32_t *__restrict__ tie_cnt) {
  __shared__ uint32_t s[kBlock / 64];
  const uint64_t T = st->T;
  const uint64_t base = (uint64_t)blockIdx.x * kTopChunk;
  uint32_t c = 0;
  for (int j = 0; j < 8; ++j) {
    uint64_t i = base + (uint64_t)j * kBlock + threadIdx.x;
    if (i < pool && sc[i] == T) ++c;
  }
  for (int o = 32; o > 0; o >>= 1) c += __shfl_down(c, o, 64);
  if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) tie_cnt[blockIdx.x] = s[0] + s[1] + s[2] + s[3];
}

__global__ __launch_bounds__(kBlock) void k_topn_emit(const uint64_t *__restrict__ sc,
                                                      uint64_t pool, TopState *__restrict__ st,
                                                      const uint32_t *__restrict__ tie_cnt,
                                                      TopCand *__restrict__ cand) {
  __shared__ unsigned long long s_pre[kBlock / 64];
  __shared__ uint32_t s_scan[kBlock];
  const uint64_t T = st->T, need = st->need, n_above = st->n_above;
  // ties in earlier blocks
  unsigned long long pre = 0;
  for (uint32_t b = threadIdx.x; b < blockIdx.x; b += kBlock) pre += tie_cnt[b];
  for (int o = 32; o > 0; o >>= 1) pre += __shfl_down(pre, o, 64);
  if ((threadIdx.x & 63) == 0) s_pre[threadIdx.x >> 6] = pre;
  __syncthreads();
  const unsigned long long prefix = s_pre[0] + s_pre[1] + s_pre[2] + s_pre[3];
  // thread t owns 8 consecutive neurons -> ranks in index order
  const uint64_t base = (uint64_t)blockIdx.x * kTopChunk + (uint64_t)threadIdx.x * 8;
  uint32_t ties = 0;
  uint64_t v[8];
  for (int j = 0; j < 8; ++j) {
    uint64_t i = base + j;
    v[j] = i < pool ? sc[i] : 0;
    if (i < pool && v[j] == T) ++ties;
    if (i < pool && v[j] > T && T != ~0ULL) {
      unsigned long long pos = atomicAdd((unsigned long long *)&st->emit_above, 1ull);
      cand[pos].idx = i;
      cand[pos].sc = v[j];
    }
  }
  if (prefix >= need) return;  // uniform across the block
  s_scan[threadIdx.x] = ties;
  __syncthreads();
  for (int o = 1; o < kBlock; o <<= 1) {
    uint32_t a = threadIdx.x >= (unsigned)o ? s_scan[threadIdx.x - o] : 0;
    __syncthreads();
    s_scan[threadIdx.x] += a;
    __syncthreads();
  }
  uint64_t rank = prefix + s_scan[threadIdx.x] - ties;
  for (int j = 0; j < 8; ++j) {
    uint64_t i = base + j;
    if (i < pool && v[j] == T) {
      if (rank < need) {
        cand[n_above + rank].idx = i;
        cand[n_above + rank].sc = T;
      }
      ++rank;
    }
  }
}

__device__ __forceinline__ bool cand_before(const TopCand &a, const TopCand &b) {
  return a.sc != b.sc ? a.sc > b.sc : a.idx < b.idx;
}

// exact final order of the <= kMaxTopN candidates: bitonic sort in LDS
__global__ __launch_bounds__(1024) void k_topn_sort(TopCand *__restrict__ cand, uint32_t m,
                                                    const uint64_t *__restrict__ currents,
                                                    uint64_t *__restrict__ top_cur) {
  __shared__ TopCand s[kMaxTopN];
  uint32_t n2 = 1;
  while (n2 < m) n2 <<= 1;
  for (uint32_t i = threadIdx.x; i < n2; i += blockDim.x) {
    if (i < m) s[i] = cand[i];
    else { s[i].sc = 0; s[i].idx = ~0ULL; }  // sorts last
  }
  __syncthreads();
  for (uint32_t size = 2; size <= n2; size <<= 1) {
    for (uint32_t stride = size >> 1; stride > 0; stride >>= 1) {
      for (uint32_t i = threadIdx.x; i < n2; i += blockDim.x) {
        uint32_t jj = i ^ stride;
        if (jj > i) {
          bool up = (i & size) == 0;
          TopCand a = s[i], b = s[jj];
          bool swap = up ? cand_before(b, a) : cand_before(a, b);
          if (swap) { s[i] = b; s[jj] = a; }
        }
      }
      __syncthreads();
    }
  }
  for (uint32_t i = threadIdx.x; i < m; i += blockDim.x) {
    cand[i] = s[i];
    top_cur[i] = currents[s[i].idx];
  }
}

// ---------------------------------------------------------------------------
// device hash set helpers (uniques of the top-N neurons)
// ---------------------------------------------------------------------------
__global__ void k_set_fill(unsigned long long *__restrict__ keys, uint64_t cap) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < cap;
       i += (uint64_t)gridDim.x * blockDim.x)
    keys[i] = kEmpty;
}

__global__ void k_set_compact(const unsigned long long *__restrict__ keys, uint64_t cap,
                              const uint32_t *__restrict__ special, uint32_t n_top,
                              uint64_t *__restrict__ out, unsigned long long *__restrict__ count) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < cap;
       i += (uint64_t)gridDim.x * blockDim.x) {
    unsigned long long kk = keys[i];
    if (kk != kEmpty) out[atomicAdd(count, 1ull)] = kk;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    bool any = false;
    for (uint32_t s = 0; s < n_top; ++s) any |= special[s] != 0;
    if (any) out[atomicAdd(count, 1ull)] = kEmpty;
  }
}

__global__ void k_set_merge(const uint64_t *__restrict__ keys, uint64_t n, FastMod fm, UniqArgs u) {
  extern __shared__ uint64_t dyn[];
  uint64_t *tbl_idx = dyn;
  uint32_t *tbl_slot = reinterpret_cast<uint32_t *>(dyn + u.tbl_size);
  build_top_tbl(u, tbl_idx, tbl_slot);
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t key = keys[i];
    uint64_t idx = fastmod(sip13_u64(key), fm);
    int slot = probe_top(tbl_idx, tbl_slot, u.tbl_size - 1, idx);
    if (slot >= 0) set_insert(u, (uint32_t)slot, key);
  }
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
static FastMod make_fastmod(uint64_t p) {
  FastMod f;
  f.p = p;
  f.magic = p ? (~0ULL) / p : 0;
  return f;
}

uint64_t n_tiles_for(uint64_t n_bases) { return (n_bases + kTile - 1) / kTile; }

uint64_t top_tbl_size(uint32_t n_top) {
  uint64_t s = 64;
  while (s < 2ull * n_top) s <<= 1;
  return s;
}

static size_t tbl_bytes(const UniqArgs &u) { return (size_t)u.tbl_size * (8 + 4); }

hipError_t launch_tile_rec(const KmerInput &in, uint32_t *tile_rec, hipStream_t s) {
  if (!in.n_tiles) return hipSuccess;
  unsigned g = (unsigned)((in.n_tiles + 255) / 256);
  hipLaunchKernelGGL(k_tile_rec, dim3(g), dim3(256), 0, s, in.offsets, in.n_recs, in.n_tiles,
                     tile_rec);
  return hipGetLastError();
}

template <int MODE>
static hipError_t launch_kmers(const KmerInput &in, int k, int canonical, uint64_t pool,
                               unsigned long long *cur, const UniqArgs &u, hipStream_t s) {
  if (!in.n_tiles) return hipSuccess;
  FastMod fm = make_fastmod(pool);
  dim3 g((unsigned)in.n_tiles), b(kBlock);
  size_t dyn = MODE == 1 ? tbl_bytes(u) : 0;
  if (k <= 32) {
    if (canonical) hipLaunchKernelGGL((k_kmers<true, MODE>), g, b, dyn, s, in, k, fm, cur, u);
    else hipLaunchKernelGGL((k_kmers<false, MODE>), g, b, dyn, s, in, k, fm, cur, u);
  } else {
    if (canonical) hipLaunchKernelGGL((k_kmers_compat<true, MODE>), g, b, dyn, s, in, k, fm, cur, u);
    else hipLaunchKernelGGL((k_kmers_compat<false, MODE>), g, b, dyn, s, in, k, fm, cur, u);
  }
  return hipGetLastError();
}

hipError_t launch_count(const KmerInput &in, int k, int canonical, uint64_t pool,
                        uint64_t *currents, hipStream_t s) {
  UniqArgs u{};
  return launch_kmers<0>(in, k, canonical, pool, (unsigned long long *)currents, u, s);
}

hipError_t launch_uniques(const KmerInput &in, int k, int canonical, uint64_t pool,
                          const UniqArgs &u, hipStream_t s) {
  return launch_kmers<1>(in, k, canonical, pool, nullptr, u, s);
}

hipError_t launch_lif_table(LifEntry *tbl, int n, LifParams lp, hipStream_t s) {
  hipLaunchKernelGGL(k_lif_table, dim3((n + 255) / 256), dim3(256), 0, s, tbl, n, lp);
  return hipGetLastError();
}

hipError_t launch_lif_apply(const uint64_t *currents, float *v, uint32_t *r, uint64_t *sc,
                            uint64_t pool, LifParams lp, const LifEntry *tbl, int tbl_n,
                            uint32_t *hist, uint64_t *stats, hipStream_t s) {
  if (!pool) return hipSuccess;
  uint64_t per = (uint64_t)kBlock * kLifPerThread;
  unsigned g = (unsigned)((pool + per - 1) / per);
  hipLaunchKernelGGL(k_lif_apply, dim3(g), dim3(kBlock), 0, s, currents, v, r, sc, pool, lp, tbl,
                     tbl_n, hist, (unsigned long long *)stats);
  return hipGetLastError();
}

hipError_t launch_topn_threshold(const uint32_t *hist, uint64_t n, uint64_t pool, TopState *st,
                                 hipStream_t s) {
  hipLaunchKernelGGL(k_topn_threshold, dim3(1), dim3(1024), 0, s, hist, n, pool, st);
  return hipGetLastError();
}

hipError_t launch_radix_hist(const uint64_t *sc, uint64_t pool, int shift, uint64_t prefix,
                             uint32_t *h256, hipStream_t s) {
  unsigned g = (unsigned)((pool + kBlock * 8 - 1) / (kBlock * 8));
  if (g > 2048) g = 2048;
  if (!g) g = 1;
  hipLaunchKernelGGL(k_radix_hist, dim3(g), dim3(kBlock), 0, s, sc, pool, shift, prefix, h256);
  return hipGetLastError();
}

static unsigned topn_blocks(uint64_t pool) {
  return (unsigned)((pool + kTopChunk - 1) / kTopChunk);
}

hipError_t launch_topn_count(const uint64_t *sc, uint64_t pool, const TopState *st,
                             uint32_t *tie_cnt, hipStream_t s) {
  if (!pool) return hipSuccess;
  hipLaunchKernelGGL(k_topn_count, dim3(topn_blocks(pool)), dim3(kBlock), 0, s, sc, pool, st,
                     tie_cnt);
  return hipGetLastError();
}

hipError_t launch_topn_emit(const uint64_t *sc, uint64_t pool, TopState *st,
                            const uint32_t *tie_cnt, TopCand *cand, hipStream_t s) {
  if (!pool) return hipSuccess;
  hipLaunchKernelGGL(k_topn_emit, dim3(topn_blocks(pool)), dim3(kBlock), 0, s, sc, pool, st,
                     tie_cnt, cand);
  return hipGetLastError();
}

hipError_t launch_topn_sort(TopCand *cand, uint32_t m, const uint64_t *currents,
                            uint64_t *top_cur, hipStream_t s) {
  if (!m) return hipSuccess;
  hipLaunchKernelGGL(k_topn_sort, dim3(1), dim3(1024), 0, s, cand, m, currents, top_cur);
  return hipGetLastError();
}

hipError_t launch_set_fill(unsigned long long *keys, uint64_t cap, hipStream_t s) {
  unsigned g = (unsigned)((cap + 255) / 256);
  if (g > 4096) g = 4096;
  if (!g) return hipSuccess;
  hipLaunchKernelGGL(k_set_fill, dim3(g), dim3(256), 0, s, keys, cap);
  return hipGetLastError();
}

hipError_t launch_set_compact(const unsigned long long *keys, uint64_t cap, const uint32_t *special,
                              uint32_t n_top, const TopCand *, uint64_t, uint64_t *out,
                              unsigned long long *count, hipStream_t s) {
  unsigned g = (unsigned)((cap + 255) / 256);
  if (g > 4096) g = 4096;
  if (!g) g = 1;
  hipLaunchKernelGGL(k_set_compact, dim3(g), dim3(256), 0, s, keys, cap, special, n_top, out,
                     count);
  return hipGetLastError();
}

hipError_t launch_set_merge(const uint64_t *keys, uint64_t n, uint64_t pool, const UniqArgs &u,
                            hipStream_t s) {
  if (!n) return hipSuccess;
  unsigned g = (unsigned)((n + 255) / 256);
  if (g > 2048) g = 2048;
  hipLaunchKernelGGL(k_set_merge, dim3(g), dim3(256), tbl_bytes(u), s, keys, n,
                     make_fastmod(pool), u);
  return hipGetLastError();
}

}  // namespace nk
