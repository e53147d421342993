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
#include <stdlib.h>

#include <algorithm>
#include <type_traits>

#include "nk_device.h"
#include "nk_gen.h"
#include "nk_kernels.h"
#include "nk_tile.h"
#include "nk_post.h"

namespace nk {

constexpr int kPerThread = kTile / kBlock;      // 16 positions per lane
constexpr unsigned long long kEmpty = ~0ULL;

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}

// ---------------------------------------------------------------------------
// first record of each tile: largest r < n_recs with offsets[r] <= tile start
// ---------------------------------------------------------------------------
__global__ void k_tile_rec(const uint64_t *__restrict__ offsets, uint64_t n_recs,
                           uint64_t n_tiles, uint64_t tile_size, uint64_t tile_base,
                           uint32_t *__restrict__ tile_rec) {
  uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n_tiles) return;
  uint64_t pos = (tile_base + t) * tile_size;
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
// Per-workgroup filter in front of the global set: a key this workgroup has
// already inserted is dropped in LDS.  Hot neurons (repeats) otherwise send
// thousands of identical inserts to one global slot, which serialise at the
// memory side.  Returns true when the key was seen before by this workgroup.
constexpr int kSeen = 1024;
__device__ __forceinline__ void seen_init(unsigned long long *seen) {
  for (int i = threadIdx.x; i < kSeen; i += blockDim.x) seen[i] = kEmpty;
}
__device__ __forceinline__ bool seen_before(unsigned long long *seen, uint64_t key) {
  uint32_t h = (uint32_t)mix64(key) & (kSeen - 1);
  for (int probe = 0; probe < 16; ++probe) {
    unsigned long long v = seen[h];
    if (v == key) return true;
    if (v == kEmpty) {
      unsigned long long prev = atomicCAS(&seen[h], kEmpty, (unsigned long long)key);
      if (prev == kEmpty) return false;
      if (prev == key) return true;
    }
    h = (h + 1) & (kSeen - 1);
  }
  return false;  // table crowded: let the global set decide
}

__device__ __forceinline__ void set_insert(const UniqArgs &u, uint32_t slot, uint64_t key) {
  if (key == kEmpty) {
    if (atomicCAS(&u.special[slot], 0u, 1u) == 0u) atomicAdd(&u.uniq[slot], 1u);
    return;
  }
  const uint64_t mask = *u.set_mask;
  uint64_t h = mix64(key) & mask;
  for (;;) {
    // read first: repeated k-mers (the hot neurons) find their key without
    // serialising on one address; a stale kEmpty only costs an extra CAS
    unsigned long long cur = __hip_atomic_load(&u.set_keys[h], __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT);
    if (cur == key) return;
    if (cur == kEmpty) {
      unsigned long long prev = atomicCAS(&u.set_keys[h], kEmpty, (unsigned long long)key);
      if (prev == kEmpty) {
        atomicAdd(&u.uniq[slot], 1u);
        if (u.xdst) {
          const unsigned long long at = atomicAdd(u.xn, 1ull);
          if (at < u.xcap) u.xdst[1 + at] = key;
        }
        return;
      }
      if (prev == key) return;
    }
    h = (h + 1) & mask;
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
  // parallel insertion (the top rows are distinct neurons): one global load
  // per thread instead of n_top dependent loads on one thread
  const uint32_t mask = u.tbl_size - 1;
  for (uint32_t s = threadIdx.x; s < u.n_top; s += blockDim.x) {
    const uint64_t idx = u.top[s].idx;
    uint32_t h = (uint32_t)idx & mask;
    while (atomicCAS(reinterpret_cast<unsigned long long *>(&tbl_idx[h]), (unsigned long long)kEmpty,
                     (unsigned long long)idx) != (unsigned long long)kEmpty)
      h = (h + 1) & mask;
    tbl_slot[h] = s;
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
  __shared__ TileLds<kTile, !CANON> L;
  __shared__ unsigned long long seen[MODE == 1 ? kSeen : 1];
  extern __shared__ uint64_t dyn[];  // MODE 1: probe table
  uint64_t *tbl_idx = dyn;
  uint32_t *tbl_slot = reinterpret_cast<uint32_t *>(dyn + (MODE == 1 ? u.tbl_size : 0));
  if (MODE == 1) {
    seen_init(seen);
    build_top_tbl(u, tbl_idx, tbl_slot);  // contains __syncthreads
  }
  const uint64_t tile = in.tile_base + blockIdx.x;
  const uint64_t T0 = tile * kTile;
  stage_tile<kTile, kBlock, !CANON>(L, in, tile, k);
#pragma unroll 4
  for (int j = 0; j < kPerThread; ++j) {
    const int q = j * kBlock + threadIdx.x;
    if (T0 + (uint64_t)q + (uint64_t)k > in.n_bases) break;
    if (!window_valid(L, T0, q, k, in.n_bases, in.pos_lo, in.pos_hi)) continue;
    const uint64_t key = window_key<kTile, !CANON, CANON>(L, q, k);
    const uint64_t idx = fastmod(sip13_u64(key), fm);
    if (MODE == 0) {
      atomicAdd(&currents[idx], 1ULL);
    } else {
      int slot = probe_top(tbl_idx, tbl_slot, u.tbl_size - 1, idx);
      if (slot >= 0 && (key == kEmpty || !seen_before(seen, key))) set_insert(u, (uint32_t)slot, key);
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
  __shared__ unsigned long long seen[MODE == 1 ? kSeen : 1];
  uint64_t *tbl_idx = dyn;
  uint32_t *tbl_slot = reinterpret_cast<uint32_t *>(dyn + (MODE == 1 ? u.tbl_size : 0));
  if (MODE == 1) {
    seen_init(seen);
    build_top_tbl(u, tbl_idx, tbl_slot);
  }

  const uint64_t T0 = (in.tile_base + blockIdx.x) * kTile;
  uint64_t r = in.tile_rec[blockIdx.x];
  for (int j = 0; j < kPerThread; ++j) {
    const uint64_t p = T0 + (uint64_t)j * kBlock + threadIdx.x;
    if (p >= in.n_bases) break;
    if (p < in.pos_lo || p >= in.pos_hi) continue;
    while (r + 1 < in.n_recs && in.offsets[r + 1] <= p) ++r;
    const uint64_t s0 = in.offsets[r], e0 = in.offsets[r + 1];
    if (p < s0 || p + (uint64_t)k > e0) continue;
    const uint64_t key = compat_key<CANON>(in.bases, s0, p, k);
    const uint64_t idx = fastmod(sip13_u64(key), fm);
    if (MODE == 0) {
      atomicAdd(&currents[idx], 1ULL);
    } else {
      int slot = probe_top(tbl_idx, tbl_slot, u.tbl_size - 1, idx);
      if (slot >= 0 && (key == kEmpty || !seen_before(seen, key))) set_insert(u, (uint32_t)slot, key);
    }
  }
}

// ---------------------------------------------------------------------------
// --kmer-width=128 (k <= 64): count (MODE 0: global atomics) and uniques of the
// top rows (MODE 1) over u128 keys.
//
// The uniques set holds a key as three 43-bit chunks in u64 words whose bit
// 63 marks the word written.  Word 0 is claimed by CAS; a lane that matches
// word 0 of a slot another lane is still publishing polls again on its next
// loop iteration (never spins inside one), so no store ordering, fence or
// intra-wave wait is needed, and distinct keys are counted exactly.
// ---------------------------------------------------------------------------
constexpr uint64_t kW128Valid = 1ull << 63;
constexpr uint64_t kW128Mask = (1ull << 43) - 1;
__device__ __forceinline__ void key128_words(const Key128 &k, uint64_t w[3]) {
  w[0] = (k.lo & kW128Mask) | kW128Valid;
  w[1] = (((k.lo >> 43) | (k.hi << 21)) & kW128Mask) | kW128Valid;
  w[2] = (k.hi >> 22) | kW128Valid;
}
__device__ __forceinline__ Key128 words_key128(uint64_t w0, uint64_t w1, uint64_t w2) {
  Key128 k;
  w0 &= kW128Mask;
  w1 &= kW128Mask;
  w2 &= ~kW128Valid;
  k.lo = w0 | (w1 << 43);
  k.hi = (w1 >> 21) | (w2 << 22);
  return k;
}
__device__ __forceinline__ void set_insert128(const UniqArgs &u, uint32_t slot, const Key128 &key) {
  uint64_t w[3];
  key128_words(key, w);
  const uint64_t mask = *u.set_mask;
  unsigned long long *S = u.set_keys;  // 3 words per slot
  uint64_t h = mix64(key.lo ^ mix64(key.hi)) & mask;
  for (;;) {
    unsigned long long cur = __hip_atomic_load(&S[3 * h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (cur == 0) {
      const unsigned long long prev = atomicCAS(&S[3 * h], 0ull, (unsigned long long)w[0]);
      if (prev == 0) {
        __hip_atomic_store(&S[3 * h + 1], (unsigned long long)w[1], __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&S[3 * h + 2], (unsigned long long)w[2], __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
        atomicAdd(&u.uniq[slot], 1u);
        if (u.xdst) {
          const unsigned long long at = atomicAdd(u.xn, 1ull);
          if (at < u.xcap) {
            u.xdst[1 + 2 * at] = key.lo;
            u.xdst[2 + 2 * at] = key.hi;
          }
        }
        return;
      }
      cur = prev;
    }
    if (cur == w[0]) {
      const unsigned long long a =
          __hip_atomic_load(&S[3 * h + 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned long long b =
          __hip_atomic_load(&S[3 * h + 2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (!(a & kW128Valid) || !(b & kW128Valid)) continue;  // being published: poll again
      if (a == w[1] && b == w[2]) return;
    }
    h = (h + 1) & mask;
  }
}

template <bool CANON, int MODE>
__global__ __launch_bounds__(kBlock) void k_kmers128(KmerInput in, int k, FastMod fm,
                                                     unsigned long long *__restrict__ currents,
                                                     UniqArgs u) {
  __shared__ TileLds<kTile, !CANON> L;
  extern __shared__ uint64_t dyn[];  // MODE 1: probe table
  uint64_t *tbl_idx = dyn;
  uint32_t *tbl_slot = reinterpret_cast<uint32_t *>(dyn + (MODE == 1 ? u.tbl_size : 0));
  if (MODE == 1) build_top_tbl(u, tbl_idx, tbl_slot);  // contains __syncthreads
  const uint64_t tile = in.tile_base + blockIdx.x;
  const uint64_t T0 = tile * kTile;
  stage_tile<kTile, kBlock, !CANON>(L, in, tile, k);
#pragma unroll 2
  for (int j = 0; j < kPerThread; ++j) {
    const int q = j * kBlock + threadIdx.x;
    if (T0 + (uint64_t)q + (uint64_t)k > in.n_bases) break;
    if (!window_valid(L, T0, q, k, in.n_bases, in.pos_lo, in.pos_hi)) continue;
    const Key128 key = window_key128<kTile, !CANON, CANON>(L, q, k);
    const uint64_t idx = fastmod(sip13_u128(key.lo, key.hi), fm);
    if (MODE == 0) {
      atomicAdd(&currents[idx], 1ULL);
    } else {
      const int slot = probe_top(tbl_idx, tbl_slot, u.tbl_size - 1, idx);
      if (slot >= 0) set_insert128(u, (uint32_t)slot, key);
    }
  }
}

// Uniques rescan for the generic count paths (nk_wide.hip: k > 32 compat,
// 128-bit keys, pools past the narrow partition): the same 8192-position
// tiles and LDS keys as k_part_gen; a window whose neuron is a top row goes
// into the uniques set.
template <int KM, bool CANON>
__global__ __launch_bounds__(kPartBlock) void k_uniq_gen(KmerInput in, int k, FastMod fm,
                                                         UniqArgs u, const uint32_t *__restrict__ tiles,
                                                         const uint32_t *__restrict__ n_list) {
  // with a tile list: workgroup i takes the i-th listed tile (uniform exit past it)
  if (tiles && blockIdx.x >= *n_list) return;
  constexpr bool kRaw = !CANON;
  __shared__ TileLds<kPartTile, kRaw> L;
  __shared__ unsigned long long seen[KM == 2 ? 1 : kSeen];
  extern __shared__ uint64_t dyn[];  // probe table
  uint64_t *tbl_idx = dyn;
  uint32_t *tbl_slot = reinterpret_cast<uint32_t *>(dyn + u.tbl_size);
  if (KM != 2) seen_init(seen);
  build_top_tbl(u, tbl_idx, tbl_slot);  // contains __syncthreads
  const uint64_t tile = tiles ? (uint64_t)tiles[blockIdx.x] : in.tile_base + blockIdx.x;
  const uint64_t T0 = tile * (uint64_t)kPartTile;
  stage_tile<kPartTile, kPartBlock, kRaw>(L, in, tile, k);
  const int q0 = threadIdx.x * kPer;
  RecCursor rc;
  rec_cursor_init<KM>(rc, in, T0 + (uint64_t)q0, tile - in.tile_base);  // (listed tile: not blockIdx)
  for (int j = 0; j < kPer; ++j) {
    const int q = q0 + j;
    if (!window_valid(L, T0, q, k, in.n_bases, in.pos_lo, in.pos_hi)) continue;
    const Key128 key = gen_key<KM, CANON>(L, in, q, T0 + (uint64_t)q, k, rc);
    const uint64_t idx = fastmod(gen_hash<KM>(key), fm);
    const int slot = probe_top(tbl_idx, tbl_slot, u.tbl_size - 1, idx);
    if (slot < 0) continue;
    if (KM == 2) set_insert128(u, (uint32_t)slot, key);
    else if (key.lo == kEmpty || !seen_before(seen, key.lo)) set_insert(u, (uint32_t)slot, key.lo);
  }
}

// Uniques of the lane-tagged wide records: entry (tile << 9 | lane) of the
// list k_uniq_tiles built is one k_part_gen lane that produced a top row's
// record; its kPer windows are keyed without staging a tile: canonical keys
// (KM 0 / 2) roll through the lane's kPer + k - 1 bytes (five 16-B loads into
// the thread's LDS slot), the rest are keyed per window from global memory.
// Hashed; those of top rows go into the set.  Grid-stride over the
// device-side list length.
constexpr int kLaneBytes = 80;  // kPer + 64 - 1 rounded up to 16 B
template <int KM, bool CANON>
__global__ __launch_bounds__(256) void k_uniq_lanes(KmerInput in, int k, FastMod fm, UniqArgs u,
                                                    const uint32_t *__restrict__ list,
                                                    const uint32_t *__restrict__ n_list,
                                                    uint32_t max_list) {
  extern __shared__ uint64_t dyn[];  // probe table
  __shared__ uint4 s_b[256 * (kLaneBytes / 16)];
  uint64_t *tbl_idx = dyn;
  uint32_t *tbl_slot = reinterpret_cast<uint32_t *>(dyn + u.tbl_size);
  build_top_tbl(u, tbl_idx, tbl_slot);  // contains __syncthreads
  constexpr bool kRoll = CANON && KM != 1;
  uint4 *mine = s_b + threadIdx.x * (kLaneBytes / 16);
  const uint8_t *bb = reinterpret_cast<const uint8_t *>(mine);
  const int sh = 2 * k - 2;
  const uint32_t n = *n_list < max_list ? *n_list : max_list;
  for (uint32_t e = blockIdx.x * blockDim.x + threadIdx.x; e < n; e += gridDim.x * blockDim.x) {
    const uint32_t ent = list[e];
    const uint64_t tile = ent >> 9;
    const uint64_t p0 = tile * (uint64_t)kPartTile + (uint64_t)(ent & 511u) * kPer;
    const bool roll = kRoll && p0 + kLaneBytes <= in.n_bases;
    if (roll) {
#pragma unroll
      for (int c = 0; c < kLaneBytes / 16; ++c)
        mine[c] = *reinterpret_cast<const uint4 *>(in.bases + p0 + 16 * c);
    }
    Key128 fwd{0, 0}, rev{0, 0};
    auto push = [&](uint8_t x) {  // one base into both rolling keys (2k bits)
      const uint64_t c = code_of(x), r = comp_of(x);
      fwd.hi = (fwd.hi << 2) | (fwd.lo >> 62);
      fwd.lo = (fwd.lo << 2) | c;
      if (k < 32) {
        fwd.lo &= (1ull << (2 * k)) - 1ull;
        fwd.hi = 0;
      } else if (k < 64) {
        fwd.hi &= (1ull << (2 * k - 64)) - 1ull;
      }
      rev.lo = (rev.lo >> 2) | (rev.hi << 62);
      rev.hi >>= 2;
      if (sh >= 64) rev.hi |= r << (sh - 64);
      else rev.lo |= r << sh;
    };
    if (roll)
      for (int i = 0; i < k - 1; ++i) push(bb[i]);
    // the record holding p0 (windows must end inside their record)
    uint64_t r = in.n_recs ? rec_of(in.offsets, in.n_recs, in.tile_rec[tile], p0) : 0;
    for (int j = 0; j < kPer; ++j) {
      const uint64_t p = p0 + (uint64_t)j;
      if (roll) push(bb[j + k - 1]);
      if (p + (uint64_t)k > in.n_bases || p < in.pos_lo || p >= in.pos_hi) continue;
      while (r + 1 < in.n_recs && in.offsets[r + 1] <= p) ++r;
      if (!in.n_recs || p + (uint64_t)k > in.offsets[r + 1]) continue;  // crosses a record end
      Key128 key{0, 0};
      if (roll) key = key128_less(rev, fwd) ? rev : fwd;
      else if (KM == 2) key = global_window_key128<CANON>(in.bases, p, k);
      else if (KM == 1) key.lo = compat_key<CANON>(in.bases, in.offsets[r], p, k);
      else key.lo = global_window_key<CANON>(in.bases, p, k);
      const uint64_t idx = fastmod(gen_hash<KM>(key), fm);
      const int slot = probe_top(tbl_idx, tbl_slot, u.tbl_size - 1, idx);
      if (slot < 0) continue;
      if (KM == 2) set_insert128(u, (uint32_t)slot, key);
      else set_insert(u, (uint32_t)slot, key.lo);
    }
  }
}

__global__ void k_set_fill128(unsigned long long *__restrict__ S, const uint64_t *__restrict__ mask) {
  const uint64_t n = 3 * (*mask + 1);
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x)
    S[i] = 0;
}

// the set's keys as (lo, hi) pairs
__global__ void k_set_compact128(const unsigned long long *__restrict__ S, uint64_t cap,
                                 uint64_t *__restrict__ out, unsigned long long *__restrict__ count) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < cap;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const unsigned long long w0 = S[3 * i];
    if (!w0) continue;
    const Key128 k = words_key128(w0, S[3 * i + 1], S[3 * i + 2]);
    const unsigned long long at = atomicAdd(count, 1ull);
    out[2 * at] = k.lo;
    out[2 * at + 1] = k.hi;
  }
}

// the union of several ranks' top k-mers ((lo, hi) pairs) into the set
// Keys to merge: a flat list (world == 0), or `world` rank segments of a
// fixed-stride all-gather buffer, each [n_r, key 0, key 1, ...] with at most
// cap keys stored (a larger n_r sets *trunc: the caller falls back to the
// variable-length exchange).  wpk: u64 words per key (2 for 128-bit keys).
__device__ __forceinline__ bool merge_src_key(const MergeSrc &m, uint64_t i, int wpk,
                                              const uint64_t **at) {
  if (!m.world) {
    *at = m.keys + (uint64_t)wpk * i;
    return true;
  }
  const uint64_t r = i / m.cap, j = i - r * m.cap;
  const uint64_t *seg = m.keys + r * m.stride;
  const uint64_t nr = seg[0] & ((1ull << 56) - 1);
  if (j == 0) {
    const uint32_t why = (nr > m.cap ? 1u : 0u) | (uint32_t)(seg[0] >> 56) << 1;
    if (why) atomicOr(m.trunc, why);
  }
  if (j >= nr) return false;
  *at = seg + 1 + (uint64_t)wpk * j;
  return true;
}

__global__ void k_set_merge128(MergeSrc m, FastMod fm, UniqArgs u) {
  extern __shared__ uint64_t dyn[];
  uint64_t *tbl_idx = dyn;
  uint32_t *tbl_slot = reinterpret_cast<uint32_t *>(dyn + u.tbl_size);
  build_top_tbl(u, tbl_idx, tbl_slot);
  const uint64_t n = m.world ? (uint64_t)m.world * m.cap : m.n;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t *at;
    if (!merge_src_key(m, i, 2, &at)) continue;
    const Key128 key{at[0], at[1]};
    const uint64_t idx = fastmod(sip13_u128(key.lo, key.hi), fm);
    const int slot = probe_top(tbl_idx, tbl_slot, u.tbl_size - 1, idx);
    if (slot >= 0) set_insert128(u, (uint32_t)slot, key);
  }
}

// ---------------------------------------------------------------------------
// K1 partitioned (k <= 32, pool <= kMaxBuckets * 32768): the MI355X-native count.
//
// Random per-k-mer global atomics run at the memory side (~20 G/s chip-wide),
// 10x below what the hash rate allows.  Instead:
//   K1a k_part     hash every k-mer of an 8192-position tile, counting-sort the
//                  tile's (bin offset u16, tile position u16) records by bucket
//                  (bucket = neuron >> 15) in LDS, reserve room in each bucket's
//                  HBM array with ONE atomic per (tile, bucket), and write the
//                  segments out as 16-B stores: each segment is padded to a
//                  multiple of 8 records with the sentinel bin kPadOff.
//   K1b k_bucket_hist  one workgroup per (bucket, slice): 32768-bin u32
//                  histogram in LDS over a contiguous slice of the bucket's
//                  records, written once as a partial.
//   K1c k_partials_add currents[i] += sum of the partials (u64).
// The records are kept: the uniques pass reads only the top neurons' buckets
// instead of re-hashing the input.
// ---------------------------------------------------------------------------
constexpr int kPartPerThread = kPartTile / kPartBlock;  // 16
constexpr uint32_t kPadOff = 0xFFFFu;                    // sentinel bin of a pad record
// MAXB: bucket capacity of the launch (256 for pools <= 8.4 M, 512 up to
// 16.7 M).  The store groups are 8 records of one bucket (the reservations
// are multiples of 8).  MAXB 256: the LDS sort area holds the tile plus the
// worst-case padding, so every group is 16-B aligned there too.  MAXB 512
// (UNPAD): the sort area holds the tile's 8192 records only and a group's
// pad records are made at store time -- 14 KB less LDS (64.5 -> 50.6 KB), so
// three workgroups share a CU instead of two (config 3's pool, 16 M).
template <int MAXB>
struct PartShape {
  static constexpr bool kUnpad = MAXB > 256;
  static constexpr int kPadded = kPartTile + 7 * MAXB;     // records + worst-case padding
  static constexpr int kSortSlots = kUnpad ? kPartTile + 8 : kPadded;
  static constexpr int kGroups = kPadded / 8;              // 8-record store groups
  static constexpr int kGroupIters = (kGroups + kPartBlock - 1) / kPartBlock;
  using GMap = typename std::conditional<(MAXB > 256), uint16_t, uint8_t>::type;
};

#if defined(NK_ABL_STAMPS)  // ablation build: per-workgroup phase timestamps
__device__ unsigned long long g_stamps[1 << 18];
#define NK_STAMP(I)                                                              \
  do {                                                                           \
    if (threadIdx.x == 0 && blockIdx.x < (1u << 14))                             \
      g_stamps[blockIdx.x * 16 + (I)] = (I) == 0 || (I) == 7                     \
          ? __builtin_amdgcn_s_memrealtime() : __builtin_amdgcn_s_memtime();    \
  } while (0)
#else
#define NK_STAMP(I) do {} while (0)
#endif
// A launch-uniform value moved into a VGPR: a VALU instruction that reads an
// SGPR operand issues at half rate on gfx950 (tools/isabench.hip: v_xor with an
// SGPR 4.15 clk vs 2.35 with a literal or VGPR), so the per-k-mer loop reads its
// masks, shift and dummy bucket from VGPRs.
__device__ __forceinline__ uint32_t in_vgpr(uint32_t x) {
#if defined(NK_K1A_VUNI)
  uint32_t v;
  asm("v_mov_b32 %0, %1" : "=v"(v) : "s"(x));
  return v;
#else
  return x;
#endif
}

constexpr uint32_t kSpanTail = 2048;  // last-dispatched workgroups that stamp the span's end

// K16: k >= 16, so the low word of the window mask is all ones.
// KEYS (the exact table, nk_table.hip): each record's key is re-extracted from
// the staged tile at store time and written beside its bin offset (pa.key);
// the position array is not written.  Records past a full region are counted
// directly as always (pa.currents, when set) and their keys spilled.
// LDS of one K1a tile (k_part; in a union with the fused histogram item, k_part_fused)
template <int MAXB, bool RAW>
struct PartLds {
  using S = PartShape<MAXB>;
  TileLds<kPartTile, RAW> L;
  uint32_t s_cnt[MAXB + 1];  // + a dummy bucket for non-k-mer positions
  uint32_t s_start[MAXB + 1];  // padded (groups, reservations)
  uint32_t s_ustart[PartShape<MAXB>::kUnpad ? MAXB + 1 : 1];  // unpadded (the LDS sort)
  uint32_t s_base[MAXB];
  uint32_t s_fit[MAXB];
  __align__(16) uint32_t s_sorted[S::kSortSlots];
  typename S::GMap s_gmap[S::kGroups];  // store group -> bucket
};

template <bool CANON, int MAXB, bool K16, bool KEYS>
__device__ __forceinline__ void part_tile(const KmerInput &in, int k, const FastMod &fm,
                                          const PartArgs &pa, PartLds<MAXB, !CANON> &sm) {
  using S = PartShape<MAXB>;
  constexpr int kSortSlots = S::kSortSlots;
  constexpr int kGroupIters = S::kGroupIters;
  TileLds<kPartTile, !CANON> &L = sm.L;
  uint32_t(&s_cnt)[MAXB + 1] = sm.s_cnt;
  uint32_t(&s_start)[MAXB + 1] = sm.s_start;
  constexpr bool kUnpad = S::kUnpad;
  uint32_t *s_ustart = sm.s_ustart;
  uint32_t(&s_base)[MAXB] = sm.s_base;
  uint32_t(&s_fit)[MAXB] = sm.s_fit;
  uint32_t(&s_sorted)[kSortSlots] = sm.s_sorted;
  typename S::GMap(&s_gmap)[S::kGroups] = sm.s_gmap;

  const int tid = threadIdx.x;
  const uint64_t tile = in.tile_base + blockIdx.x;
  const uint64_t T0 = tile * (uint64_t)kPartTile;
  const uint32_t B = pa.n_buckets;
  NK_STAMP(0);
  NK_STAMP(8);
  // the launch's span (nk_count_spans): its first workgroups start it, its
  // last-dispatched workgroups end it (workgroups run for about the same time
  // and are dispatched in index order, so no earlier one ends last); stamping
  // every workgroup (an end barrier + two global atomics each) cost the step
  // ~5 us (profiles/r02_s15)
  if (pa.span && tid == 0 && blockIdx.x < 8u)
    atomicMin(pa.span, (unsigned long long)__builtin_amdgcn_s_memrealtime());
  for (uint32_t b = tid; b <= B; b += kPartBlock) s_cnt[b] = 0;
  stage_tile<kPartTile, kPartBlock, !CANON, !CANON>(L, in, tile, k);  // syncs (INV: pack_kmer only)
  NK_STAMP(2);
#if defined(NK_ABL_STAGEONLY)  // ablation: staging only
  if (L.F[tid] == 0x12345678u && tid == 1000000) pa.overflow[0] = 1u;
  return;
#endif

  // phase 1: this lane's 16 consecutive positions q0..q0+15.  The first
  // window is extracted from the bit streams, the next 15 are rolled in from
  // two 32-bit code words (forward MSB-first, complement LSB-first), exactly
  // the reference's slide for k <= 32 (src/models.rs:254-269).  The body is
  // branch-free: a position that starts no k-mer goes to a dummy bucket.
  const int q0 = tid * kPartPerThread;
  const uint64_t rem = in.n_bases - T0;  // >= 1
  const uint64_t nrange = rem >= (uint64_t)k ? rem - (uint64_t)k + 1 : 0;
  uint32_t ok = ~(L.WIN[q0 >> 5] >> (q0 & 31)) & 0xFFFFu;
  if (nrange < (uint64_t)q0 + kPartPerThread)
    ok &= nrange > (uint64_t)q0 ? (1u << (uint32_t)(nrange - q0)) - 1u : 0u;
  {  // chunked input: only windows starting in [pos_lo, pos_hi) (uniform per launch)
    const uint64_t p0 = T0 + (uint64_t)q0;
    if (in.pos_lo > p0) ok &= in.pos_lo - p0 >= 16 ? 0u : ~((1u << (uint32_t)(in.pos_lo - p0)) - 1u);
    if (in.pos_hi < p0 + kPartPerThread)
      ok &= in.pos_hi > p0 ? (1u << (uint32_t)(in.pos_hi - p0)) - 1u : 0u;
  }
  const int twok = 2 * k;
  const uint64_t mask2k = (k >= 32) ? ~0ULL : ((1ULL << twok) - 1ULL);
  uint64_t fwd, rev;
  {
    const int w = q0 >> 4;  // q0 is 16-aligned: shift 0
    const uint64_t x = ((uint64_t)L.F[w] << 32) | L.F[w + 1];
    fwd = x >> (64 - twok);
    rev = (((uint64_t)L.R[w + 1] << 32) | L.R[w]) & mask2k;
  }
  uint32_t inF, inR;  // codes of the 15 bases rolled in: positions q0+k .. q0+k+14
  {
    const int s0 = q0 + k;
    const int w = s0 >> 4, sh = 2 * (s0 & 15);
    inF = (uint32_t)(((((uint64_t)L.F[w] << 32) | L.F[w + 1]) << sh) >> 32);
    inR = (uint32_t)((((uint64_t)L.R[w + 1] << 32) | L.R[w]) >> sh);
  }
  uint64_t invz = 0;  // non-canonical: invalid-byte bits of positions q0 .. q0+47
  if (!CANON) {
    const int iw = q0 >> 4;
    invz = (uint64_t)L.INV[iw] | ((uint64_t)L.INV[iw + 1] << 16) | ((uint64_t)L.INV[iw + 2] << 32);
  }
  const uint32_t kmask = (k >= 32) ? 0xFFFFFFFFu : ((1u << k) - 1u);
  const uint32_t bbits = in_vgpr(pa.bin_bits), bmask = in_vgpr((1u << pa.bin_bits) - 1u);
  const uint32_t Bv = in_vgpr(B), pv = in_vgpr((uint32_t)fm.p);
  uint32_t E[kPartPerThread];  // bucket << 16 | rank
  uint32_t O[kPartPerThread];  // bin offset within the bucket
  // Window j as a funnel shift of two 96-bit words (no serial roll):
  //   fwd_j = ({fwd_0, inF} >> (32 - 2j)) & mask2k
  //   rev_j = ((inR << 2k | rev_0) >> 2j) & mask2k
  // two v_alignbit + two v_and per strand and position (the serial
  // fwd = fwd << 2 | c, rev = rev >> 2 | cc << (2k - 2) roll is 1 % slower
  // in an A/B, K1a 0.4212 vs 0.4245-0.4268 ms).
  const uint32_t g0 = inF, g1 = (uint32_t)fwd, g2 = (uint32_t)(fwd >> 32);
  const unsigned __int128 X = ((unsigned __int128)inR << twok) | rev;
  const uint32_t x0 = (uint32_t)X, x1 = (uint32_t)(X >> 32), x2 = (uint32_t)(X >> 64);
  const uint32_t mlo = in_vgpr((uint32_t)mask2k), mhi = in_vgpr((uint32_t)(mask2k >> 32));
#pragma unroll
  for (int j = 0; j < kPartPerThread; ++j) {
    if (j) {
      const uint32_t flo = __builtin_amdgcn_alignbit(g1, g0, 32 - 2 * j);
      const uint32_t rlo = __builtin_amdgcn_alignbit(x1, x0, 2 * j);
      fwd = ((uint64_t)(__builtin_amdgcn_alignbit(g2, g1, 32 - 2 * j) & mhi) << 32) |
            (K16 ? flo : flo & mlo);
      rev = ((uint64_t)(__builtin_amdgcn_alignbit(x2, x1, 2 * j) & mhi) << 32) |
            (K16 ? rlo : rlo & mlo);
    }
    uint64_t key;
    if (CANON) {
      key = fwd < rev ? fwd : rev;
    } else {
      key = fwd;
      if (((uint32_t)(invz >> j)) & kmask) {  // pack_kmer skips non-ACGT bytes (rare)
        const uint8_t *raw = reinterpret_cast<const uint8_t *>(L.RAWB);
        uint64_t pk = 0;
        for (int i = 0; i < k; ++i) {
          const uint8_t bb = raw[q0 + j + i];
          if (valid_byte(bb)) pk = (pk << 2) | code_of(bb);
        }
        key = pk;
      }
    }
#if defined(NK_ABL_NOHASH)  // ablation builds only (tools/ablate_k1a.sh): hash -> identity
    const uint32_t idx = fastmod32(key, fm);
#else
    const uint32_t idx = fastmod32_p(sip13_u64(key), fm, pv);
#endif
    const uint32_t b = ((ok >> j) & 1u) ? (idx >> bbits) : Bv;
#if defined(NK_ABL_NORANK)  // ablation: no LDS rank atomic (records collide; timing only)
    const uint32_t rank = (uint32_t)j;
    if (tid == 0 && j == 0) atomicAdd(&s_cnt[b], 1u);
#else
    const uint32_t rank = atomicAdd(&s_cnt[b], 1u);
#endif
    E[j] = (b << 16) | rank;
    O[j] = idx & bmask;
  }
  __syncthreads();
  NK_STAMP(3);
#if defined(NK_ABL_NOSORT)  // ablation: stop after the hash + rank phase
  if (tid == 0) pa.overflow[0] = s_cnt[0] == 0x7FFFFFFFu;
  if (E[0] == 0xFFFFFFFFu || O[kPartPerThread - 1] == 0xFFFFFFFFu) pa.overflow[1] = 1u;
  return;
#endif
  // exclusive scan of the padded bucket counts (one wave) + HBM reservation
  // (one atomic per non-empty bucket: entries in the low 40 bits, segments
  // above).  Reservations are multiples of 8 records, so every segment starts
  // 16-B aligned in the bucket array (cap is a multiple of 64).
  if (tid < 64) {
    uint32_t carry = 0;
    for (uint32_t b0 = 0; b0 < B; b0 += 64) {
      uint32_t b = b0 + tid;
      uint32_t c = b < B ? (s_cnt[b] + 7u) & ~7u : 0;
      uint32_t x = c;
      for (int o = 1; o < 64; o <<= 1) {
        uint32_t y = __shfl_up(x, o, 64);
        if (tid >= o) x += y;
      }
      if (b < B) s_start[b] = carry + x - c;
      carry += __shfl(x, 63, 64);
    }
    if (tid == 0) s_start[B] = carry;
  } else if (kUnpad && tid < 128) {  // the unpadded starts (the dummy bucket B last), wave 1
    const uint32_t l = tid - 64;
    uint32_t carry = 0;
    for (uint32_t b0 = 0; b0 <= B; b0 += 64) {
      uint32_t b = b0 + l;
      uint32_t c = b <= B ? s_cnt[b] : 0;
      uint32_t x = c;
      for (int o = 1; o < 64; o <<= 1) {
        uint32_t y = __shfl_up(x, o, 64);
        if (l >= (uint32_t)o) x += y;
      }
      if (b <= B) s_ustart[b] = carry + x - c;
      carry += __shfl(x, 63, 64);
    }
  }
  // this tile's sub-region: its XCD in a one-launch count (workgroup i runs on
  // XCD i mod 8); by the tile, not the workgroup, so that the many small
  // launches of a chunked count (file ingest) still fill the eight evenly
  // (block 0 of every launch went to sub-region 0)
  const uint32_t xs = (uint32_t)tile & ((1u << pa.sub_shift) - 1u);
  for (uint32_t b = tid; b < B; b += kPartBlock) {
    const uint32_t c = (s_cnt[b] + 7u) & ~7u;
    uint32_t fit = 0, base = 0;
    if (c) {
      const uint64_t v = ((uint64_t)b << pa.sub_shift) | xs;
      unsigned long long ret = atomicAdd(&pa.fill[v], (unsigned long long)c | (1ull << 40));
      uint64_t eb = ret & ((1ull << 40) - 1);
      uint64_t seg = ret >> 40;
#if !defined(NK_ABL_NODESC)  // ablation: no descriptor writes (the uniques break; traffic only)
      if (seg < pa.max_segs)
        pa.desc[v * pa.max_segs + seg] = make_uint2((uint32_t)tile, (uint32_t)eb);
#endif
      fit = eb >= pa.cap ? 0u : (uint32_t)(pa.cap - eb < c ? pa.cap - eb : c);
      // past the region, or past the descriptor table (chunked input: a tile can
      // add a segment per launch): the uniques of this bucket fall back to a rescan
      if (fit < c || (seg >= pa.max_segs && (!KEYS || pa.desc))) pa.overflow[b] = 1u;
      base = (uint32_t)(xs * pa.cap + eb);  // from the bucket's first sub-region
    }
    s_base[b] = base;
    s_fit[b] = fit;
  }
  __syncthreads();
  NK_STAMP(4);
  // phase 2: counting-sort the records in LDS (positions that start no k-mer
  // land in the dummy bucket's region after the last group and are dropped);
  // one thread per bucket writes its pad records and its group map entries
  {
    uint32_t st[kPartPerThread];
#pragma unroll
    for (int j = 0; j < kPartPerThread; ++j) st[j] = kUnpad ? s_ustart[E[j] >> 16] : s_start[E[j] >> 16];
#pragma unroll
    for (int j = 0; j < kPartPerThread; ++j)
      s_sorted[st[j] + (E[j] & 0xFFFFu)] = O[j] | ((uint32_t)(q0 + j) << 16);
  }
  for (uint32_t b = tid; b < B; b += kPartBlock) {
    const uint32_t c = s_cnt[b], st = s_start[b], cp = (c + 7u) & ~7u;
    if (!kUnpad)
      for (uint32_t i = c; i < cp; ++i) s_sorted[st + i] = 0xFFFFFFFFu;
    for (uint32_t g = st >> 3; g < (st + cp) >> 3; ++g) s_gmap[g] = (typename S::GMap)b;
  }
  __syncthreads();
  NK_STAMP(5);
  // phase 3: each thread moves 8-record groups -> one 16-B store into the
  // offset array and one into the position array
  const uint32_t n_groups = s_start[B] >> 3;
#pragma unroll
  for (int it = 0; it < kGroupIters; ++it) {
    const uint32_t g = (uint32_t)tid + (uint32_t)it * kPartBlock;
    if (g >= n_groups) break;
    const uint32_t b = s_gmap[g];
    const uint32_t j8 = g * 8 - s_start[b];
    uint4 w0, w1;
    if (kUnpad) {  // the group's records from the unpadded sort, its pads made here
      const uint32_t src = s_ustart[b] + j8, c = s_cnt[b];
      uint32_t w[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) w[i] = j8 + (uint32_t)i < c ? s_sorted[src + i] : 0xFFFFFFFFu;
      w0 = make_uint4(w[0], w[1], w[2], w[3]);
      w1 = make_uint4(w[4], w[5], w[6], w[7]);
    } else {
      w0 = *reinterpret_cast<const uint4 *>(&s_sorted[g * 8]);
      w1 = *reinterpret_cast<const uint4 *>(&s_sorted[g * 8 + 4]);
    }
#if defined(NK_ABL_NOWRITE)  // ablation: LDS sort kept, no HBM record stores
    if (w0.x == 0x12345678u && w1.w == 0x9ABCDEF0u) pa.overflow[b] = 1u;
    continue;
#endif
    if (j8 < s_fit[b]) {
      const uint64_t dst = ((uint64_t)b << pa.sub_shift) * pa.cap + s_base[b] + j8;
      // v_perm: bytes {lo16(a), lo16(b)} and {hi16(a), hi16(b)}
      const uint4 off = make_uint4(__builtin_amdgcn_perm(w0.y, w0.x, 0x05040100u),
                                   __builtin_amdgcn_perm(w0.w, w0.z, 0x05040100u),
                                   __builtin_amdgcn_perm(w1.y, w1.x, 0x05040100u),
                                   __builtin_amdgcn_perm(w1.w, w1.z, 0x05040100u));
      const uint4 pos = make_uint4(__builtin_amdgcn_perm(w0.y, w0.x, 0x07060302u),
                                   __builtin_amdgcn_perm(w0.w, w0.z, 0x07060302u),
                                   __builtin_amdgcn_perm(w1.y, w1.x, 0x07060302u),
                                   __builtin_amdgcn_perm(w1.w, w1.z, 0x07060302u));
      // nontemporal: the records are read once, by K1b, from HBM (A/B: K1a
      // 0.4177-0.4179 vs 0.4205-0.4217 ms with plain stores)
      typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
      // (plain stores instead wrote as much at pool 16 M, also with the
      // sub-regions per XCD: profiles/r05_l, r05_p)
#if defined(NK_K1A_OFF_PLAIN)  // A/B: the offsets K1b reads next kept in the caches (MALL)
      *reinterpret_cast<u32x4 *>(pa.off + dst) = u32x4{off.x, off.y, off.z, off.w};
#else
      __builtin_nontemporal_store(u32x4{off.x, off.y, off.z, off.w}, reinterpret_cast<u32x4 *>(pa.off + dst));
#endif
      if (!KEYS)
        __builtin_nontemporal_store(u32x4{pos.x, pos.y, pos.z, pos.w}, reinterpret_cast<u32x4 *>(pa.pos + dst));
      if constexpr (KEYS) {
        if (pa.pos)  // the count's arena: positions kept for a multi-GPU uniques pass
          __builtin_nontemporal_store(u32x4{pos.x, pos.y, pos.z, pos.w}, reinterpret_cast<u32x4 *>(pa.pos + dst));
        const uint32_t w[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
        uint64_t kk[8];
#pragma unroll
        for (int i = 0; i < 8; ++i)
          kk[i] = (w[i] & 0xFFFFu) != kPadOff ? window_key<kPartTile, !CANON, CANON>(L, (int)(w[i] >> 16), k)
                                               : 0ull;
        // plain stores: a lane's 64 B are four 16-B stores 64 B apart across
        // the wave, completed in L2 (nontemporal ones left partial lines:
        // K1a<KEYS> 1.2 ms vs 0.40, profiles/r03_t2)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          reinterpret_cast<ulonglong2 *>(pa.key + dst)[i] = make_ulonglong2(kk[2 * i], kk[2 * i + 1]);
      }
    } else {  // bucket region full: count directly (correct, slow, rare)
      const uint32_t w[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
      for (int i = 0; i < 8; ++i) {
        if ((w[i] & 0xFFFFu) == kPadOff) continue;
        if (!KEYS || pa.currents)
          atomicAdd(&pa.currents[((uint64_t)b << pa.bin_bits) | (w[i] & 0xFFFFu)], 1ULL);
        if constexpr (KEYS) {  // the table takes this bucket from the side list
          const unsigned long long at = atomicAdd(pa.n_spill, 1ull);
          if (at < pa.spill_cap)
            pa.spill[at] = window_key<kPartTile, !CANON, CANON>(L, (int)(w[i] >> 16), k);
        }
      }
    }
  }
  if (pa.span && blockIdx.x + kSpanTail >= gridDim.x) {  // its last stores are issued: end time
    __syncthreads();
    if (tid == 0) atomicMax(pa.span + 1, (unsigned long long)__builtin_amdgcn_s_memrealtime());
  }
#if defined(NK_ABL_STAMPS)
  __syncthreads();
  NK_STAMP(6);
  if (threadIdx.x == 0 && blockIdx.x < (1u << 14)) {
    unsigned hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    unsigned xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    g_stamps[blockIdx.x * 16 + 1] = ((unsigned long long)xcc << 32) | hw;
  }
  NK_STAMP(7);
#endif
}

template <bool CANON, int MAXB, bool K16 = false, bool KEYS = false>
__global__ __launch_bounds__(kPartBlock) void k_part(KmerInput in, int k, FastMod fm, PartArgs pa) {
  __shared__ PartLds<MAXB, !CANON> sm;
  part_tile<CANON, MAXB, K16, KEYS>(in, k, fm, pa, sm);
}

// Spikes of a neuron in the derived state: the LIF from (v, r) = (0, 0) of
// its count (k_lif_apply's fresh branch).
__device__ __forceinline__ uint64_t fresh_spikes(uint64_t cnt, const LifParams &lp,
                                                 const LifEntry *tbl, int tbl_n, float &v,
                                                 uint32_t &r) {
  v = 0.0f;
  r = 0u;
  if ((lp.skip_zero && cnt == 0) || lp.steps == 0) return 0;
  if (cnt < (uint64_t)tbl_n) {
    const LifEntry e = tbl[cnt];
    v = e.v;
    r = e.r;
    return e.spikes;
  }
  return lif_closed(lif_current(cnt, lp.steps), lp.steps, lp.thr, lp.leak, lp.refr, v, r);
}

// partials == nullptr: add the histogram into pa.currents instead (u64; plain
// read-modify-write of the bins this workgroup owns when slices == 1, atomics
// otherwise; bins that stayed zero are not touched)
#ifndef NK_HIST_KU
#define NK_HIST_KU 4
#endif
constexpr int kK1bLifLds = 1024;  // counts whose fresh spikes the write-through K1b keeps in LDS
// (u32 in LDS: every spike count fits below 2^32 steps)
__device__ __forceinline__ int k1b_lds_entries(const K1bLif &L) {
  return L.lp.steps >= (1ull << 32) ? 0 : L.tbl_n < kK1bLifLds ? L.tbl_n : kK1bLifLds;
}
// LIF: the write-through K1b also runs the LIF from the reset state (pa.lif).
// (Measured and not kept, profiles/r04_s15: the bins and the spike histogram
// as packed u16 pairs, 78 KB of LDS, two workgroups per CU -- equal.)
template <int BB, int KU = NK_HIST_KU, bool LIF = false>  // 2^BB bins per bucket (pa.bin_bits)
__global__ __launch_bounds__(kHistBlock) void k_bucket_hist(PartArgs pa, uint64_t pool,
                                                            uint32_t slices,
                                                            uint32_t *__restrict__ partials) {
  constexpr uint32_t kBins = 1u << BB;
  __shared__ uint32_t h[kBins + 1];  // + a spill bin for pad records
  __shared__ uint32_t s_sh[LIF ? kHistBins : 1];  // spike histogram of the bucket
  __shared__ uint32_t s_tsp[LIF ? kK1bLifLds : 1];  // spikes of the small counts (pa.lif.tbl)
  __shared__ unsigned long long s_acc[2];
  const uint32_t b = blockIdx.x, r = blockIdx.y;  // buckets on x: up to 65536 of them
  for (int i = threadIdx.x; i <= (int)kBins; i += kHistBlock) h[i] = 0;
  if (LIF) {
    for (int i = threadIdx.x; i < kHistBins; i += kHistBlock) s_sh[i] = 0;
    if (threadIdx.x < 2) s_acc[threadIdx.x] = 0;
    // the write-through's LIF reads these instead of a dependent global load
    // per bin (fresh_spikes: tbl[count])
    for (int i = threadIdx.x; i < k1b_lds_entries(pa.lif); i += kHistBlock)
      s_tsp[i] = (uint32_t)pa.lif.tbl[i].spikes;
  }
  auto bin = [](uint32_t off) { return off < kBins ? off : kBins; };
  __syncthreads();
  // the bucket's records: its sub-regions' (pa.sub_shift) in order, this
  // slice's share [lo, hi) of them
  const uint32_t nsub = 1u << pa.sub_shift;
  uint64_t n = 0;
  for (uint32_t x = 0; x < nsub; ++x) {
    const uint64_t f = pa.fill[((uint64_t)b << pa.sub_shift) | x] & ((1ull << 40) - 1);
    n += f < pa.cap ? f : pa.cap;
  }
  const uint64_t lo_all = n * r / slices, hi_all = n * (r + 1) / slices;
  uint64_t c0 = 0;
  for (uint32_t x = 0; x < nsub; ++x) {
    const uint64_t vb = ((uint64_t)b << pa.sub_shift) | x;
    uint64_t nv = pa.fill[vb] & ((1ull << 40) - 1);
    if (nv > pa.cap) nv = pa.cap;
    const uint64_t a = lo_all > c0 ? lo_all : c0, z = hi_all < c0 + nv ? hi_all : c0 + nv;
    const uint64_t lo = a - c0, hi = z > a ? z - c0 : lo;  // (uniform) this sub-region's part
    c0 += nv;
    if (lo >= hi) continue;
    const uint16_t *src = pa.off + vb * pa.cap;
    // 8 records (16 B) per lane per step where aligned
    uint64_t i = lo;
    for (; i < hi && (i & 7); ++i)
      if (threadIdx.x == 0) atomicAdd(&h[bin(src[i])], 1u);
    const uint64_t hi8 = i + ((hi - i) & ~7ull);
    const uint64_t step = 8ull * kHistBlock;
    // NK_HIST_KU 16-B loads per lane per round, software-pipelined: the next
    // round's loads are in flight while this round's 8*KU LDS atomics issue.
    // Loads past hi8 are clamped to a valid address (static wait counts) and
    // their records skipped, so there is no serial tail of single loads.
    auto hist8 = [&](const uint4 &v) {
      atomicAdd(&h[bin(v.x & 0xFFFFu)], 1u); atomicAdd(&h[bin(v.x >> 16)], 1u);
      atomicAdd(&h[bin(v.y & 0xFFFFu)], 1u); atomicAdd(&h[bin(v.y >> 16)], 1u);
      atomicAdd(&h[bin(v.z & 0xFFFFu)], 1u); atomicAdd(&h[bin(v.z >> 16)], 1u);
      atomicAdd(&h[bin(v.w & 0xFFFFu)], 1u); atomicAdd(&h[bin(v.w >> 16)], 1u);
    };
    uint64_t j = i + 8ull * threadIdx.x;
    if (j < hi8) {
      auto load_round = [&](uint64_t jb, uint4 *v) {
#pragma unroll
        for (int t = 0; t < KU; ++t) {
          const uint64_t jt = jb + (uint64_t)t * step;
          // nontemporal: each record is read once (A/B: step 0.561 vs 0.575-0.578 ms)
          typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
          const u32x4 q = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(src + (jt < hi8 ? jt : i)));
          v[t] = make_uint4(q.x, q.y, q.z, q.w);
        }
      };
      uint4 cur[KU];
      load_round(j, cur);
      for (;;) {
        const uint64_t jn = j + (uint64_t)KU * step;
        const bool more = jn < hi8;
        uint4 nxt[KU];
        load_round(more ? jn : j, nxt);
#pragma unroll
        for (int t = 0; t < KU; ++t)
          if (j + (uint64_t)t * step < hi8) hist8(cur[t]);
        if (!more) break;
        j = jn;
#pragma unroll
        for (int t = 0; t < KU; ++t) cur[t] = nxt[t];
      }
    }
    for (uint64_t j = hi8 + threadIdx.x; j < hi; j += kHistBlock) atomicAdd(&h[bin(src[j])], 1u);
  }  // sub-regions
  __syncthreads();
  const uint64_t nb0 = (uint64_t)b << BB;
  const uint64_t nbins = pool - nb0 < (uint64_t)kBins ? pool - nb0 : kBins;
  if (!partials && pa.out) {  // write-through: every bin, the overflow target folded + re-zeroed
    const bool ov = pa.overflow[b] || (pa.over_coarse && pa.over_coarse[b >> pa.coarse_shift]);
    unsigned long long *o = pa.out + nb0, *ovf = pa.currents + nb0;
    auto count = [&](uint32_t t) -> unsigned long long {
      unsigned long long x = h[t];
      if (ov) {
        const unsigned long long e = ovf[t];
        if (e) {
          x += e;
          ovf[t] = 0;
        }
      }
      return x;
    };
    if (!LIF) {
      for (uint32_t t = threadIdx.x; t < nbins; t += kHistBlock) o[t] = count(t);
      return;
    }
    // fused LIF from the reset state (k_lif_apply's fresh branch): 4 bins per
    // lane, the currents as two 16-B stores and the u8 mirror as one 4-B store
    const K1bLif &L = pa.lif;
    unsigned long long my_sp = 0, my_mx = 0;
    const uint64_t nt = (uint64_t)k1b_lds_entries(L);
    auto lif = [&](unsigned long long x) -> uint32_t {
      float v;
      uint32_t rr;
      const uint64_t sp = (L.lp.skip_zero && x == 0) || L.lp.steps == 0 ? 0ull
                          : x < nt ? (uint64_t)s_tsp[x]
                                   : fresh_spikes(x, L.lp, L.tbl, L.tbl_n, v, rr);
      if (sp) {
        my_sp += sp;
        my_mx = sp > my_mx ? sp : my_mx;
        atomicAdd(&s_sh[sp < (uint64_t)(kHistBins - 1) ? (uint32_t)sp : (uint32_t)(kHistBins - 1)], 1u);
      }
      return sp < 255 ? (uint32_t)sp : 255u;
    };
    uint8_t *m8 = L.sc8 + nb0;
    // wave w of each 4096-bin span writes its 256 bins as two lane-contiguous
    // 1 KB stores of currents (lane l: bins 2l, 2l+1 and 128+2l, 129+2l) and
    // two 128-B stores of the u8 mirror
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (uint32_t s0 = wv * 256; s0 < nbins; s0 += 4 * kHistBlock) {
#pragma unroll
      for (uint32_t half = 0; half < 2; ++half) {
        const uint32_t t = s0 + 128 * half + 2 * lane;
        if (t + 2 <= nbins) {
          const unsigned long long x0 = count(t), x1 = count(t + 1);
          *reinterpret_cast<ulonglong2 *>(o + t) = make_ulonglong2(x0, x1);
          *reinterpret_cast<uint16_t *>(m8 + t) = (uint16_t)(lif(x0) | lif(x1) << 8);
        } else if (t < nbins) {
          const unsigned long long x = count(t);
          o[t] = x;
          m8[t] = (uint8_t)lif(x);
        }
      }
    }
    for (int sh = 32; sh > 0; sh >>= 1) {
      my_sp += __shfl_down(my_sp, sh, 64);
      const unsigned long long om = __shfl_down(my_mx, sh, 64);
      my_mx = om > my_mx ? om : my_mx;
    }
    if ((threadIdx.x & 63) == 0 && my_sp) {
      atomicAdd(&s_acc[0], my_sp);
      atomicMax(&s_acc[1], my_mx);
    }
    __syncthreads();
    if (threadIdx.x == 0 && s_acc[0]) {
      atomicAdd(&L.stats[0], s_acc[0]);
      atomicMax(&L.stats[1], s_acc[1]);
    }
    uint32_t *hc = L.hist + (size_t)(b & (kHistCopies - 1)) * kHistBins;
    for (int i = threadIdx.x + 1; i < kHistBins; i += kHistBlock)
      if (s_sh[i]) atomicAdd(&hc[i], s_sh[i]);
    return;
  }
  if (!partials) {
    unsigned long long *cur = pa.currents + nb0;
    for (uint32_t t = threadIdx.x; t < nbins; t += kHistBlock) {
      const uint32_t x = h[t];
      if (!x) continue;
      if (slices == 1) cur[t] += x;
      else atomicAdd(&cur[t], (unsigned long long)x);
    }
    return;
  }
  uint32_t *dst = partials + (uint64_t)r * pool + nb0;
  for (uint32_t t = threadIdx.x; t < nbins; t += kHistBlock) dst[t] = h[t];
}

// ---------------------------------------------------------------------------
// K1a + K1b fused across batches (k_part_fused, round 6).  K1a is bound by its
// SipHash instructions with HBM ~80 % idle; K1b is bound by HBM and LDS
// atomics.  So the count of batch i+1 also histograms batch i's records: each
// workgroup hashes its tile (part_tile) and some also take an item of the
// previous batch's K1b (HistJob).  K1a's 51.5 KB of LDS (three workgroups per
// CU) holds no 32768-bin u32 histogram, so an item is one (bucket, slice,
// third of the bins): it reads the slice's records once and adds each record
// at byte address off * 4 - third * R * 4 of the union.  A record of another
// third lands past the histogram: below 0 (wrapped) or past the workgroup's
// LDS allocation the hardware drops the access (tools/oobtest.hip), and between
// R words and the allocation's end is unread space of the same union -- so no
// compare, no branch: one ds_add per record per third.  The partials are
// k_bucket_hist's (slice r of bucket b at partials[r * pool + b * 32768 ...]).
// ---------------------------------------------------------------------------
constexpr uint32_t kFuseRange = (kBinsPerBucket + kFusePasses - 1) / kFusePasses;  // bins per third
static_assert(kFuseRange * 4 <= sizeof(PartLds<256, false>), "a third of a bucket fits the K1a union");
// a pad record (0xFFFF) lands past the allocation in every third
static_assert(4 * 0xFFFFull - 4ull * kFuseRange * (kFusePasses - 1) >= 64 * 1024,
              "pad records stay past the allocation");
#ifndef NK_FUSE_KU
#define NK_FUSE_KU 2  // 16-B loads per lane per round (registers: the kernel keeps 6 waves per SIMD)
#endif

// item -> (third, bucket, slice); the three thirds of one slice are
// consecutive items (workgroups close in time: the slice's second and third
// reads come from the caches)
__device__ __forceinline__ void fused_hist_item(const HistJob &hj, uint32_t item, uint32_t *h) {
  const uint32_t third = item % kFusePasses;
  const uint32_t rest = item / kFusePasses;
  const uint32_t b = rest % hj.n_buckets, r = rest / hj.n_buckets;
  const uint64_t nb0 = (uint64_t)b << kBinBits;
  const uint64_t nbins = hj.pool - nb0 < (uint64_t)kBinsPerBucket ? hj.pool - nb0 : kBinsPerBucket;
  const uint64_t t0 = (uint64_t)third * kFuseRange;
  if (t0 >= nbins) return;  // (uniform)
  const uint32_t cnt = (uint32_t)(nbins - t0 < kFuseRange ? nbins - t0 : kFuseRange);
  const uint32_t base = (uint32_t)t0 * 4u;
  const int tid = threadIdx.x;
  __syncthreads();  // (the LDS: the tile's stores or the previous item read it)
  for (uint32_t t = tid; t < kFuseRange; t += kPartBlock) h[t] = 0;
  __syncthreads();
  char *hb = reinterpret_cast<char *>(h);
  auto add = [&](uint32_t off) { atomicAdd(reinterpret_cast<uint32_t *>(hb + ((off << 2) - base)), 1u); };
  // this slice's share [lo, hi) of the bucket's records, sub-region by sub-region
  const uint32_t nsub = 1u << hj.sub_shift;
  uint64_t n = 0;
  for (uint32_t x = 0; x < nsub; ++x) {
    const uint64_t f = hj.fill[((uint64_t)b << hj.sub_shift) | x] & ((1ull << 40) - 1);
    n += f < hj.cap ? f : hj.cap;
  }
  const uint64_t lo_all = n * r / hj.slices, hi_all = n * (r + 1) / hj.slices;
  uint64_t c0 = 0;
  for (uint32_t x = 0; x < nsub; ++x) {
    const uint64_t vb = ((uint64_t)b << hj.sub_shift) | x;
    uint64_t nv = hj.fill[vb] & ((1ull << 40) - 1);
    if (nv > hj.cap) nv = hj.cap;
    const uint64_t a = lo_all > c0 ? lo_all : c0, z = hi_all < c0 + nv ? hi_all : c0 + nv;
    const uint64_t lo = a - c0, hi = z > a ? z - c0 : lo;
    c0 += nv;
    if (lo >= hi) continue;  // (uniform)
    const uint16_t *src = hj.off + vb * hj.cap;
    uint64_t i = lo;
    for (; i < hi && (i & 7); ++i)
      if (tid == 0) add(src[i]);
    const uint64_t hi8 = i + ((hi - i) & ~7ull);
    constexpr uint64_t step = 8ull * kPartBlock;
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    // NK_FUSE_KU 16-B loads per lane per round, the next round's in flight
    // while this round's records are added (as k_bucket_hist)
    uint64_t j = i + 8ull * tid;
    if (j < hi8) {
      auto load_round = [&](uint64_t jb, u32x4 *v) {
#pragma unroll
        for (int t = 0; t < NK_FUSE_KU; ++t) {
          const uint64_t jt = jb + (uint64_t)t * step;
          v[t] = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(src + (jt < hi8 ? jt : i)));
        }
      };
      u32x4 cur[NK_FUSE_KU];
      load_round(j, cur);
      for (;;) {
        const uint64_t jn = j + (uint64_t)NK_FUSE_KU * step;
        const bool more = jn < hi8;
        u32x4 nxt[NK_FUSE_KU];
        load_round(more ? jn : j, nxt);
#pragma unroll
        for (int t = 0; t < NK_FUSE_KU; ++t)
          if (j + (uint64_t)t * step < hi8) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              add(cur[t][e] & 0xFFFFu);
              add(cur[t][e] >> 16);
            }
          }
        if (!more) break;
        j = jn;
#pragma unroll
        for (int t = 0; t < NK_FUSE_KU; ++t) cur[t] = nxt[t];
      }
    }
    for (uint64_t q = hi8 + tid; q < hi; q += kPartBlock) add(src[q]);
  }
  __syncthreads();
  uint32_t *dst = hj.partials + (uint64_t)r * hj.pool + nb0 + t0;
  for (uint32_t t = tid; t < cnt; t += kPartBlock) dst[t] = h[t];
}

// K1a of this batch + K1b items of the previous one (workgroups [0, n_host)
// take items [ceil(w * n_items / n_host), ceil((w + 1) * n_items / n_host)):
// spread over the first part of the grid, so no item is in the tail)
template <bool CANON, bool K16>
__global__ __launch_bounds__(kPartBlock) __attribute__((amdgpu_waves_per_eu(CANON ? 6 : 4))) void k_part_fused(
    KmerInput in, int k, FastMod fm, PartArgs pa, HistJob hj) {
  // the only LDS object of the kernel: a dropped or unread third-of-bucket
  // access can touch nothing else
  __shared__ union FU {
    PartLds<256, !CANON> a;
    uint32_t h[sizeof(PartLds<256, !CANON>) / 4];
  } sm;
  part_tile<CANON, 256, K16, false>(in, k, fm, pa, sm.a);
  const uint32_t w = blockIdx.x;
  if (w >= hj.n_host) return;
  const uint32_t i0 = (uint32_t)(((uint64_t)w * hj.n_items + hj.n_host - 1) / hj.n_host);
  const uint32_t i1 = (uint32_t)(((uint64_t)(w + 1) * hj.n_items + hj.n_host - 1) / hj.n_host);
  for (uint32_t it = i0; it < i1; ++it) fused_hist_item(hj, it, sm.h);
}

__global__ void k_partials_add(const uint32_t *__restrict__ partials, uint32_t slices,
                               uint64_t pool, unsigned long long *__restrict__ currents) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < pool;
       i += (uint64_t)gridDim.x * blockDim.x) {
    unsigned long long s = currents[i];
    for (uint32_t r = 0; r < slices; ++r) s += partials[(uint64_t)r * pool + i];
    currents[i] = s;
  }
}

// Key of the k-mer at absolute position p (k <= 32) from three 16-B loads,
// through the same conversion as the tile staging.
template <bool CANON>
__device__ __forceinline__ uint64_t vec_window_key(const uint8_t *bases, uint64_t n_bases,
                                                   uint64_t p, int k) {
  const uint64_t a = p & ~15ull;
  uint32_t F[3], R[3], INV[3];
  for (int c = 0; c < 3; ++c) {
    const uint64_t g = a + 16ull * c;
    uint4 v;
    if (g + 16 <= n_bases) {
      v = *reinterpret_cast<const uint4 *>(bases + g);
    } else {
      uint32_t w[4] = {0, 0, 0, 0};
      for (int j = 0; j < 16; ++j)
        if (g + j < n_bases) w[j >> 2] |= (uint32_t)bases[g + j] << (8 * (j & 3));
      v = make_uint4(w[0], w[1], w[2], w[3]);
    }
    Conv4 x = conv4(v.x), y = conv4(v.y), z = conv4(v.z), t = conv4(v.w);
    F[c] = (x.fnib << 24) | (y.fnib << 16) | (z.fnib << 8) | t.fnib;
    R[c] = x.rnib | (y.rnib << 8) | (z.rnib << 16) | (t.rnib << 24);
    INV[c] = x.inv | (y.inv << 4) | (z.inv << 8) | (t.inv << 12);
  }
  const int q = (int)(p - a), s = 2 * q, twok = 2 * k;
  const uint64_t hi64 = ((uint64_t)F[0] << 32) | F[1];
  const uint64_t fwd = ((hi64 << s) | (((uint64_t)F[2] << s) >> 32)) >> (64 - twok);
  if (CANON) {
    const uint64_t mask2k = (k >= 32) ? ~0ULL : ((1ULL << twok) - 1ULL);
    const uint64_t lo64 = ((uint64_t)R[1] << 32) | R[0];
    const uint64_t rev = ((lo64 >> s) | (((uint64_t)R[2] << 32) << (32 - s))) & mask2k;
    return fwd < rev ? fwd : rev;
  }
  const uint64_t inv = ((uint64_t)INV[0] | ((uint64_t)INV[1] << 16) | ((uint64_t)INV[2] << 32)) >> q;
  const uint64_t kmask = (1ull << k) - 1ull;
  if (!(inv & kmask)) return fwd;
  return global_window_key<false>(bases, p, k);
}

// Last index a in [0, n) with d[a].y <= x (d sorted by .y, d[0].y <= x), found
// by one wave with 64-ary steps: 2-4 dependent loads instead of ~log2(n).
__device__ uint64_t wave_search_le(const uint2 *d, uint64_t n, uint64_t x) {
  const int lane = threadIdx.x & 63;
  uint64_t lo = 0, hi = n;
  while (hi - lo > 1) {
    const uint64_t step = (hi - lo + 63) / 64;
    const uint64_t idx = lo + (uint64_t)lane * step;
    const bool ok = idx < hi && d[idx].y <= x;
    const uint64_t mask = __ballot(ok);
    const int last = 63 - __clzll((long long)mask);  // lane 0 always ok
    lo = lo + (uint64_t)last * step;
    const uint64_t nh = lo + step;
    hi = nh < hi ? nh : hi;
  }
  return lo;
}

// Uniques from the kept records, in ONE flat kernel, k_uniq_scan: stream the
// records of the buckets holding top-N neurons (16-B loads), test each bin
// offset against an LDS bitmap of the bucket's top bins, collect hits {top
// row, record index} in LDS; then each workgroup resolves its hits to base
// positions (record -> segment through an LDS table of the slice's segments),
// recomputes each hit's key from the bases, deduplicates in LDS and inserts
// into the global hash set.  The set is emptied beforehand (by the prep kernel
// of the count, or by k_set_fill), never by this kernel's own blocks, so no
// block can insert into a slot another block has yet to clear.  Hits never
// serialise inside a wave and no lane waits on another's latency.
constexpr int kScanBuf = 4096;

// A scan hit {bucket | top row | record index} as k_uniq_hits takes it:
// top row << 48 | base position of the k-mer (segment a holds the record).
__device__ __forceinline__ unsigned long long hit_at(const PartArgs &pa, uint64_t b, uint64_t a,
                                                     unsigned long long e) {
  const uint64_t i = e & ((1ull << 38) - 1);
  const uint64_t slot = (e >> 38) & 0x3FFu;
  const uint64_t p = (uint64_t)pa.desc[(uint64_t)b * pa.max_segs + a].x * kPartTile +
                     pa.pos[(uint64_t)b * pa.cap + i];
  return (slot << 48) | p;
}

// Same, the segment found by a binary search of descriptors [a, z) in global
// memory (d[a].y <= the record index).
__device__ unsigned long long resolve_hit(const PartArgs &pa, uint64_t b, uint64_t a, uint64_t z,
                                          unsigned long long e) {
  const uint64_t i = e & ((1ull << 38) - 1);
  const uint2 *d = pa.desc + (uint64_t)b * pa.max_segs;
  while (z - a > 1) {
    const uint64_t m = (a + z) >> 1;
    if (d[m].y <= i) a = m;
    else z = m;
  }
  return hit_at(pa, b, a, e);
}

template <bool CANON>
__global__ __launch_bounds__(kHistBlock) void k_uniq_scan(KmerInput in, int k, PartArgs pa,
                                                          UniqArgs u,
                                                          const uint32_t *__restrict__ tbuckets,
                                                          const uint32_t *__restrict__ n_tb,
                                                          uint32_t slices) {
  __shared__ uint32_t bits[65536 / 32];  // covers the pad sentinel bin (never set)
  __shared__ uint32_t t_off[kMaxTopN];
  __shared__ uint32_t t_slot[kMaxTopN];
  __shared__ unsigned long long buf[kScanBuf];
  __shared__ unsigned long long seen[kSeen];
  __shared__ uint32_t t_n, s_nh;
  __shared__ uint64_t s_seg[2];
  if (blockIdx.y >= *n_tb) return;
  const uint32_t b = tbuckets[blockIdx.y], r = blockIdx.x;
  for (int i = threadIdx.x; i < 65536 / 32; i += kHistBlock) bits[i] = 0;
  seen_init(seen);
  if (threadIdx.x == 0) { t_n = 0; s_nh = 0; }
  __syncthreads();
  for (uint32_t s = threadIdx.x; s < u.n_top; s += kHistBlock) {
    const uint64_t idx = u.top[s].idx;
    if ((idx >> pa.bin_bits) == b) {
      const uint32_t off = (uint32_t)(idx & ((1u << pa.bin_bits) - 1u));
      const uint32_t t = atomicAdd(&t_n, 1u);
      t_off[t] = off;
      t_slot[t] = s;
      atomicOr(&bits[off >> 5], 1u << (off & 31));
    }
  }
  __syncthreads();
  // sub-regions (pa.sub_shift): slice r scans sub-region r mod 2^sub_shift,
  // its share r >> sub_shift of (slices >> sub_shift); vb indexes the region,
  // the fill and the descriptors (the host passes a multiple of 2^sub_shift)
  const uint64_t vb = ((uint64_t)b << pa.sub_shift) | (r & ((1u << pa.sub_shift) - 1u));
  const uint32_t rs = r >> pa.sub_shift, ns_sl = slices >> pa.sub_shift;
  uint64_t n = pa.fill[vb] & ((1ull << 40) - 1);
  if (n > pa.cap) n = pa.cap;
  const uint64_t lo = n * rs / ns_sl, hi = n * (rs + 1) / ns_sl;
  uint64_t n_seg = pa.fill[vb] >> 40;
  if (n_seg > pa.max_segs) n_seg = pa.max_segs;
  const uint32_t tn = t_n;
  const uint16_t *src = pa.off + vb * pa.cap;
  // a hit's key into the set: recomputed from the bases at its position
  auto insert_hit = [&](unsigned long long h) {
    const uint32_t slot = (uint32_t)(h >> 48);
    const uint64_t p = h & ((1ull << 48) - 1);
    const uint64_t key = vec_window_key<CANON>(in.bases, in.n_bases, p, k);
    if (key == kEmpty || !seen_before(seen, key)) set_insert(u, slot, key);
  };
  // one hit record: bucket | top row | record index (< 2^38)
  auto push = [&](uint64_t i, uint32_t off) {
    uint32_t slot = 0;
    for (uint32_t t = 0; t < tn; ++t)
      if (t_off[t] == off) slot = t_slot[t];
    const unsigned long long e = ((unsigned long long)b << 48) |
                                 ((unsigned long long)slot << 38) | i;
    const uint32_t at = atomicAdd(&s_nh, 1u);
    if (at < kScanBuf) buf[at] = e;
    else insert_hit(resolve_hit(pa, vb, 0, n_seg, e));  // LDS list full (very hit-dense slice)
  };
  // 8 records per 16-B load, eight loads in flight per lane (the slice is a
  // few dozen loads per lane: latency, not bandwidth, bounds a shallow loop);
  // no barrier in the loop
#ifndef NK_U1_KU
#define NK_U1_KU 4
#endif
  constexpr int kU = NK_U1_KU;  // 16-B loads in flight per lane
  const uint64_t lo8 = lo & ~7ull;
  const uint64_t step = 8ull * kHistBlock;
  for (uint64_t c0 = lo8 + 8ull * threadIdx.x; c0 < hi; c0 += kU * step) {
    uint4 v[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {  // unconditional (clamped) loads: one round trip
      const uint64_t c = c0 + u * step;
      v[u] = *reinterpret_cast<const uint4 *>(src + (c < hi ? c : lo8));
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const uint64_t base = c0 + u * step;
      if (base >= hi) break;
      const uint64_t w01 = ((uint64_t)v[u].y << 32) | v[u].x;
      const uint64_t w23 = ((uint64_t)v[u].w << 32) | v[u].z;
      uint32_t hm = 0;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint32_t off = (uint32_t)(((j < 4 ? w01 : w23) >> (16 * (j & 3))) & 0xFFFFu);
        const uint64_t i = base + j;
        if (i >= lo && i < hi && ((bits[off >> 5] >> (off & 31)) & 1u)) hm |= 1u << j;
      }
#pragma unroll 1
      while (hm) {
        const int j = __ffs(hm) - 1;
        hm &= hm - 1;
        push(base + j, (uint32_t)(((j < 4 ? w01 : w23) >> (16 * (j & 3))) & 0xFFFFu));
      }
    }
  }
  __syncthreads();
  const uint32_t nh = s_nh < (uint32_t)kScanBuf ? s_nh : (uint32_t)kScanBuf;
  if (!nh) return;
  // resolve the buffered hits to base positions here (k_uniq_hits then only
  // recomputes keys): the slice's segments, found by two waves with 64-ary
  // searches, have their first-record indices staged in LDS (the bitmap is
  // done with), so each hit costs an LDS search plus two parallel loads
  // instead of a chain of ~log2(segments) dependent global loads
  const uint2 *d = pa.desc + vb * pa.max_segs;
  if (threadIdx.x < 128) {
    const uint64_t x = threadIdx.x < 64 ? lo : hi - 1;
    const uint64_t a = wave_search_le(d, n_seg, x);
    if ((threadIdx.x & 63) == 0) s_seg[threadIdx.x >> 6] = a;
  }
  __syncthreads();
  const uint64_t s0 = s_seg[0], ns = s_seg[1] - s0 + 1;
  uint32_t *tab = bits;
  const bool staged = ns <= (uint64_t)(65536 / 32);
  if (staged)
    for (uint32_t j = threadIdx.x; j < ns; j += kHistBlock) tab[j] = d[s0 + j].y;
  __syncthreads();
  for (uint32_t h = threadIdx.x; h < nh; h += kHistBlock) {
    const unsigned long long e = buf[h];
    unsigned long long out;
    if (staged) {
      const uint64_t i = e & ((1ull << 38) - 1);
      uint32_t a = 0, z = (uint32_t)ns;  // last j with tab[j] <= i (tab[0] <= lo <= i)
      while (z - a > 1) {
        const uint32_t m = (a + z) >> 1;
        if (tab[m] <= i) a = m;
        else z = m;
      }
      out = hit_at(pa, vb, s0 + a, e);
    } else {
      out = resolve_hit(pa, vb, s0, s0 + ns, e);
    }
    insert_hit(out);
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

__device__ __forceinline__ bool cand_before(const TopCand &a, const TopCand &b) {
  return a.sc != b.sc ? a.sc > b.sc : a.idx < b.idx;
}

// Exclusive prefix sum over the threads of a block (blockDim.x <= 1024, a
// multiple of 64); *total gets the block sum.  Two barriers.
template <typename T>
__device__ __forceinline__ T block_excl_scan(T x, T *s_w, T *total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  T incl = x;
  for (int o = 1; o < 64; o <<= 1) {
    const T y = __shfl_up(incl, o, 64);
    if (lane >= o) incl += y;
  }
  if (lane == 63) s_w[w] = incl;
  __syncthreads();
  T pre = 0, tot = 0;
  for (int i = 0; i < nw; ++i) {
    const T v = s_w[i];
    pre += i < w ? v : (T)0;
    tot += v;
  }
  __syncthreads();
  *total = tot;
  return pre + incl - x;
}

// (top_post_block: nk_post.h)

#ifndef NK_LIF_PER_THREAD
#define NK_LIF_PER_THREAD 8
#endif
constexpr int kLifPerThread = NK_LIF_PER_THREAD;

constexpr int kLifBlock = 1024;
constexpr int kLifWaves = kLifBlock / 64;

// Fused top-N keys: (spikes << 24) | (0xFFFFFF - index), so that descending
// u64 order is exactly (spikes desc, index asc) (src/spiking_hash.rs:661-673).
// Needs index < 2^24 (pool <= 2^24: the fused path's pool bound) and
// spikes < 2^40 (else the selection defers to the host's exact path).
constexpr int kKeyIdxBits = 24;
constexpr uint64_t kKeyIdxMask = (1ull << kKeyIdxBits) - 1;
constexpr uint64_t kKeyMaxSpikes = 1ull << 40;
constexpr uint32_t kDeferMark = 0xFFFFFFFFu;  // bcnt of a block whose list could not be built
__device__ __forceinline__ uint64_t top_key(uint64_t sc, uint64_t idx) {
  return (sc << kKeyIdxBits) | (kKeyIdxMask - idx);
}
__device__ __forceinline__ uint64_t key_idx(uint64_t key) { return kKeyIdxMask - (key & kKeyIdxMask); }
__device__ __forceinline__ uint64_t key_sc(uint64_t key) { return key >> kKeyIdxBits; }

// Bitonic sort of one u64 per lane across a wave64, descending (registers +
// shuffles).  Empty lanes carry 0.
__device__ __forceinline__ uint64_t wave_sort64_desc(uint64_t x) {
  const int lane = threadIdx.x & 63;
  for (int size = 2; size <= 64; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      const uint64_t y = __shfl_xor(x, stride, 64);
      const bool up = (lane & size) == 0, lower = (lane & stride) == 0;
      if (lower == up ? y > x : x > y) x = y;
    }
  }
  return x;
}

// Block-local top `want` rows of this LIF block (want <= kFuseMaxTopN) from its
// spike histogram `sh` (bin = min(spikes, 4095)): rows above the block
// threshold, then the threshold ties in index order.  They go out as keys,
// sorted descending, to gout, their number to *gcnt.  Returns false when the
// threshold falls in the clamp bin or a count is too large for a key (the
// final step then defers to the host's exact path).
__device__ bool block_top(const uint32_t *sh, const uint64_t *scv, uint64_t base, uint64_t pool,
                          uint32_t want, uint64_t *out, uint64_t *gout, uint32_t *gcnt) {
  __shared__ uint32_t s_w[kLifWaves];
  __shared__ uint32_t s_T, s_above, s_need, s_n, s_big;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  // thread t owns bins 4095-4t .. 4092-4t (counted from the top)
  uint32_t loc = 0;
  for (int j = 0; j < 4; ++j) loc += sh[kHistBins - 1 - (4 * t + j)];
  uint32_t total;
  const uint32_t before = block_excl_scan(loc, s_w, &total);
  if (t == 0) {  // fewer rows than `want` in this block: take everything
    s_T = 0;
    s_above = total - sh[0];
    s_need = want - s_above;
    s_n = 0;
    s_big = 0;
  }
  __syncthreads();
  if (total >= want && before < want && before + loc >= want) {
    uint32_t cum = before;
    for (int j = 0; j < 4; ++j) {
      const int bin = kHistBins - 1 - (4 * t + j);
      const uint32_t h = sh[bin];
      if (cum + h >= want) {
        s_T = (uint32_t)bin;
        s_above = cum;
        s_need = want - cum;
        break;
      }
      cum += h;
    }
  }
  __syncthreads();
  const uint64_t T = s_T;
  const uint32_t above = s_above, need = s_need;
  if (T == (uint64_t)(kHistBins - 1)) return false;
  for (int j = 0; j < kLifPerThread; ++j) {
    const uint64_t i = base + (uint64_t)j * kLifBlock + t;
    if (i < pool && scv[j] > T) {
      if (scv[j] >= kKeyMaxSpikes) s_big = 1;
      out[atomicAdd(&s_n, 1u)] = top_key(scv[j], i);
    }
  }
  // ties: index order is (row j, thread t)
  uint32_t run = 0;
  for (int j = 0; j < kLifPerThread && run < need; ++j) {
    const uint64_t i = base + (uint64_t)j * kLifBlock + t;
    const bool tie = i < pool && scv[j] == T;
    const uint64_t bal = __ballot(tie);
    if (lane == 0) s_w[w] = (uint32_t)__popcll(bal);
    __syncthreads();
    uint32_t pre = run, row = 0;
    for (int q = 0; q < kLifWaves; ++q) {
      pre += q < w ? s_w[q] : 0u;
      row += s_w[q];
    }
    const uint32_t r = pre + (uint32_t)__popcll(bal & ((1ull << lane) - 1ull));
    if (tie && r < need) out[above + r] = top_key(T, i);
    run += row;
    __syncthreads();
  }
  __syncthreads();
  if (s_big) return false;
  if (t < 64) {  // this block's rows, sorted, to its candidate slot (wave 0)
    const uint32_t n = above + (run < need ? run : need);
    uint64_t x = (uint32_t)t < n ? out[t] : 0ull;
    x = wave_sort64_desc(x);
    if ((uint32_t)t < n) gout[t] = x;
    if (t == 0) *gcnt = n;
  }
  return true;
}

// Selection left to the host's exact path: flag it, and leave the uniques pass
// that is already queued with no work (no top buckets, no hits).
__device__ void defer_to_host(const TopFuse &tf) {
  tf.st->T = kHistBins - 1;
  tf.st->n_above = 0;
  tf.st->need = 0;
  tf.st->emit_above = 0;
  tf.st->refine = 1u;
  for (int i = 0; i < 4; ++i) tf.post.flags[i] = 0;
  *tf.post.n_hits = 0;
  if (tf.post.set_mask) *tf.post.set_mask = 0;  // the (idle) uniques pass clears one slot
  if (tf.seg) {  // the slice exports no rows, only the refine flag (k_slice_seg's rule)
    tf.seg[0] = kSegRefine;
    tf.seg[1] = tf.seg_stats[0];
    tf.seg[2] = tf.seg_stats[1];
  }
}

// The final selection over the blocks' candidate lists C (one block of
// kLifBlock threads).  The global top rows are the top rows of C (every global
// top row is in its block's list), so the threshold comes from a histogram of
// C alone; ties at the threshold are taken in index order, which is block
// order and, inside a block's list, list order.  Then the rows are sorted and
// the uniques bookkeeping (k_top_post) is done by wave 0.
__device__ void final_top(uint64_t pool, const uint64_t *currents, uint32_t nb,
                          const TopFuse &tf) {
  __shared__ uint32_t s_h[kHistBins];
  __shared__ uint32_t s_w32[kLifWaves];
  __shared__ uint32_t s_T, s_above, s_need, s_na, s_bad;
  __shared__ uint32_t s_ab[kFuseMaxBlocks], s_tb[kFuseMaxBlocks];
  __shared__ uint64_t s_fin[kFuseMaxTopN];
  const int t = threadIdx.x;
  const uint32_t want = (uint32_t)(tf.want < pool ? tf.want : pool);
  const uint32_t W = tf.want, M = nb * W;
  for (int i = t; i < kHistBins; i += kLifBlock) s_h[i] = 0;
  if ((uint32_t)t < nb) { s_ab[t] = 0; s_tb[t] = 0; }
  if (t == 0) { s_na = 0; s_bad = 0; }
  __syncthreads();
  if ((uint32_t)t < nb && tf.bcnt[t] == kDeferMark) s_bad = 1;
  constexpr int U = 8;
  uint64_t cv[U];
  uint32_t cn[U];
  // unconditional loads at clamped indices: the U loads of a chunk are in
  // flight together (one round trip); masked afterwards
  auto load_chunk = [&](uint32_t c0) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      uint32_t id = c0 + u * kLifBlock + t;
      id = id < M ? id : M - 1;
      cn[u] = tf.bcnt[id / W];
      cv[u] = tf.bcand[id];
    }
  };
  auto live = [&](uint32_t c0, int u) {
    const uint32_t id = c0 + u * kLifBlock + t;
    return id < M && id % W < cn[u];
  };
  const bool one_chunk = M <= (uint32_t)(U * kLifBlock);
  __syncthreads();
  // (1) histogram of the candidates' spike counts -> threshold T
  for (uint32_t c0 = 0; c0 < M; c0 += U * kLifBlock) {
    load_chunk(c0);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (!live(c0, u)) continue;
      const uint64_t sc = key_sc(cv[u]);
      atomicAdd(&s_h[sc < (uint64_t)(kHistBins - 1) ? (uint32_t)sc : (uint32_t)(kHistBins - 1)], 1u);
    }
  }
  __syncthreads();
  {
    uint32_t loc = 0;
    for (int j = 0; j < 4; ++j) loc += s_h[kHistBins - 1 - (4 * t + j)];
    uint32_t total;
    const uint32_t before = block_excl_scan(loc, s_w32, &total);
    if (t == 0) { s_T = 0; s_above = total - s_h[0]; s_need = want - (total - s_h[0]); }
    __syncthreads();
    if (total >= want && before < want && before + loc >= want) {
      uint32_t cum = before;
      for (int j = 0; j < 4; ++j) {
        const int bin = kHistBins - 1 - (4 * t + j);
        if (cum + s_h[bin] >= want) {
          s_T = (uint32_t)bin;
          s_above = cum;
          s_need = want - cum;
          break;
        }
        cum += s_h[bin];
      }
    }
    __syncthreads();
  }
  const uint64_t T = s_T;
  const uint32_t n_above = s_above, need = s_need;
  if (T == (uint64_t)(kHistBins - 1) || s_bad) {  // spike counts >= 4095: host radix refine
    if (t == 0) defer_to_host(tf);
    return;
  }
  // (2) rows above T (any order: sorted below) and per-list tie counts
  for (uint32_t c0 = 0; c0 < M; c0 += U * kLifBlock) {
    if (!one_chunk) load_chunk(c0);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (!live(c0, u)) continue;
      const uint32_t id = c0 + u * kLifBlock + t;
      const uint64_t sc = key_sc(cv[u]);
      if (sc > T) {
        atomicAdd(&s_ab[id / W], 1u);
        const uint32_t at = atomicAdd(&s_na, 1u);
        if (at < kFuseMaxTopN) s_fin[at] = cv[u];
      } else if (sc == T) {
        atomicAdd(&s_tb[id / W], 1u);
      }
    }
  }
  __syncthreads();
  uint32_t ttot;
  const uint32_t tpre = block_excl_scan((uint32_t)t < nb ? s_tb[t] : 0u, s_w32, &ttot);
  if ((uint32_t)t < nb) s_tb[t] = tpre;
  if (t == 0 && (s_na != n_above || ttot < need)) s_bad = 1;  // cannot happen; be safe
  __syncthreads();
  if (s_bad) {
    if (t == 0) defer_to_host(tf);
    return;
  }
  // (3) ties: the first `need` in block order, list order inside a block
  for (uint32_t c0 = 0; c0 < M; c0 += U * kLifBlock) {
    if (!one_chunk) load_chunk(c0);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (!live(c0, u) || key_sc(cv[u]) != T) continue;
      const uint32_t id = c0 + u * kLifBlock + t;
      const uint32_t b = id / W;
      const uint32_t r = s_tb[b] + (id % W - s_ab[b]);
      if (r < need) s_fin[n_above + r] = cv[u];
    }
  }
  __syncthreads();
  if (t >= 64) return;
  // (4) wave 0: exact order, rows and currents out, uniques bookkeeping
  // (as k_top_post), all without block barriers
  const int lane = t;
  const uint32_t m = want;
  const bool row = (uint32_t)lane < m;
  const uint64_t key = wave_sort64_desc(row ? s_fin[lane] : 0ull);
  const uint64_t idx = key_idx(key), sc = key_sc(key);
  // a row outside the pool (a selection the refine redoes) is never indexed;
  // it counts as an overflowed bucket, which sends the host down the rescan
  const bool in_pool = idx < pool;
  const uint64_t cur = (row && in_pool) ? currents[idx] : 0ull;
  const PostArgs &pa = tf.post;
  const uint32_t bk = in_pool ? (uint32_t)(idx >> pa.bin_bits) : 0u;
  const bool bk_ok = in_pool && (!pa.n_over || bk < pa.n_over);
  const uint32_t over = (row && pa.part) ? (bk_ok ? pa.overflow[bk] : 1u) : 0u;
  if (row) {
    tf.cand[lane].idx = idx;
    tf.cand[lane].sc = sc;
    tf.top_cur[lane] = cur;
    pa.uniq[lane] = 0;
    pa.special[lane] = 0;
  }
  if (tf.seg) {  // the slice's all-gather segment (nk_slice_export; k_slice_seg's layout)
    const bool bad = __ballot(row && !in_pool) != 0;  // a row the passes left unfilled
    if (row && !bad) {
      tf.seg[3 + 3 * (uint64_t)lane] = idx + tf.seg_lo;
      tf.seg[4 + 3 * (uint64_t)lane] = sc;
      tf.seg[5 + 3 * (uint64_t)lane] = cur;
    }
    if (lane == 0) {
      tf.seg[0] = bad ? kSegRefine : (uint64_t)m;
      tf.seg[1] = tf.seg_stats[0];
      tf.seg[2] = tf.seg_stats[1];
    }
  }
  unsigned long long sum = cur;
  for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o, 64);
  bool first = row && pa.part;  // first row of its bucket in the list
  for (int j = 0; j < 64; ++j) {
    const uint32_t bj = __shfl(bk, j, 64);
    if (j < lane && bj == bk) first = false;
  }
  const uint64_t fb = __ballot(first);
  if (first) pa.tbuckets[__popcll(fb & ((1ull << lane) - 1ull))] = bk;
  const bool any_over = __ballot(over != 0) != 0;
  if (lane == 0) {
    uint64_t cap = 64;
    while (cap < 2 * (uint64_t)sum + 2 && cap < (1ull << 48)) cap <<= 1;  // (bounded, as k_top_post)
    pa.flags[0] = cap > pa.set_alloc ? 1u : 0u;  // set too small
    pa.flags[1] = any_over ? 1u : 0u;            // a top bucket overflowed
    pa.flags[2] = (uint32_t)__popcll(fb);        // distinct top buckets
    pa.flags[3] = 0;
    *pa.set_mask = (cap > pa.set_alloc ? pa.set_alloc : cap) - 1;
    *pa.n_hits = 0;
    tf.st->T = T;
    tf.st->n_above = n_above;
    tf.st->need = need;
    tf.st->emit_above = n_above;
    tf.st->refine = 0u;
  }
}

__device__ __forceinline__ uint64_t spikes_at(const SpikeSrc &s, uint64_t i) {
  if (s.sc8) {  // 1 B per neuron; 255 means "255 or more": the exact value below
    const uint32_t v = s.sc8[i];
    if (v < 255u) return v;
  }
  if (s.sc) return s.sc[i];
  float v;
  uint32_t r;
  return fresh_spikes(s.cur[i], s.lp, s.tbl, s.tbl_n, v, r);
}

// the derived state written out (materialised): v / r / spike counts
__global__ void k_lif_derive(const uint64_t *__restrict__ cur, float *__restrict__ V,
                             uint32_t *__restrict__ R, uint64_t *__restrict__ SC, uint64_t pool,
                             LifParams lp, const LifEntry *__restrict__ tbl, int tbl_n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < pool;
       i += (uint64_t)gridDim.x * blockDim.x) {
    float v;
    uint32_t r;
    const uint64_t sp = fresh_spikes(cur[i], lp, tbl, tbl_n, v, r);
    V[i] = v;
    R[i] = r;
    SC[i] = sp;
  }
}

__global__ __launch_bounds__(kLifBlock) void k_lif_apply(uint64_t *__restrict__ currents,
                                                      const uint32_t *__restrict__ partials,
                                                      uint32_t slices, int cur_zero,
                                                      const uint32_t *__restrict__ over,
                                                      int over_bits, int fresh, int derive,
                                                      float *__restrict__ V,
                                                      uint32_t *__restrict__ R,
                                                      uint64_t *__restrict__ SC, uint64_t pool,
                                                      LifParams lp,
                                                      const LifEntry *__restrict__ tbl, int tbl_n,
                                                      uint32_t *__restrict__ hist,
                                                      unsigned long long *__restrict__ stats,
                                                      TopFuse tf, uint8_t *__restrict__ sc8) {
  __shared__ uint32_t sh[kHistBins];
  __shared__ unsigned long long s_sp[kLifWaves];
  __shared__ unsigned long long s_mx[kLifWaves];
  __shared__ uint64_t s_cand[kFuseMaxTopN];
  for (int i = threadIdx.x; i < kHistBins; i += kLifBlock) sh[i] = 0;
  __syncthreads();
  const uint64_t base = (uint64_t)blockIdx.x * kLifBlock * kLifPerThread;
  unsigned long long my_sp = 0, my_mx = 0;
  uint32_t n_zero = 0;  // neurons of this thread with spike count 0 (histogram bin 0)
  // all loads of this thread's neurons first (a few round trips), then the LIF
  uint64_t cntv[kLifPerThread], scv[kLifPerThread];
  float vin[kLifPerThread];
  uint32_t rin[kLifPerThread];
  auto idx_of = [&](int j) {  // clamped: unconditional loads
    const uint64_t i = base + (uint64_t)j * kLifBlock + threadIdx.x;
    return i < pool ? i : pool - 1;
  };
#pragma unroll
  for (int j = 0; j < kLifPerThread; ++j) {
    const uint64_t i = idx_of(j);
    // cur_zero: the partials (wire) hold it all; over: the count zeroed the
    // currents and only overflowed buckets added into them
    cntv[j] = (cur_zero || (over && !over[i >> over_bits])) ? 0ull : currents[i];
    scv[j] = fresh ? 0 : SC[i];
    vin[j] = fresh ? 0.0f : V[i];
    rin[j] = fresh ? 0u : R[i];
  }
  for (uint32_t r = 0; r < slices; ++r) {  // fused K1c: fold the partials in
    const uint32_t *pr = partials + (uint64_t)r * pool;
    uint32_t pv[kLifPerThread];
#pragma unroll
    for (int j = 0; j < kLifPerThread; ++j) pv[j] = pr[idx_of(j)];
#pragma unroll
    for (int j = 0; j < kLifPerThread; ++j) cntv[j] += pv[j];
  }
  LifEntry ev[kLifPerThread];  // closed-form table rows of fresh neurons
#pragma unroll
  for (int j = 0; j < kLifPerThread; ++j)
    ev[j] = tbl[cntv[j] < (uint64_t)tbl_n ? cntv[j] : (uint64_t)tbl_n - 1];
#pragma unroll
  for (int j = 0; j < kLifPerThread; ++j) {
    const uint64_t i = base + (uint64_t)j * kLifBlock + threadIdx.x;
    if (i >= pool) {
      scv[j] = 0;
      continue;
    }
    const uint64_t cnt = cntv[j];
    if (slices) currents[i] = cnt;
    // fresh state (after nk_reset): v = r = spikes = 0 without reading them,
    // and every neuron is written
    uint64_t sc = scv[j];
    if (!(lp.skip_zero && cnt == 0) && lp.steps != 0) {
      float v = vin[j];
      uint32_t r = rin[j];
      uint64_t sp;
      if (v == 0.0f && r == 0 && cnt < (uint64_t)tbl_n) {
        const LifEntry e = ev[j];
        sp = e.spikes;
        v = e.v;
        r = e.r;
      } else {
        sp = lif_closed(lif_current(cnt, lp.steps), lp.steps, lp.thr, lp.leak, lp.refr, v, r);
      }
      sc += sp;
      if (!(fresh && derive)) {  // derived: a function of the count, not written
        V[i] = v;
        R[i] = r;
        SC[i] = sc;
      }
      my_sp += sp;
    } else if (fresh && !derive) {
      V[i] = 0.0f;
      R[i] = 0u;
      SC[i] = 0;
    }
    scv[j] = sc;
    if (sc8) sc8[i] = sc < 255 ? (uint8_t)sc : (uint8_t)255;  // the top-N passes' compact copy
    my_mx = sc > my_mx ? sc : my_mx;
    // neurons that never spiked (most of a large pool) are counted in a
    // register: same-address LDS atomics of a whole wave serialise
    if (sc == 0) ++n_zero;
  }
  // the histogram: bins the lanes of a wave share are added once per bin for
  // the two most common ones (a uniform pool -- a 12.5 Gbase config-4 shard,
  // every neuron spiking 333-334 times -- sent all 64 lanes to one LDS bin:
  // k_lif_apply 5 ms against 0.02 ms at config 2, profiles/r04_t3); the rest
  // one atomic per lane
#pragma unroll
  for (int j = 0; j < kLifPerThread; ++j) {
    const uint64_t sc = scv[j];
    const uint32_t bin = sc < (uint64_t)(kHistBins - 1) ? (uint32_t)sc : (uint32_t)(kHistBins - 1);
    bool pend = sc != 0;  // (i >= pool: scv 0)
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      const uint64_t m = __ballot(pend);
      if (!m) break;
      const uint32_t v = (uint32_t)__shfl((int)bin, __ffsll((long long)m) - 1, 64);
      const bool mine = pend && bin == v;
      const uint64_t same = __ballot(mine);
      if (mine) {
        if ((threadIdx.x & 63) == (uint32_t)(__ffsll((long long)same) - 1))
          atomicAdd(&sh[v], (uint32_t)__popcll(same));
        pend = false;
      }
    }
    if (pend) atomicAdd(&sh[bin], 1u);
  }
  // wave reductions
  for (int o = 32; o > 0; o >>= 1) {
    my_sp += __shfl_down(my_sp, o, 64);
    unsigned long long om = __shfl_down(my_mx, o, 64);
    my_mx = om > my_mx ? om : my_mx;
    n_zero += __shfl_down(n_zero, o, 64);
  }
  if ((threadIdx.x & 63) == 0 && n_zero) atomicAdd(&sh[0], n_zero);
  if ((threadIdx.x & 63) == 0) { s_sp[threadIdx.x >> 6] = my_sp; s_mx[threadIdx.x >> 6] = my_mx; }
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long a = 0, m = 0;
    for (int w = 0; w < kLifWaves; ++w) { a += s_sp[w]; m = s_mx[w] > m ? s_mx[w] : m; }
    if (a) atomicAdd(&stats[0], a);
    if (m) atomicMax(&stats[1], m);
  }
  // 8 copies of the global histogram (blocks b, b+8, ... share one), summed by
  // the threshold step: the hot spike-count bins see 8x fewer atomics each.
  // Bin 0 (never-spiking neurons: nearly all of a large pool) is not counted:
  // the threshold step takes it as the rest of the pool, so no block sends an
  // atomic to that one hot address
  if (!tf.want) {  // the separate top-N kernels read the global histogram
    uint32_t *hc = hist + (size_t)(blockIdx.x & (kHistCopies - 1)) * kHistBins;
    for (int i = threadIdx.x + 1; i < kHistBins; i += kLifBlock)
      if (sh[i]) atomicAdd(&hc[i], sh[i]);
    return;
  }
  // fused top-N: this block's candidates (the final step is k_top_final)
  if (!block_top(sh, scv, base, pool, tf.want, s_cand, tf.bcand + (uint64_t)blockIdx.x * tf.want,
                 tf.bcnt + blockIdx.x) &&
      threadIdx.x == 0)
    tf.bcnt[blockIdx.x] = kDeferMark;  // the final step defers to the host's exact path
}

// After the LIF kernel (the kernel boundary makes every block's candidates
// and currents visible): one block of kLifBlock threads.
__global__ __launch_bounds__(kLifBlock) void k_top_final(uint64_t pool,
                                                      const uint64_t *__restrict__ currents,
                                                      uint32_t nb, TopFuse tf) {
  final_top(pool, currents, nb, tf);
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
  // thread t owns bins [4095-4t-3, 4095-4t] i.e. counting from the top.  Bin
  // 0 is not counted by the LIF: it holds the rest of the pool's neurons
  auto bin_count = [&](int bin) -> unsigned long long {
    unsigned long long h = 0;
    for (int c = 0; c < kHistCopies; ++c) h += hist[c * kHistBins + bin];
    return h;
  };
  unsigned long long loc = 0;
  for (int j = 0; j < 4; ++j) {
    const int bin = kHistBins - 1 - (4 * t + j);
    if (bin) loc += bin_count(bin);
  }
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
  const unsigned long long spiking = part[1023];  // neurons in bins >= 1
  // the thread whose bins reach `want` (t = 1023 also when only bin 0 can)
  if (before < want && (part[t] >= want || (t == 1023 && spiking < want))) {
    unsigned long long cum = before;
    for (int j = 0; j < 4; ++j) {
      int bin = kHistBins - 1 - (4 * t + j);
      const unsigned long long h = bin ? bin_count(bin) : (pool > spiking ? pool - spiking : 0ull);
      if (cum + h >= want || bin == 0) {
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
__global__ __launch_bounds__(kBlock) void k_radix_hist(SpikeSrc sc, uint64_t pool,
                                                       int shift, uint64_t prefix,
                                                       uint32_t *__restrict__ h256) {
  __shared__ uint32_t sh[256];
  sh[threadIdx.x] = 0;
  __syncthreads();
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < pool;
       i += (uint64_t)gridDim.x * kBlock) {
    uint64_t v = spikes_at(sc, i);
    uint64_t hi = (shift + 8 >= 64) ? 0 : (v >> (shift + 8));
    if (hi == prefix) atomicAdd(&sh[(v >> shift) & 255], 1u);
  }
  __syncthreads();
  if (sh[threadIdx.x]) atomicAdd(&h256[threadIdx.x], sh[threadIdx.x]);
}

constexpr int kTopChunk = kBlock * 8;  // neurons per block in count/emit

// spike counts of neurons base .. base + 7 (0 past the pool): from the u8
// mirror with one 8-B load where aligned and whole
__device__ __forceinline__ void spikes8(const SpikeSrc &sc, uint64_t base, uint64_t pool,
                                        uint64_t (&v)[8]) {
  if (sc.sc8 && base + 8 <= pool && !((uintptr_t)(sc.sc8 + base) & 7)) {
    const uint2 w = *reinterpret_cast<const uint2 *>(sc.sc8 + base);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint32_t b = ((j < 4 ? w.x : w.y) >> (8 * (j & 3))) & 0xFFu;
      v[j] = b;
      if (b == 255u) v[j] = spikes_at(sc, base + j);  // 255 or more: the exact value
    }
    return;
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = base + j < pool ? spikes_at(sc, base + j) : 0;
}

// one pass over the spike counts: the rows above T are emitted (any order:
// k_topn_sort orders them) and each block's ties (== T) counted
__global__ __launch_bounds__(kBlock) void k_topn_count(SpikeSrc sc,
                                                       uint64_t pool, TopState *__restrict__ st,
                                                       uint32_t *__restrict__ tie_cnt,
                                                       TopCand *__restrict__ cand) {
  __shared__ uint32_t s[kBlock / 64];
  const uint64_t T = st->T;
  // thread t owns 8 consecutive neurons of the block's chunk (the u8 mirror:
  // one 8-B load per lane)
  const uint64_t base = (uint64_t)blockIdx.x * kTopChunk + (uint64_t)threadIdx.x * 8;
  uint64_t v[8];
  spikes8(sc, base, pool, v);
  uint32_t c = 0;
  for (int j = 0; j < 8; ++j) {
    const uint64_t i = base + j;
    if (i >= pool) break;
    if (v[j] == T) ++c;
    if (v[j] > T && T != ~0ULL) {
      const unsigned long long pos = atomicAdd((unsigned long long *)&st->emit_above, 1ull);
      if (pos < (unsigned long long)kMaxTopN) {  // (a threshold inconsistent with the counts
        cand[pos].idx = i;                        // must not write past the candidates)
        cand[pos].sc = v[j];
      }
    }
  }
  for (int o = 32; o > 0; o >>= 1) c += __shfl_down(c, o, 64);
  if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) tie_cnt[blockIdx.x] = s[0] + s[1] + s[2] + s[3];
}

// in-place exclusive scan of the per-block tie counts (one block; the counts
// sum to <= pool < 2^32).  The counts pass through LDS a piece at a time with
// coalesced loads; each thread sums a contiguous run of kPer entries of its
// piece from LDS, stored one pad word per kPer entries so that the runs of a
// wave's lanes start in different banks.
constexpr uint32_t kTieScanPiece = 16384;
__device__ __forceinline__ uint32_t tie_slot(uint32_t e) { return e + (e >> 4); }
__global__ __launch_bounds__(1024) void k_tie_scan(uint32_t *__restrict__ cnt, uint32_t n) {
  __shared__ uint32_t s_w[16];
  __shared__ uint32_t s_c[kTieScanPiece + kTieScanPiece / 16];
  constexpr uint32_t kPer = kTieScanPiece / 1024;  // 16: matches tie_slot's pad
  uint32_t carry = 0;
  for (uint32_t p0 = 0; p0 < n; p0 += kTieScanPiece) {
    const uint32_t m = n - p0 < kTieScanPiece ? n - p0 : kTieScanPiece;
    for (uint32_t i = threadIdx.x; i < m; i += 1024) s_c[tie_slot(i)] = cnt[p0 + i];
    __syncthreads();
    const uint32_t lo = threadIdx.x * kPer;
    uint32_t sum = 0;
    for (uint32_t i = lo; i < lo + kPer && i < m; ++i) sum += s_c[tie_slot(i)];
    uint32_t tot;
    uint32_t run = carry + block_excl_scan<uint32_t>(sum, s_w, &tot);
    for (uint32_t i = lo; i < lo + kPer && i < m; ++i) {
      const uint32_t x = s_c[tie_slot(i)];
      s_c[tie_slot(i)] = run;
      run += x;
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < m; i += 1024) cnt[p0 + i] = s_c[tie_slot(i)];
    carry += tot;
    __syncthreads();
  }
}

// the first `need` ties in index order (the rows above T were emitted by
// k_topn_count): only blocks whose earlier ties fall short of `need` read
// their spike counts
__global__ __launch_bounds__(kBlock) void k_topn_emit(SpikeSrc sc,
                                                      uint64_t pool, TopState *__restrict__ st,
                                                      const uint32_t *__restrict__ tie_cnt,
                                                      TopCand *__restrict__ cand) {
  __shared__ uint32_t s_scan[kBlock];
  const uint64_t T = st->T, need = st->need, n_above = st->n_above;
  // ties in earlier blocks (k_tie_scan turned the counts into an exclusive scan)
  const unsigned long long prefix = tie_cnt[blockIdx.x];
  if (prefix >= need) return;  // uniform across the block
  // thread t owns 8 consecutive neurons -> ranks in index order
  const uint64_t base = (uint64_t)blockIdx.x * kTopChunk + (uint64_t)threadIdx.x * 8;
  uint32_t ties = 0;
  uint64_t v[8];
  spikes8(sc, base, pool, v);
  for (int j = 0; j < 8; ++j) {
    uint64_t i = base + j;
    if (i < pool && v[j] == T) ++ties;
  }
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


// exact final order of the <= kMaxTopN candidates: bitonic sort in LDS
__global__ __launch_bounds__(1024) void k_topn_sort(TopCand *__restrict__ cand, uint32_t m, uint64_t n,
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
    top_cur[i] = s[i].idx < n ? currents[s[i].idx] : 0ull;  // (an unfilled row: the caller checks)
  }
}

// ---------------------------------------------------------------------------
// device hash set helpers (uniques of the top-N neurons)
// ---------------------------------------------------------------------------
__global__ void k_set_fill(unsigned long long *__restrict__ keys, const uint64_t *__restrict__ mask) {
  const uint64_t cap = *mask + 1;
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

__global__ void k_set_merge(MergeSrc m, FastMod fm, UniqArgs u) {
  extern __shared__ uint64_t dyn[];
  __shared__ unsigned long long seen[kSeen];
  uint64_t *tbl_idx = dyn;
  uint32_t *tbl_slot = reinterpret_cast<uint32_t *>(dyn + u.tbl_size);
  seen_init(seen);
  build_top_tbl(u, tbl_idx, tbl_slot);
  const uint64_t n = m.world ? (uint64_t)m.world * m.cap : m.n;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t *at;
    if (!merge_src_key(m, i, 1, &at)) continue;
    uint64_t key = *at;
    uint64_t idx = fastmod(sip13_u64(key), fm);
    int slot = probe_top(tbl_idx, tbl_slot, u.tbl_size - 1, idx);
    if (slot >= 0 && (key == kEmpty || !seen_before(seen, key))) set_insert(u, (uint32_t)slot, key);
  }
}

// [n, keys...] with min(n, cap) keys of wpk words each (the all-gather form)
__global__ void k_pad_keys(const uint64_t *__restrict__ src, const unsigned long long *__restrict__ n_src,
                           uint64_t cap, int wpk, uint64_t *__restrict__ dst) {
  const uint64_t n = *n_src;
  const uint64_t w = (n < cap ? n : cap) * (uint64_t)wpk;
  if (blockIdx.x == 0 && threadIdx.x == 0) dst[0] = n;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < w;
       i += (uint64_t)gridDim.x * blockDim.x)
    dst[1 + i] = src[i];
}

// ---------------------------------------------------------------------------
// Multi-GPU step with one host synchronisation (neurokmer_amd/dist.py::
// finalize_step): the currents cross the wire as u32, the LIF reads them back
// from the reduced wire vector, and this shard's distinct top k-mers go
// straight into its all-gather segment [hdr, keys...] with hdr = n | flags << 56
// (flags: 1 set too small, 2 top bucket overflowed, 4 top-N deferred to the
// host refine), so every rank sees every rank's reasons to redo the slow way.
// ---------------------------------------------------------------------------
// over != nullptr (partitioned count): the zeroed currents only hold the
// direct adds of overflowed buckets, so only those buckets are read
__global__ void k_wire32(const uint64_t *__restrict__ cur, const uint32_t *__restrict__ partials,
                         uint32_t slices, const uint32_t *__restrict__ over, int over_bits,
                         uint64_t pool, uint32_t *__restrict__ wire) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < pool;
       i += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t x = (!over || over[i >> over_bits]) ? cur[i] : 0ull;
    for (uint32_t r = 0; r < slices; ++r) x += partials[(uint64_t)r * pool + i];
    wire[i] = (uint32_t)x;
  }
}

__global__ void k_export_keys(const unsigned long long *__restrict__ S,
                              const uint64_t *__restrict__ set_mask, int w128, uint64_t cap_out,
                              uint64_t *__restrict__ dst, unsigned long long *__restrict__ count) {
  const uint64_t n = *set_mask + 1;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x) {
    if (w128) {
      const unsigned long long w0 = S[3 * i];
      if (!w0) continue;
      const Key128 k = words_key128(w0, S[3 * i + 1], S[3 * i + 2]);
      const unsigned long long at = atomicAdd(count, 1ull);
      if (at < cap_out) {
        dst[1 + 2 * at] = k.lo;
        dst[2 + 2 * at] = k.hi;
      }
    } else {
      const unsigned long long kk = S[i];
      if (kk == kEmpty) continue;
      const unsigned long long at = atomicAdd(count, 1ull);
      if (at < cap_out) dst[1 + at] = kk;
    }
  }
}

// the segment header (one lane) and, with mp.S, the next merge's prep (the
// whole grid: one launch fewer between the export and the merge)
__global__ void k_export_hdr(unsigned long long *__restrict__ count, const uint32_t *__restrict__ special,
                             uint32_t n_top, const TopState *__restrict__ st,
                             const uint32_t *__restrict__ post_flags, int w128, uint64_t cap_out,
                             uint64_t *__restrict__ dst, MergePrep mp) {
  if (mp.S) {
    const uint64_t nw = w128 ? 3 * mp.cap : mp.cap;
    const unsigned long long fill = w128 ? 0ull : kEmpty;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nw;
         i += (uint64_t)gridDim.x * blockDim.x)
      mp.S[i] = fill;
    if (blockIdx.x == 0) {
      for (uint32_t t = threadIdx.x; t < mp.m; t += blockDim.x) {
        mp.uniq[t] = 0;
        mp.special[t] = 0;
      }
      if (threadIdx.x == 0) {
        *mp.mask = mp.cap - 1;
        *mp.trunc = 0;
      }
    }
  }
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  uint64_t n = *count;
  *count = 0;  // ready for the next export
  uint64_t flags = (st && st->refine) ? 4u : 0u;
  if (post_flags) flags |= (post_flags[0] ? 1u : 0u) | (post_flags[1] ? 2u : 0u);
  if (!w128 && post_flags && !(st && st->refine)) {  // the kEmpty key lives outside the set
    bool any = false;
    for (uint32_t s = 0; s < n_top; ++s) any |= special[s] != 0;
    if (any) {
      if (n < cap_out) dst[1 + n] = kEmpty;
      ++n;
    }
  }
  dst[0] = n | (flags << 56);
}

// Everything a merge starts from, in one launch: the set emptied at capacity
// cap (3 words per key for 128-bit keys), its mask word, the uniques column,
// the kEmpty flags and the truncation word zeroed.
__global__ void k_merge_prep(unsigned long long *__restrict__ S, uint64_t *__restrict__ mask,
                             uint64_t cap, int w128, uint32_t *__restrict__ uniq,
                             uint32_t *__restrict__ special, uint32_t m, uint32_t *__restrict__ trunc) {
  const uint64_t n = w128 ? 3 * cap : cap;
  const unsigned long long fill = w128 ? 0ull : kEmpty;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x)
    S[i] = fill;
  if (blockIdx.x == 0) {
    for (uint32_t t = threadIdx.x; t < m; t += blockDim.x) {
      uniq[t] = 0;
      special[t] = 0;
    }
    if (threadIdx.x == 0) {
      *mask = cap - 1;
      *trunc = 0;
    }
  }
}

hipError_t launch_merge_prep(unsigned long long *set_keys, uint64_t *mask, uint64_t cap, int w128,
                             uint32_t *uniq, uint32_t *special, uint32_t m, uint32_t *trunc,
                             hipStream_t s) {
  unsigned g = (unsigned)(((w128 ? 3 : 1) * cap + 255) / 256);
  if (g > 2048) g = 2048;
  if (!g) g = 1;
  hipLaunchKernelGGL(k_merge_prep, dim3(g), dim3(256), 0, s, set_keys, mask, cap, w128, uniq, special,
                     m, trunc);
  return hipGetLastError();
}

hipError_t launch_wire32(const uint64_t *cur, const uint32_t *partials, uint32_t slices,
                         const uint32_t *over, int over_bits, uint64_t pool, uint32_t *wire,
                         hipStream_t s) {
  if (!pool) return hipSuccess;
  unsigned g = (unsigned)((pool + 255) / 256);
  if (g > 8192) g = 8192;
  hipLaunchKernelGGL(k_wire32, dim3(g), dim3(256), 0, s, cur, partials, slices, over, over_bits, pool,
                     wire);
  return hipGetLastError();
}

hipError_t launch_export(const unsigned long long *set_keys, const uint64_t *set_mask,
                         uint64_t set_alloc, int w128, bool uniq, bool appended,
                         const uint32_t *special, uint32_t n_top, const TopState *st,
                         const uint32_t *post_flags, uint64_t cap_out, uint64_t *dst,
                         unsigned long long *count, hipStream_t s, const MergePrep &mp) {
  if (uniq && !appended) {  // scan the set; grid for the largest capacity, blocks past *set_mask + 1 idle
    unsigned g = (unsigned)((set_alloc + 255) / 256);
    if (g > 1024) g = 1024;
    hipLaunchKernelGGL(k_export_keys, dim3(g), dim3(256), 0, s, set_keys, set_mask, w128, cap_out,
                       dst, count);
  }
  unsigned g = 1, b = 1;
  if (mp.S) {
    g = (unsigned)std::min<uint64_t>(((w128 ? 3 : 1) * mp.cap + 255) / 256, 2048);
    b = 256;
  }
  hipLaunchKernelGGL(k_export_hdr, dim3(g ? g : 1), dim3(b), 0, s, count, special, n_top, st,
                     uniq ? post_flags : nullptr, w128, cap_out, dst, mp);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
uint64_t n_tiles_for(uint64_t n_bases, uint64_t tile) { return (n_bases + tile - 1) / tile; }

uint64_t top_tbl_size(uint32_t n_top) {
  uint64_t s = 64;
  while (s < 2ull * n_top) s <<= 1;
  return s;
}

static size_t tbl_bytes(const UniqArgs &u) { return (size_t)u.tbl_size * (8 + 4); }

hipError_t launch_tile_rec(const KmerInput &in, uint64_t tile_size, uint32_t *tile_rec,
                           hipStream_t s) {
  if (!in.n_tiles) return hipSuccess;
  unsigned g = (unsigned)((in.n_tiles + 255) / 256);
  hipLaunchKernelGGL(k_tile_rec, dim3(g), dim3(256), 0, s, in.offsets, in.n_recs, in.n_tiles,
                     tile_size, in.tile_base, tile_rec);
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

uint32_t lif_blocks(uint64_t pool) {
  const uint64_t per = (uint64_t)kLifBlock * kLifPerThread;
  return (uint32_t)((pool + per - 1) / per);
}

hipError_t launch_lif_derive(const uint64_t *currents, float *v, uint32_t *r, uint64_t *sc,
                             uint64_t pool, LifParams lp, const LifEntry *tbl, int tbl_n,
                             hipStream_t s) {
  if (!pool) return hipSuccess;
  unsigned g = (unsigned)((pool + 255) / 256);
  if (g > 8192) g = 8192;
  hipLaunchKernelGGL(k_lif_derive, dim3(g), dim3(256), 0, s, currents, v, r, sc, pool, lp, tbl, tbl_n);
  return hipGetLastError();
}

hipError_t launch_lif_apply(uint64_t *currents, const uint32_t *partials, uint32_t slices,
                            int cur_zero, const uint32_t *over, int over_bits, int fresh, int derive,
                            float *v, uint32_t *r, uint64_t *sc, uint64_t pool, LifParams lp,
                            const LifEntry *tbl, int tbl_n, uint32_t *hist, uint64_t *stats,
                            const TopFuse &tf, hipStream_t s, uint8_t *sc8) {
  if (!pool) return hipSuccess;
  const unsigned g = lif_blocks(pool);
  if (tf.want && (tf.want > kFuseMaxTopN || g > kFuseMaxBlocks || pool > (1ull << 24)))
    return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_lif_apply, dim3(g), dim3(kLifBlock), 0, s, currents, partials, slices, cur_zero, over, over_bits, fresh, derive,
                     v, r, sc, pool, lp, tbl, tbl_n, hist, (unsigned long long *)stats, tf, sc8);
  if (tf.want)
    hipLaunchKernelGGL(k_top_final, dim3(1), dim3(kLifBlock), 0, s, pool, currents, g, tf);
  return hipGetLastError();
}

hipError_t launch_topn_threshold(const uint32_t *hist, uint64_t n, uint64_t pool, TopState *st,
                                 hipStream_t s) {
  hipLaunchKernelGGL(k_topn_threshold, dim3(1), dim3(1024), 0, s, hist, n, pool, st);
  return hipGetLastError();
}

hipError_t launch_radix_hist(const SpikeSrc &sc, uint64_t pool, int shift, uint64_t prefix,
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

hipError_t launch_topn_count(const SpikeSrc &sc, uint64_t pool, TopState *st,
                             uint32_t *tie_cnt, TopCand *cand, hipStream_t s) {
  if (!pool) return hipSuccess;
  hipLaunchKernelGGL(k_topn_count, dim3(topn_blocks(pool)), dim3(kBlock), 0, s, sc, pool, st,
                     tie_cnt, cand);
  hipLaunchKernelGGL(k_tie_scan, dim3(1), dim3(1024), 0, s, tie_cnt, (uint32_t)topn_blocks(pool));
  return hipGetLastError();
}

hipError_t launch_topn_emit(const SpikeSrc &sc, uint64_t pool, TopState *st,
                            const uint32_t *tie_cnt, TopCand *cand, hipStream_t s) {
  if (!pool) return hipSuccess;
  hipLaunchKernelGGL(k_topn_emit, dim3(topn_blocks(pool)), dim3(kBlock), 0, s, sc, pool, st,
                     tie_cnt, cand);
  return hipGetLastError();
}

hipError_t launch_topn_sort(TopCand *cand, uint32_t m, uint64_t n, const uint64_t *currents,
                            uint64_t *top_cur, hipStream_t s) {
  if (!m) return hipSuccess;
  hipLaunchKernelGGL(k_topn_sort, dim3(1), dim3(1024), 0, s, cand, m, n, currents, top_cur);
  return hipGetLastError();
}

hipError_t launch_set_fill(unsigned long long *keys, const uint64_t *mask, uint64_t max_cap,
                           hipStream_t s) {
  unsigned g = (unsigned)((max_cap + 255) / 256);
  if (g > 2048) g = 2048;
  if (!g) return hipSuccess;
  hipLaunchKernelGGL(k_set_fill, dim3(g), dim3(256), 0, s, keys, mask);
  return hipGetLastError();
}

// --kmer-width=128
template <int MODE>
static hipError_t launch_kmers128(const KmerInput &in, int k, int canonical, uint64_t pool,
                                  unsigned long long *cur, const UniqArgs &u, hipStream_t s) {
  if (!in.n_tiles) return hipSuccess;
  if (k < 1 || k > 64) return hipErrorInvalidValue;
  FastMod fm = make_fastmod(pool);
  dim3 g((unsigned)in.n_tiles), b(kBlock);
  size_t dyn = MODE == 1 ? tbl_bytes(u) : 0;
  if (canonical) hipLaunchKernelGGL((k_kmers128<true, MODE>), g, b, dyn, s, in, k, fm, cur, u);
  else hipLaunchKernelGGL((k_kmers128<false, MODE>), g, b, dyn, s, in, k, fm, cur, u);
  return hipGetLastError();
}
hipError_t launch_uniq_gen(const KmerInput &in, int k, int canonical, int km, uint64_t pool,
                           const UniqArgs &u, hipStream_t s, const uint32_t *tiles,
                           const uint32_t *n_list, uint32_t max_list) {
  if (!in.n_tiles) return hipSuccess;
  if (km < 0 || km > 2 || k < 1 || k > 64 || (km == 0 && k > 32) || (km == 1 && k <= 32))
    return hipErrorInvalidValue;
  const FastMod fm = make_fastmod(pool);
  const uint64_t nb = tiles ? std::min<uint64_t>(max_list, in.n_tiles) : in.n_tiles;
  if (!nb) return hipSuccess;
  const dim3 g((unsigned)nb), b(kPartBlock);
  const size_t dyn = tbl_bytes(u);
#define NK_UG(KM_, C_) hipLaunchKernelGGL((k_uniq_gen<KM_, C_>), g, b, dyn, s, in, k, fm, u, tiles, n_list)
  if (canonical) {
    if (km == 0) NK_UG(0, true);
    else if (km == 1) NK_UG(1, true);
    else NK_UG(2, true);
  } else {
    if (km == 0) NK_UG(0, false);
    else if (km == 1) NK_UG(1, false);
    else NK_UG(2, false);
  }
#undef NK_UG
  return hipGetLastError();
}

hipError_t launch_uniq_lanes(const KmerInput &in, int k, int canonical, int km, uint64_t pool,
                             const UniqArgs &u, const uint32_t *list, const uint32_t *n_list,
                             uint32_t max_list, hipStream_t s) {
  if (!in.n_tiles || !max_list) return hipSuccess;
  if (km < 0 || km > 2 || k < 1 || k > 64 || (km == 0 && k > 32) || (km == 1 && k <= 32))
    return hipErrorInvalidValue;
  const FastMod fm = make_fastmod(pool);
  const dim3 g((unsigned)std::min<uint64_t>((max_list + 255) / 256, 1024)), b(256);
  const size_t dyn = tbl_bytes(u);
#define NK_UL(KM_, C_) hipLaunchKernelGGL((k_uniq_lanes<KM_, C_>), g, b, dyn, s, in, k, fm, u, list, n_list, max_list)
  if (canonical) {
    if (km == 0) NK_UL(0, true);
    else if (km == 1) NK_UL(1, true);
    else NK_UL(2, true);
  } else {
    if (km == 0) NK_UL(0, false);
    else if (km == 1) NK_UL(1, false);
    else NK_UL(2, false);
  }
#undef NK_UL
  return hipGetLastError();
}

hipError_t launch_count128(const KmerInput &in, int k, int canonical, uint64_t pool,
                           uint64_t *currents, hipStream_t s) {
  UniqArgs u{};
  return launch_kmers128<0>(in, k, canonical, pool, (unsigned long long *)currents, u, s);
}
hipError_t launch_uniques128(const KmerInput &in, int k, int canonical, uint64_t pool,
                             const UniqArgs &u, hipStream_t s) {
  return launch_kmers128<1>(in, k, canonical, pool, nullptr, u, s);
}
hipError_t launch_set_fill128(unsigned long long *set3, const uint64_t *mask, uint64_t max_cap,
                              hipStream_t s) {
  unsigned g = (unsigned)((3 * max_cap + 255) / 256);
  if (g > 2048) g = 2048;
  if (!g) return hipSuccess;
  hipLaunchKernelGGL(k_set_fill128, dim3(g), dim3(256), 0, s, set3, mask);
  return hipGetLastError();
}
hipError_t launch_set_compact128(const unsigned long long *set3, uint64_t cap, uint64_t *out,
                                 unsigned long long *count, hipStream_t s) {
  unsigned g = (unsigned)((cap + 255) / 256);
  if (g > 4096) g = 4096;
  if (!g) g = 1;
  hipLaunchKernelGGL(k_set_compact128, dim3(g), dim3(256), 0, s, set3, cap, out, count);
  return hipGetLastError();
}
hipError_t launch_set_merge128(const MergeSrc &m, uint64_t pool, const UniqArgs &u, hipStream_t s) {
  const uint64_t n = m.world ? (uint64_t)m.world * m.cap : m.n;
  if (!n) return hipSuccess;
  unsigned g = (unsigned)((n + 255) / 256);
  if (g > 2048) g = 2048;
  hipLaunchKernelGGL(k_set_merge128, dim3(g), dim3(256), tbl_bytes(u), s, m, make_fastmod(pool), u);
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

hipError_t launch_set_merge(const MergeSrc &m, uint64_t pool, const UniqArgs &u, hipStream_t s) {
  const uint64_t n = m.world ? (uint64_t)m.world * m.cap : m.n;
  if (!n) return hipSuccess;
  unsigned g = (unsigned)((n + 255) / 256);
  if (g > 2048) g = 2048;
  hipLaunchKernelGGL(k_set_merge, dim3(g), dim3(256), tbl_bytes(u), s, m, make_fastmod(pool), u);
  return hipGetLastError();
}

hipError_t launch_pad_keys(const uint64_t *src, const unsigned long long *n_src, uint64_t cap,
                           int wpk, uint64_t *dst, hipStream_t s) {
  unsigned g = (unsigned)((cap * wpk + 255) / 256);
  if (g > 1024) g = 1024;
  if (!g) g = 1;
  hipLaunchKernelGGL(k_pad_keys, dim3(g), dim3(256), 0, s, src, n_src, cap, wpk, dst);
  return hipGetLastError();
}

hipError_t launch_part(const KmerInput &in, int k, int canonical, uint64_t pool,
                       const PartArgs &pa, hipStream_t s) {
  if (!in.n_tiles) return hipSuccess;
  FastMod fm = make_fastmod(pool);
  const dim3 g((unsigned)in.n_tiles), bl(kPartBlock);
  const size_t dyn = 0;
  if (pa.n_buckets > (uint32_t)kMaxBuckets) return hipErrorInvalidValue;
  if (pa.key) {  // the exact table's records (key beside the bin offset)
    if (!pa.spill || !pa.n_spill) return hipErrorInvalidValue;
    if (pa.n_buckets <= 256) {
      if (canonical && k >= 16) hipLaunchKernelGGL((k_part<true, 256, true, true>), g, bl, dyn, s, in, k, fm, pa);
      else if (canonical) hipLaunchKernelGGL((k_part<true, 256, false, true>), g, bl, dyn, s, in, k, fm, pa);
      else hipLaunchKernelGGL((k_part<false, 256, false, true>), g, bl, dyn, s, in, k, fm, pa);
    } else {
      if (canonical) hipLaunchKernelGGL((k_part<true, kMaxBuckets, false, true>), g, bl, dyn, s, in, k, fm, pa);
      else hipLaunchKernelGGL((k_part<false, kMaxBuckets, false, true>), g, bl, dyn, s, in, k, fm, pa);
    }
    return hipGetLastError();
  }
  if (pa.n_buckets <= 256) {
#if !defined(NK_K1A_NO_K16)  // (A/B: the masked low word)
    if (canonical && k >= 16) hipLaunchKernelGGL((k_part<true, 256, true>), g, bl, dyn, s, in, k, fm, pa);
    else
#endif
    if (canonical) hipLaunchKernelGGL((k_part<true, 256>), g, bl, dyn, s, in, k, fm, pa);
    else hipLaunchKernelGGL((k_part<false, 256>), g, bl, dyn, s, in, k, fm, pa);
  } else {
    if (canonical) hipLaunchKernelGGL((k_part<true, kMaxBuckets>), g, bl, dyn, s, in, k, fm, pa);
    else hipLaunchKernelGGL((k_part<false, kMaxBuckets>), g, bl, dyn, s, in, k, fm, pa);
  }
  return hipGetLastError();
}

bool part_fused_ok(const PartArgs &pa) {
  return pa.n_buckets <= 256 && !pa.key && pa.bin_bits == (uint32_t)kBinBits;
}

hipError_t launch_part_fused(const KmerInput &in, int k, int canonical, uint64_t pool,
                             const PartArgs &pa, const HistJob &hj, hipStream_t s) {
  if (!in.n_tiles) return hipSuccess;
  if (!part_fused_ok(pa) || (hj.n_items && (hj.n_host == 0 || hj.n_host > in.n_tiles || !hj.partials ||
                                             !hj.off || !hj.fill || !hj.slices ||
                                             hj.n_buckets > (uint32_t)kMaxBuckets)))
    return hipErrorInvalidValue;
  const FastMod fm = make_fastmod(pool);
  const dim3 g((unsigned)in.n_tiles), bl(kPartBlock);
  if (canonical && k >= 16) hipLaunchKernelGGL((k_part_fused<true, true>), g, bl, 0, s, in, k, fm, pa, hj);
  else if (canonical) hipLaunchKernelGGL((k_part_fused<true, false>), g, bl, 0, s, in, k, fm, pa, hj);
  else hipLaunchKernelGGL((k_part_fused<false, false>), g, bl, 0, s, in, k, fm, pa, hj);
  return hipGetLastError();
}

hipError_t launch_bucket_hist(const PartArgs &pa, uint64_t pool, uint32_t slices,
                              uint32_t *partials, hipStream_t s) {
  if (!pa.n_buckets) return hipSuccess;
  const dim3 g(pa.n_buckets, slices);
  if (pa.lif.sc8) {  // the fused LIF: write-through only
    if (partials || !pa.out || slices != 1 || pa.bin_bits != 15) return hipErrorInvalidValue;
    hipLaunchKernelGGL((k_bucket_hist<15, NK_HIST_KU, true>), g, dim3(kHistBlock), 0, s, pa, pool, slices,
                       partials);
    return hipGetLastError();
  }
  switch (pa.bin_bits) {
    case 12: hipLaunchKernelGGL(k_bucket_hist<12>, g, dim3(kHistBlock), 0, s, pa, pool, slices, partials); break;
    case 13: hipLaunchKernelGGL(k_bucket_hist<13>, g, dim3(kHistBlock), 0, s, pa, pool, slices, partials); break;
    case 14: hipLaunchKernelGGL(k_bucket_hist<14>, g, dim3(kHistBlock), 0, s, pa, pool, slices, partials); break;
    case 15: hipLaunchKernelGGL(k_bucket_hist<15>, g, dim3(kHistBlock), 0, s, pa, pool, slices, partials); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_partials_add(const uint32_t *partials, uint32_t slices, uint64_t pool,
                               uint64_t *currents, hipStream_t s) {
  unsigned g = (unsigned)((pool + 255) / 256);
  if (g > 4096) g = 4096;
  if (!g) return hipSuccess;
  hipLaunchKernelGGL(k_partials_add, dim3(g), dim3(256), 0, s, partials, slices, pool,
                     (unsigned long long *)currents);
  return hipGetLastError();
}

// Diagnostic (measure, do not estimate): the cost of
// recomputing every kept record's key from its position, as an exact-table
// pass without K1a<KEYS>'s 8-B key per record would have to.  One workgroup
// per (slice, virtual bucket): each thread takes 8-record groups, finds the
// group's segment (tile) in an LDS copy of the slice's descriptors, loads the
// 8 positions and recomputes the keys from the bases (vec_window_key, as the
// uniques scan does for its hits); the keys are XOR-folded into *sink.
constexpr int kGatherTab = 4096;
template <bool CANON>
__global__ __launch_bounds__(256) void k_diag_key_gather(KmerInput in, int k, PartArgs pa,
                                                         uint32_t slices,
                                                         unsigned long long *__restrict__ sink) {
  __shared__ uint32_t tab[kGatherTab];
  __shared__ uint64_t s_seg[2];
  const uint64_t v = blockIdx.y, r = blockIdx.x;
  uint64_t n = pa.fill[v] & ((1ull << 40) - 1);
  if (n > pa.cap) n = pa.cap;
  uint64_t n_seg = pa.fill[v] >> 40;
  if (n_seg > pa.max_segs) n_seg = pa.max_segs;
  const uint64_t lo = (n * r / slices) & ~7ull;
  const uint64_t hi = r + 1 == slices ? n : (n * (r + 1) / slices) & ~7ull;
  if (lo >= hi || !n_seg) return;
  const uint2 *d = pa.desc + v * pa.max_segs;
  if (threadIdx.x < 128) {
    const uint64_t a = wave_search_le(d, n_seg, threadIdx.x < 64 ? lo : hi - 1);
    if ((threadIdx.x & 63) == 0) s_seg[threadIdx.x >> 6] = a;
  }
  __syncthreads();
  const uint64_t s0 = s_seg[0], ns = s_seg[1] - s0 + 1;
  const bool staged = ns <= (uint64_t)kGatherTab;
  if (staged)
    for (uint32_t j = threadIdx.x; j < ns; j += blockDim.x) tab[j] = d[s0 + j].y;
  __syncthreads();
  const uint16_t *off = pa.off + v * pa.cap, *pos = pa.pos + v * pa.cap;
  unsigned long long acc = 0;
  for (uint64_t g = lo / 8 + threadIdx.x; g < hi / 8; g += blockDim.x) {
    const uint64_t i = g * 8;
    uint64_t a = 0, z = ns;  // last segment whose first record <= i
    while (z - a > 1) {
      const uint64_t m = (a + z) >> 1;
      if ((staged ? (uint64_t)tab[m] : (uint64_t)d[s0 + m].y) <= i) a = m;
      else z = m;
    }
    const uint64_t t0 = (uint64_t)d[s0 + a].x * kPartTile;
    const uint4 o = *reinterpret_cast<const uint4 *>(off + i);
    const uint4 q = *reinterpret_cast<const uint4 *>(pos + i);
    const uint32_t ow[4] = {o.x, o.y, o.z, o.w}, qw[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (((ow[j >> 1] >> (16 * (j & 1))) & 0xFFFFu) == kPadOff) continue;
      const uint64_t p = t0 + ((qw[j >> 1] >> (16 * (j & 1))) & 0xFFFFu);
      acc ^= vec_window_key<CANON>(in.bases, in.n_bases, p, k);
    }
  }
  for (int o = 32; o; o >>= 1) acc ^= __shfl_xor(acc, o, 64);
  if ((threadIdx.x & 63) == 0 && acc) atomicXor(sink, acc);
}

hipError_t launch_diag_key_gather(const KmerInput &in, int k, int canonical, const PartArgs &pa,
                                  unsigned long long *sink, hipStream_t s) {
  if (!pa.desc || !pa.pos || k > 32) return hipErrorInvalidValue;
  const uint64_t V = (uint64_t)pa.n_buckets << pa.sub_shift;
  const uint32_t slices = (uint32_t)std::max<uint64_t>(1, 4096 / V);
  const dim3 g(slices, (unsigned)V);
  if (canonical)
    hipLaunchKernelGGL(k_diag_key_gather<true>, g, dim3(256), 0, s, in, k, pa, slices, sink);
  else
    hipLaunchKernelGGL(k_diag_key_gather<false>, g, dim3(256), 0, s, in, k, pa, slices, sink);
  return hipGetLastError();
}

// the set must be empty (kEmpty) up to *u.set_mask: the caller clears it
hipError_t launch_part_uniques(const KmerInput &in, int k, int canonical, const PartArgs &pa,
                               const UniqArgs &u, const uint32_t *tbuckets, const uint32_t *n_tb,
                               uint32_t max_tb, uint32_t slices, hipStream_t s) {
  if (!max_tb) return hipSuccess;
  if (canonical)
    hipLaunchKernelGGL(k_uniq_scan<true>, dim3(slices, max_tb), dim3(kHistBlock), 0, s, in, k, pa,
                       u, tbuckets, n_tb, slices);
  else
    hipLaunchKernelGGL(k_uniq_scan<false>, dim3(slices, max_tb), dim3(kHistBlock), 0, s, in, k, pa,
                       u, tbuckets, n_tb, slices);
  return hipGetLastError();
}

// After the top-N sort: size the uniques hash set from the top rows' currents
// (distinct keys <= their sum), list the distinct buckets holding top rows and
// flag the rare cases the host must redo (set too small, a top bucket whose
// region overflowed).  One block.
__global__ __launch_bounds__(1024) void k_top_post(const TopCand *__restrict__ top,
                                                   const uint64_t *__restrict__ top_cur,
                                                   uint32_t m, PostArgs pa) {
  top_post_block(top, top_cur, m, pa);
}

hipError_t launch_top_post(const TopCand *top, const uint64_t *top_cur, uint32_t m,
                           uint64_t set_alloc, const uint32_t *overflow, int part,
                           uint64_t *set_mask, uint32_t *tbuckets, uint32_t *flags,
                           uint32_t *uniq, uint32_t *special, unsigned long long *n_hits,
                           uint32_t bin_bits, hipStream_t s, uint32_t n_over) {
  PostArgs pa{set_alloc, overflow, part, set_mask, tbuckets, flags, uniq, special, n_hits, bin_bits,
              n_over};
  hipLaunchKernelGGL(k_top_post, dim3(1), dim3(1024), 0, s, top, top_cur, m, pa);
  return hipGetLastError();
}

__global__ void k_set_word(uint64_t *__restrict__ w, uint64_t v) { *w = v; }
hipError_t launch_set_word(uint64_t *w, uint64_t v, hipStream_t s) {
  hipLaunchKernelGGL(k_set_word, dim3(1), dim3(1), 0, s, w, v);
  return hipGetLastError();
}

// One launch zeroes up to kZeroMax buffers (16-B stores for the bulk).
__global__ void k_zero(ZeroList z) {
  const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (int b = 0; b < z.n; ++b) {
    uint8_t *p = (uint8_t *)z.ptr[b];
    const uint64_t n = z.bytes[b];
    const uint32_t f = 0x01010101u * z.fill[b];
    const uint64_t n16 = ((uintptr_t)p & 15) ? 0 : n / 16;
    for (uint64_t i = tid; i < n16; i += stride) reinterpret_cast<uint4 *>(p)[i] = make_uint4(f, f, f, f);
    for (uint64_t i = n16 * 16 + tid; i < n; i += stride) p[i] = (uint8_t)f;
  }
}

// tile -> first record (blocks [0, tr_blocks)) + the zero list (the rest)
__global__ void k_prep(const uint64_t *__restrict__ offsets, uint64_t n_recs, uint64_t n_tiles,
                       uint64_t tile_size, uint64_t tile_base, uint32_t *__restrict__ tile_rec,
                       unsigned tr_blocks, ZeroList z, unsigned long long *span) {
  if (span && blockIdx.x == 0 && threadIdx.x < 2) span[threadIdx.x] = threadIdx.x ? 0ull : ~0ull;
  if (blockIdx.x < tr_blocks) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n_tiles) return;
    const uint64_t pos = (tile_base + t) * tile_size;
    uint64_t lo = 0, hi = n_recs;
    while (hi - lo > 1) {
      const uint64_t mid = (lo + hi) >> 1;
      if (offsets[mid] <= pos) lo = mid;
      else hi = mid;
    }
    tile_rec[t] = (uint32_t)lo;
    return;
  }
  const uint64_t tid = (uint64_t)(blockIdx.x - tr_blocks) * blockDim.x + threadIdx.x;
  const uint64_t stride = (uint64_t)(gridDim.x - tr_blocks) * blockDim.x;
  for (int b = 0; b < z.n; ++b) {
    uint8_t *p = (uint8_t *)z.ptr[b];
    const uint64_t n = z.bytes[b];
    const uint32_t f = 0x01010101u * z.fill[b];
    const uint64_t n16 = ((uintptr_t)p & 15) ? 0 : n / 16;
    for (uint64_t i = tid; i < n16; i += stride) reinterpret_cast<uint4 *>(p)[i] = make_uint4(f, f, f, f);
    for (uint64_t i = n16 * 16 + tid; i < n; i += stride) p[i] = (uint8_t)f;
  }
}

hipError_t launch_prep(const KmerInput &in, uint64_t tile_size, uint32_t *tile_rec,
                       const ZeroList &z, hipStream_t s, unsigned long long *span) {
  uint64_t tot = 0;
  for (int b = 0; b < z.n; ++b) tot += z.bytes[b];
  const unsigned tr = (unsigned)((in.n_tiles + 255) / 256);
  unsigned g = (unsigned)((tot / 16 + 255) / 256);
  if (g > 1024) g = 1024;
  if (!g) g = 1;
  hipLaunchKernelGGL(k_prep, dim3(tr + g), dim3(256), 0, s, in.offsets, in.n_recs, in.n_tiles,
                     tile_size, in.tile_base, tile_rec, tr, z, span);
  return hipGetLastError();
}

hipError_t launch_zero(const ZeroList &z, hipStream_t s) {
  uint64_t tot = 0;
  for (int b = 0; b < z.n; ++b) tot += z.bytes[b];
  if (!tot) return hipSuccess;
  unsigned g = (unsigned)((tot / 16 + 255) / 256);
  if (g > 2048) g = 2048;
  if (!g) g = 1;
  hipLaunchKernelGGL(k_zero, dim3(g), dim3(256), 0, s, z);
  return hipGetLastError();
}

// Everything the host needs after a finalize, written straight into mapped
// host memory: [TopState | stats[2] | set mask | flags[4] | cand[m] | uniq[m]],
// then the completion word `done = seq` the host spins on.  Every wave fences
// its own stores at system scope before the barrier, so the word is published
// after all of them; the kernel touches no memory after it.
__global__ void k_gather(const TopState *__restrict__ st, const uint64_t *__restrict__ stats,
                         const uint64_t *__restrict__ mask, const uint32_t *__restrict__ flags,
                         const uint32_t *__restrict__ flag3, const TopCand *__restrict__ cand,
                         const uint32_t *__restrict__ uniq, uint32_t m, uint8_t *__restrict__ out,
                         uint64_t *done, uint64_t seq) {
  ResultHdr *h = reinterpret_cast<ResultHdr *>(out);
  TopCand *c = reinterpret_cast<TopCand *>(out + sizeof(ResultHdr));
  uint32_t *u = reinterpret_cast<uint32_t *>(out + sizeof(ResultHdr) + (size_t)m * sizeof(TopCand));
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    h->st = *st;
    h->stats[0] = stats[0];
    h->stats[1] = stats[1];
    h->mask = mask ? *mask : 0;
    for (int i = 0; i < 4; ++i) h->flags[i] = flags ? flags[i] : 0;
    if (flag3) h->flags[3] = *flag3;
  }
  for (uint32_t i = threadIdx.x; i < m; i += blockDim.x) {
    c[i] = cand[i];
    u[i] = uniq ? uniq[i] : 0;
  }
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(done, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

hipError_t launch_gather(const TopState *st, const uint64_t *stats, const uint64_t *mask,
                         const uint32_t *flags, const uint32_t *flag3, const TopCand *cand,
                         const uint32_t *uniq, uint32_t m, uint8_t *out, uint64_t *done,
                         uint64_t seq, hipStream_t s) {
  hipLaunchKernelGGL(k_gather, dim3(1), dim3(1024), 0, s, st, stats, mask, flags, flag3, cand, uniq, m,
                     out, done, seq);
  return hipGetLastError();
}

}  // namespace nk

namespace nk {
// ---------------------------------------------------------------------------
// Diagnostic: the count kernel's per-k-mer hash work alone (SipHash-1-3 +
// exact % pool, nk_device.h), keys generated in registers, no memory traffic
// but one store per thread.  nk_diag_hash_ms times it: the VALU floor of K1a.
// ---------------------------------------------------------------------------
constexpr int kDiagPer = 64;
// W128: SipHash-1-3 of 16-byte keys (--kmer-width=128, the config-5 count's
// hash: K1g's floor), else of u64 keys (K1a's)
template <bool W128>
__global__ __launch_bounds__(256) void k_diag_hash(FastMod fm, uint64_t n_keys,
                                                   uint32_t *__restrict__ out) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t key = (t * 0x9E3779B97F4A7C15ull) ^ 0x4E4B4D52ull;
  uint32_t acc = 0;
  const uint64_t first = t * kDiagPer;
#pragma unroll 16
  for (int i = 0; i < kDiagPer; ++i) {
    if (first + (uint64_t)i < n_keys)
      acc ^= fastmod32(W128 ? sip13_u128(key, key >> 17) : sip13_u64(key), fm);
    key += 0xD1B54A32D192ED03ull;
  }
  out[t] = acc;
}

hipError_t launch_diag_hash(uint64_t n_keys, uint64_t pool, uint32_t *out, hipStream_t s,
                            int width) {
  const uint64_t threads = (n_keys + kDiagPer - 1) / kDiagPer;
  const uint64_t blocks = (threads + 255) / 256;
  if (width == 128)
    hipLaunchKernelGGL(k_diag_hash<true>, dim3((uint32_t)blocks), dim3(256), 0, s,
                       make_fastmod(pool), n_keys, out);
  else
    hipLaunchKernelGGL(k_diag_hash<false>, dim3((uint32_t)blocks), dim3(256), 0, s,
                       make_fastmod(pool), n_keys, out);
  return hipGetLastError();
}

uint64_t diag_hash_out_words(uint64_t n_keys) {
  return ((n_keys + kDiagPer - 1) / kDiagPer + 255) / 256 * 256;
}
}  // namespace nk

#if defined(NK_ABL_STAMPS)
extern "C" int nk_diag_stamps(unsigned long long *out, size_t n) {
  if (n > (1u << 18)) n = 1u << 18;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(nk::g_stamps), n * 8, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif
