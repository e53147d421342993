// Exact k-mer count table (nk_exact.h).  The key extraction, the per-neuron
// distinct count and the lookups are kernels of this file; the sort and the
// run-length encoding are rocPRIM's device radix sort / RLE.
#include <cstring>  // before rocprim: its texture_cache_iterator uses memset

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_reduce_by_key.hpp>
#include <rocprim/device/device_run_length_encode.hpp>

#include "nk_device.h"
#include "nk_exact.h"
#include "nk_tile.h"

namespace nk {

namespace {

constexpr int kXTile = kTile;     // 4096 positions per workgroup
constexpr int kXBlock = kBlock;   // 256 threads
constexpr int kXPer = kXTile / kXBlock;

constexpr int kXWaves = kXBlock / 64;
static_assert(kXPer * kXWaves == 64, "one wave scans the per-(round, wave) counts");

// A tile's valid keys compacted in position order (q = j * kXBlock + tid):
// slot[j] = the key's index within the tile, *base = the tile's first index
// in the global key array (one atomic per tile), *total = its key count.  The
// keys are then staged in LDS and stored coalesced (each lane writing its own
// run of keys touched 64 cache lines per store instruction: the extraction ran
// at 1.8 TB/s, profiles/r02_s18).
struct TileSlots {
  uint32_t pre[kXPer * kXWaves];
  uint32_t total;
  unsigned long long base;
};
__device__ __forceinline__ void tile_slots(uint32_t ok, uint32_t (&slot)[kXPer], TileSlots &T,
                                           unsigned long long *n_keys) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint64_t below = (1ull << lane) - 1ull;
#pragma unroll
  for (int j = 0; j < kXPer; ++j) {
    const uint64_t m = __ballot((ok >> j) & 1u);
    slot[j] = (uint32_t)__popcll(m & below);
    if (lane == 0) T.pre[j * kXWaves + w] = (uint32_t)__popcll(m);
  }
  __syncthreads();
  if (threadIdx.x < 64) {
    const uint32_t c = T.pre[threadIdx.x];
    uint32_t incl = c;
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(incl, o, 64);
      if (lane >= o) incl += y;
    }
    T.pre[threadIdx.x] = incl - c;
    if (threadIdx.x == 63) {
      T.total = incl;
      T.base = incl ? atomicAdd(n_keys, (unsigned long long)incl) : 0ull;
    }
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kXPer; ++j) slot[j] += T.pre[j * kXWaves + w];
}

// k <= 32: keys from the staged tile, exactly as the count kernels derive them
template <bool CANON>
__global__ __launch_bounds__(kXBlock) void k_keys_tile(KmerInput in, int k,
                                                       uint64_t *__restrict__ keys,
                                                       unsigned long long *__restrict__ n_keys) {
  __shared__ TileLds<kXTile, !CANON> L;
  __shared__ TileSlots T;
  __shared__ uint64_t s_out[kXTile];
  const uint64_t tile = in.tile_base + blockIdx.x;
  const uint64_t T0 = tile * kXTile;
  stage_tile<kXTile, kXBlock, !CANON>(L, in, tile, k);
  uint64_t kv[kXPer];  // fixed slots (no dynamic register indexing) + a valid mask
  uint32_t ok = 0;
#pragma unroll
  for (int j = 0; j < kXPer; ++j) {
    const int q = j * kXBlock + threadIdx.x;
    kv[j] = 0;
    if (T0 + (uint64_t)q + (uint64_t)k > in.n_bases) continue;
    if (!window_valid(L, T0, q, k, in.n_bases, in.pos_lo, in.pos_hi)) continue;
    kv[j] = window_key<kXTile, !CANON, CANON>(L, q, k);
    ok |= 1u << j;
  }
  uint32_t slot[kXPer];
  tile_slots(ok, slot, T, n_keys);
#pragma unroll
  for (int j = 0; j < kXPer; ++j)
    if ((ok >> j) & 1u) s_out[slot[j]] = kv[j];
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < T.total; i += kXBlock) keys[T.base + i] = s_out[i];
}

// k > 32 (NK_KMER_COMPAT): the reference's release-build keys, one window per
// position, walking the records like the count kernel
template <bool CANON>
__global__ __launch_bounds__(kXBlock) void k_keys_compat(KmerInput in, int k,
                                                         uint64_t *__restrict__ keys,
                                                         unsigned long long *__restrict__ n_keys) {
  __shared__ TileSlots T;
  __shared__ uint64_t s_out[kXTile];
  const uint64_t T0 = (in.tile_base + blockIdx.x) * kXTile;
  uint64_t r = in.tile_rec[blockIdx.x];
  uint64_t kv[kXPer];
  uint32_t ok = 0;
#pragma unroll
  for (int j = 0; j < kXPer; ++j) {
    kv[j] = 0;
    const uint64_t p = T0 + (uint64_t)j * kXBlock + threadIdx.x;
    if (p >= in.n_bases || p < in.pos_lo || p >= in.pos_hi) continue;
    while (r + 1 < in.n_recs && in.offsets[r + 1] <= p) ++r;
    const uint64_t s0 = in.offsets[r], e0 = in.offsets[r + 1];
    if (p < s0 || p + (uint64_t)k > e0) continue;
    kv[j] = compat_key<CANON>(in.bases, s0, p, k);
    ok |= 1u << j;
  }
  uint32_t slot[kXPer];
  tile_slots(ok, slot, T, n_keys);
#pragma unroll
  for (int j = 0; j < kXPer; ++j)
    if ((ok >> j) & 1u) s_out[slot[j]] = kv[j];
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < T.total; i += kXBlock) keys[T.base + i] = s_out[i];
}

// NK_KMER_128 (k <= 64): the 128-bit keys of the staged tile, exactly as the
// 128-bit count kernels derive them (nk_tile.h window_key128); staged and
// stored one 64-bit half at a time
using u128 = unsigned __int128;
template <bool CANON>
__global__ __launch_bounds__(kXBlock) void k_keys_tile128(KmerInput in, int k,
                                                          uint64_t *__restrict__ keys2,
                                                          unsigned long long *__restrict__ n_keys) {
  __shared__ TileLds<kXTile, !CANON> L;
  __shared__ TileSlots T;
  __shared__ uint64_t s_out[kXTile];
  const uint64_t tile = in.tile_base + blockIdx.x;
  const uint64_t T0 = tile * kXTile;
  stage_tile<kXTile, kXBlock, !CANON>(L, in, tile, k);
  uint32_t ok = 0;
#pragma unroll
  for (int j = 0; j < kXPer; ++j) {
    const int q = j * kXBlock + threadIdx.x;
    if (T0 + (uint64_t)q + (uint64_t)k > in.n_bases) continue;
    if (window_valid(L, T0, q, k, in.n_bases, in.pos_lo, in.pos_hi)) ok |= 1u << j;
  }
  uint32_t slot[kXPer];
  tile_slots(ok, slot, T, n_keys);
  uint64_t hi[kXPer];
#pragma unroll
  for (int j = 0; j < kXPer; ++j) {
    hi[j] = 0;
    if (!((ok >> j) & 1u)) continue;
    const Key128 key = window_key128<kXTile, !CANON, CANON>(L, j * kXBlock + threadIdx.x, k);
    s_out[slot[j]] = key.lo;
    hi[j] = key.hi;
  }
  __syncthreads();
  uint64_t *dst = keys2 + 2 * T.base;
  for (uint32_t i = threadIdx.x; i < T.total; i += kXBlock) dst[2 * i] = s_out[i];
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kXPer; ++j)
    if ((ok >> j) & 1u) s_out[slot[j]] = hi[j];
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < T.total; i += kXBlock) dst[2 * i + 1] = s_out[i];
}

__global__ void k_kpn128(const u128 *__restrict__ uniq, const unsigned long long *__restrict__ n_uniq,
                         FastMod fm, uint32_t *__restrict__ kpn) {
  const uint64_t n = *n_uniq;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const u128 x = uniq[i];
    atomicAdd(&kpn[fastmod(sip13_u128((uint64_t)x, (uint64_t)(x >> 64)), fm)], 1u);
  }
}

__global__ void k_lookup128(const u128 *__restrict__ uniq, const uint32_t *__restrict__ cnt,
                            const unsigned long long *__restrict__ n_uniq,
                            const uint64_t *__restrict__ q2, uint64_t nq, uint32_t *__restrict__ out,
                            uint32_t *__restrict__ present) {
  const uint64_t n = n_uniq ? *n_uniq : 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nq;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const u128 key = ((u128)q2[2 * i + 1] << 64) | q2[2 * i];
    uint64_t lo = 0, hi = n;
    while (lo < hi) {
      const uint64_t mid = (lo + hi) >> 1;
      if (uniq[mid] < key) lo = mid + 1;
      else hi = mid;
    }
    const bool hit = lo < n && uniq[lo] == key;
    out[i] = hit ? cnt[lo] : 0u;
    present[i] = hit ? 1u : 0u;
  }
}

// (max_sc - sc[i], i): ascending keys = spikes descending; i ascending on
// entry, so the stable radix sort keeps ties in index order
__global__ void k_rank_keys(const uint64_t *__restrict__ sc, uint64_t pool, uint64_t max_sc,
                            uint64_t *__restrict__ keys, uint32_t *__restrict__ idx) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < pool;
       i += (uint64_t)gridDim.x * blockDim.x) {
    keys[i] = max_sc - sc[i];
    idx[i] = (uint32_t)i;
  }
}

__global__ void k_kpn(const uint64_t *__restrict__ uniq, const unsigned long long *__restrict__ n_uniq,
                      FastMod fm, uint32_t *__restrict__ kpn) {
  const uint64_t n = *n_uniq;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x)
    atomicAdd(&kpn[fastmod(sip13_u64(uniq[i]), fm)], 1u);
}

__global__ void k_lookup(TableView t, const uint64_t *__restrict__ q, uint64_t nq,
                         uint32_t *__restrict__ out, uint32_t *__restrict__ present) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nq;
       i += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t at;
    const bool hit = table_find(t, q[i], &at);
    out[i] = hit ? t.cnt[at] : 0u;
    present[i] = hit ? 1u : 0u;
  }
}

__global__ void k_top_uniques(const TopCand *__restrict__ cand, uint32_t m,
                              const uint32_t *__restrict__ kpn, uint32_t *__restrict__ uniq) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < m) uniq[i] = kpn[cand[i].idx];
}

constexpr unsigned long long kDEmpty = ~0ULL;

__device__ __forceinline__ uint64_t dmix(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}

// counts[key] += v in the delta; returns true if the key was new to the delta
__device__ bool delta_add(const DeltaArgs &d, uint64_t key, uint32_t v) {
  if (key == kDEmpty) return atomicAdd(&d.meta[0], (unsigned long long)v) == 0;
  uint64_t h = dmix(key) & d.mask;
  for (;;) {
    unsigned long long cur = d.keys[h];
    if (cur == kDEmpty) {
      cur = atomicCAS(&d.keys[h], kDEmpty, (unsigned long long)key);
      if (cur == kDEmpty) {
        atomicAdd(&d.vals[h], v);
        return true;
      }
    }
    if (cur == key) {
      atomicAdd(&d.vals[h], v);
      return false;
    }
    h = (h + 1) & d.mask;
  }
}

__device__ bool delta_get(const DeltaArgs &d, uint64_t key, uint32_t *v) {
  if (key == kDEmpty) {
    *v = (uint32_t)d.meta[0];
    return d.meta[0] != 0;
  }
  uint64_t h = dmix(key) & d.mask;
  for (;;) {
    const unsigned long long cur = d.keys[h];
    if (cur == kDEmpty) return false;
    if (cur == key) {
      *v = d.vals[h];
      return true;
    }
    h = (h + 1) & d.mask;
  }
}

__global__ void k_delta_clear(DeltaArgs d) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i <= d.mask;
       i += (uint64_t)gridDim.x * blockDim.x) {
    d.keys[i] = kDEmpty;
    d.vals[i] = 0;
  }
  if (blockIdx.x == 0 && threadIdx.x < 2) d.meta[threadIdx.x] = 0;
}

__global__ void k_delta_rehash(DeltaArgs from, DeltaArgs to) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i <= from.mask;
       i += (uint64_t)gridDim.x * blockDim.x)
    if (from.keys[i] != kDEmpty) delta_add(to, from.keys[i], from.vals[i]);
  if (blockIdx.x == 0 && threadIdx.x < 2) to.meta[threadIdx.x] = from.meta[threadIdx.x];
}

__global__ void k_seq_accumulate(const uint64_t *__restrict__ keys,
                                 const unsigned long long *__restrict__ n_keys, FastMod fm,
                                 unsigned long long *__restrict__ currents,
                                 uint8_t *__restrict__ touched, DeltaArgs d, TableView t) {
  const uint64_t n = *n_keys;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t key = keys[i];
    const uint64_t idx = fastmod(sip13_u64(key), fm);
    atomicAdd(&currents[idx], 1ULL);  // :217-223,236-241,251-254
    touched[idx] = 1;                 // local_unique[idx] = true
    uint64_t at;
    if (delta_add(d, key, 1) && !table_find(t, key, &at))
      atomicAdd(&d.meta[1], 1ull);    // a key new to `counts`
  }
}

__global__ __launch_bounds__(256) void k_seq_lif(uint64_t pool, unsigned long long *__restrict__ currents,
                                                 uint8_t *__restrict__ touched,
                                                 uint32_t *__restrict__ kpn, float *__restrict__ V,
                                                 uint32_t *__restrict__ R,
                                                 uint64_t *__restrict__ SC, float thr, float leak,
                                                 uint32_t refr, uint32_t *__restrict__ hist,
                                                 unsigned long long *__restrict__ stats) {
  __shared__ uint32_t sh[kHistBins];
  for (int i = threadIdx.x; i < kHistBins; i += 256) sh[i] = 0;
  __syncthreads();
  unsigned long long sp = 0, mx = 0;
  uint32_t n_zero = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < pool;
       i += (uint64_t)gridDim.x * 256) {
    if (touched[i]) {  // :258-263 kmer_per_neuron[idx] += 1 per sequence
      kpn[i] += 1;
      touched[i] = 0;
    }
    const unsigned long long cur = currents[i];
    uint64_t sc = SC[i];
    if (cur != 0) {  // :266-271: `current > 0.0 && neuron.update(current as f32)`
      const float c = (float)(double)cur;
      uint32_t r = R[i];
      if (r > 0) {
        R[i] = r - 1;
      } else {
        const float v = lif_step(V[i], leak, c);
        if (v >= thr) {
          V[i] = 0.0f;
          R[i] = refr;
          sc += 1;
          SC[i] = sc;
          sp += 1;
        } else {
          V[i] = v;
        }
      }
      currents[i] = 0;  // :270
    }
    mx = sc > mx ? sc : mx;
    if (sc == 0) ++n_zero;  // bin 0 in a register (same-address atomics serialise)
    else atomicAdd(&sh[sc < (uint64_t)(kHistBins - 1) ? (uint32_t)sc : (uint32_t)(kHistBins - 1)], 1u);
  }
  for (int o = 32; o > 0; o >>= 1) {
    sp += __shfl_down(sp, o, 64);
    const unsigned long long om = __shfl_down(mx, o, 64);
    mx = om > mx ? om : mx;
    n_zero += __shfl_down(n_zero, o, 64);
  }
  if ((threadIdx.x & 63) == 0 && n_zero) atomicAdd(&sh[0], n_zero);
  if ((threadIdx.x & 63) == 0) {
    if (sp) atomicAdd(&stats[0], sp);
    atomicMax(&stats[1], mx);
  }
  __syncthreads();
  uint32_t *hc = hist + (size_t)(blockIdx.x & (kHistCopies - 1)) * kHistBins;
  for (int i = threadIdx.x; i < kHistBins; i += 256)
    if (sh[i]) atomicAdd(&hc[i], sh[i]);
}

__global__ void k_lookup2(TableView t, DeltaArgs d, const uint64_t *__restrict__ q, uint64_t nq,
                          uint32_t *__restrict__ out, uint32_t *__restrict__ present) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nq;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t key = q[i];
    uint64_t at;
    const bool hm = table_find(t, key, &at);
    uint32_t dv = 0;
    const bool hd = d.keys && delta_get(d, key, &dv);
    out[i] = (hm ? t.cnt[at] : 0u) + (hd ? dv : 0u);  // u32 wrap like AtomicU32
    present[i] = (hm || hd) ? 1u : 0u;
  }
}

unsigned grid_for(uint64_t n, unsigned cap) {
  uint64_t g = (n + 255) / 256;
  if (g > cap) g = cap;
  return g ? (unsigned)g : 1u;
}

}  // namespace

hipError_t exact_keys(const KmerInput &in, int k, int canonical, uint64_t *keys,
                      unsigned long long *n_keys, hipStream_t s) {
  if (!in.n_tiles) return hipSuccess;
  const dim3 g((unsigned)in.n_tiles), b(kXBlock);
  if (k <= 32) {
    if (canonical) hipLaunchKernelGGL(k_keys_tile<true>, g, b, 0, s, in, k, keys, n_keys);
    else hipLaunchKernelGGL(k_keys_tile<false>, g, b, 0, s, in, k, keys, n_keys);
  } else {
    if (canonical) hipLaunchKernelGGL(k_keys_compat<true>, g, b, 0, s, in, k, keys, n_keys);
    else hipLaunchKernelGGL(k_keys_compat<false>, g, b, 0, s, in, k, keys, n_keys);
  }
  return hipGetLastError();
}

// The u64 table sort: rocPRIM's onesweep radix sort.  NK_SORT_BITS (A/B
// builds) replaces its default gfx950 config (8 bits per pass: 8 passes of
// ~590 us over 115 M keys) with NK_SORT_BITS per pass, 512 x NK_SORT_IPT keys
// per block.
#ifndef NK_SORT_BITS
#define NK_SORT_BITS 0
#endif
#ifndef NK_SORT_IPT
#define NK_SORT_IPT 8
#endif
#if NK_SORT_BITS
using KeySortCfg = rocprim::radix_sort_config<
    rocprim::default_config, rocprim::default_config,
    rocprim::radix_sort_onesweep_config<rocprim::kernel_config<512, NK_SORT_IPT>,
                                        rocprim::kernel_config<512, NK_SORT_IPT>, NK_SORT_BITS,
                                        rocprim::block_radix_rank_algorithm::match>>;
#else
using KeySortCfg = rocprim::default_config;
#endif

size_t exact_temp_bytes(size_t n, int end_bit) {
  size_t a = 0, b = 0;
  (void)rocprim::radix_sort_keys<KeySortCfg>(nullptr, a, (const uint64_t *)nullptr, (uint64_t *)nullptr, n, 0,
                                 end_bit);
  (void)rocprim::run_length_encode(nullptr, b, (const uint64_t *)nullptr, n, (uint64_t *)nullptr,
                                   (uint32_t *)nullptr, (unsigned long long *)nullptr);
  return (a > b ? a : b) + 256;
}

hipError_t exact_sort_rle(uint64_t *keys, uint64_t *keys_sorted, size_t n, int end_bit,
                          uint64_t *uniq, uint32_t *cnt, unsigned long long *n_uniq, void *tmp,
                          size_t tmp_bytes, hipStream_t s) {
  if (!n) return hipMemsetAsync(n_uniq, 0, sizeof(unsigned long long), s);
  size_t tb = tmp_bytes;
  hipError_t e = rocprim::radix_sort_keys<KeySortCfg>(tmp, tb, (const uint64_t *)keys, keys_sorted, n, 0,
                                          end_bit, s);
  if (e != hipSuccess) return e;
  tb = tmp_bytes;
  return rocprim::run_length_encode(tmp, tb, (const uint64_t *)keys_sorted, n, uniq, cnt, n_uniq,
                                    s);
}

// ---- multi-GPU table ---------------------------------------------------------
constexpr int kOwnerMax = 4096;
constexpr int kOwnerPer = 16;  // entries per thread (4096 per 256-thread block)

__global__ __launch_bounds__(256) void k_owner_hist(const uint64_t *__restrict__ uniq,
                                                    const unsigned long long *__restrict__ n_uniq,
                                                    uint32_t world,
                                                    unsigned long long *__restrict__ cnt,
                                                    const uint32_t *__restrict__ tcnt) {
  __shared__ uint32_t h[kOwnerMax];
  for (uint32_t r = threadIdx.x; r < world; r += 256) h[r] = 0;
  __syncthreads();
  const uint64_t n = *n_uniq;
  const uint64_t base = (uint64_t)blockIdx.x * 256 * kOwnerPer;
  for (int j = 0; j < kOwnerPer; ++j) {
    const uint64_t i = base + (uint64_t)j * 256 + threadIdx.x;
    if (i < n && (!tcnt || tcnt[i])) atomicAdd(&h[exact_owner(uniq[i], world)], 1u);
  }
  __syncthreads();
  for (uint32_t r = threadIdx.x; r < world; r += 256)
    if (h[r]) atomicAdd(&cnt[r], (unsigned long long)h[r]);
}

// block-aggregated scatter: LDS ranks per owner, one global reservation per
// (block, owner)
__global__ __launch_bounds__(256) void k_owner_scatter(const uint64_t *__restrict__ uniq,
                                                       const uint32_t *__restrict__ cnt,
                                                       const unsigned long long *__restrict__ n_uniq,
                                                       uint32_t world,
                                                       unsigned long long *__restrict__ cursor,
                                                       uint64_t *__restrict__ out_keys,
                                                       uint32_t *__restrict__ out_cnt,
                                                       int skip_zero) {
  __shared__ uint32_t h[kOwnerMax];
  __shared__ unsigned long long b0[kOwnerMax];
  for (uint32_t r = threadIdx.x; r < world; r += 256) h[r] = 0;
  __syncthreads();
  const uint64_t n = *n_uniq;
  const uint64_t base = (uint64_t)blockIdx.x * 256 * kOwnerPer;
  uint32_t own[kOwnerPer], rk[kOwnerPer];
  for (int j = 0; j < kOwnerPer; ++j) {
    const uint64_t i = base + (uint64_t)j * 256 + threadIdx.x;
    const bool live = i < n && (!skip_zero || cnt[i]);
    own[j] = live ? exact_owner(uniq[i], world) : world;
    rk[j] = live ? atomicAdd(&h[own[j]], 1u) : 0u;
  }
  __syncthreads();
  for (uint32_t r = threadIdx.x; r < world; r += 256)
    b0[r] = h[r] ? atomicAdd(&cursor[r], (unsigned long long)h[r]) : 0ull;
  __syncthreads();
  for (int j = 0; j < kOwnerPer; ++j) {
    const uint64_t i = base + (uint64_t)j * 256 + threadIdx.x;
    if (own[j] == world) continue;
    const uint64_t at = b0[own[j]] + rk[j];
    out_keys[at] = uniq[i];
    out_cnt[at] = cnt[i];
  }
}

hipError_t exact_owner_hist(const uint64_t *uniq, const unsigned long long *n_uniq, size_t max_n,
                            uint32_t world, unsigned long long *cnt, hipStream_t s,
                            const uint32_t *tcnt) {
  if (!max_n) return hipSuccess;
  if (!world || world > (uint32_t)kOwnerMax) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_owner_hist, dim3(grid_for(max_n, 256 * kOwnerPer)), dim3(256), 0, s, uniq,
                     n_uniq, world, cnt, tcnt);
  return hipGetLastError();
}

hipError_t exact_owner_scatter(const uint64_t *uniq, const uint32_t *cnt,
                               const unsigned long long *n_uniq, size_t max_n, uint32_t world,
                               unsigned long long *cursor, uint64_t *out_keys, uint32_t *out_cnt,
                               hipStream_t s, bool skip_zero) {
  if (!max_n) return hipSuccess;
  if (!world || world > (uint32_t)kOwnerMax) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_owner_scatter, dim3(grid_for(max_n, 256 * kOwnerPer)), dim3(256), 0, s,
                     uniq, cnt, n_uniq, world, cursor, out_keys, out_cnt, skip_zero ? 1 : 0);
  return hipGetLastError();
}

size_t exact_merge_temp_bytes(size_t n, int end_bit) {
  size_t a = 0, b = 0;
  (void)rocprim::radix_sort_pairs(nullptr, a, (const uint64_t *)nullptr, (uint64_t *)nullptr,
                                  (const uint32_t *)nullptr, (uint32_t *)nullptr, n, 0, end_bit);
  (void)rocprim::reduce_by_key(nullptr, b, (const uint64_t *)nullptr, (const uint32_t *)nullptr, n,
                               (uint64_t *)nullptr, (uint32_t *)nullptr,
                               (unsigned long long *)nullptr, rocprim::plus<uint32_t>(),
                               rocprim::equal_to<uint64_t>());
  return (a > b ? a : b) + 256;
}

hipError_t exact_merge_pairs(const uint64_t *keys, const uint32_t *cnt, size_t n, int end_bit,
                             uint64_t *keys_sorted, uint32_t *cnt_sorted, uint64_t *uniq,
                             uint32_t *uniq_cnt, unsigned long long *n_uniq, void *tmp,
                             size_t tmp_bytes, hipStream_t s) {
  if (!n) return hipMemsetAsync(n_uniq, 0, sizeof(unsigned long long), s);
  size_t tb = tmp_bytes;
  hipError_t e = rocprim::radix_sort_pairs(tmp, tb, keys, keys_sorted, cnt, cnt_sorted, n, 0,
                                           end_bit, s);
  if (e != hipSuccess) return e;
  tb = tmp_bytes;
  return rocprim::reduce_by_key(tmp, tb, (const uint64_t *)keys_sorted, (const uint32_t *)cnt_sorted,
                                n, uniq, uniq_cnt, n_uniq, rocprim::plus<uint32_t>(),
                                rocprim::equal_to<uint64_t>(), s);
}

hipError_t exact_kpn(const uint64_t *uniq, const unsigned long long *n_uniq, size_t max_n,
                     uint64_t pool, uint32_t *kpn, hipStream_t s) {
  if (!pool || !max_n) return hipSuccess;
  FastMod fm;
  fm.p = pool;
  fm.magic = (~0ULL) / pool;
  hipLaunchKernelGGL(k_kpn, dim3(grid_for(max_n, 8192)), dim3(256), 0, s, uniq, n_uniq, fm, kpn);
  return hipGetLastError();
}

hipError_t exact_lookup(const TableView &t, const uint64_t *q, size_t nq, uint32_t *out,
                        uint32_t *present, hipStream_t s) {
  if (!nq) return hipSuccess;
  hipLaunchKernelGGL(k_lookup, dim3(grid_for(nq, 4096)), dim3(256), 0, s, t, q, (uint64_t)nq, out,
                     present);
  return hipGetLastError();
}

hipError_t delta_clear(const DeltaArgs &d, hipStream_t s) {
  hipLaunchKernelGGL(k_delta_clear, dim3(grid_for(d.mask + 1, 4096)), dim3(256), 0, s, d);
  return hipGetLastError();
}

hipError_t delta_rehash(const DeltaArgs &from, const DeltaArgs &to, hipStream_t s) {
  hipLaunchKernelGGL(k_delta_rehash, dim3(grid_for(from.mask + 1, 4096)), dim3(256), 0, s, from,
                     to);
  return hipGetLastError();
}

hipError_t seq_accumulate(const uint64_t *keys, const unsigned long long *n_keys, size_t max_n,
                          uint64_t pool, unsigned long long *currents, uint8_t *touched,
                          const DeltaArgs &d, const TableView &t, hipStream_t s) {
  if (!max_n || !pool) return hipSuccess;
  FastMod fm;
  fm.p = pool;
  fm.magic = (~0ULL) / pool;
  hipLaunchKernelGGL(k_seq_accumulate, dim3(grid_for(max_n, 4096)), dim3(256), 0, s, keys, n_keys,
                     fm, currents, touched, d, t);
  return hipGetLastError();
}

hipError_t seq_lif(uint64_t pool, unsigned long long *currents, uint8_t *touched, uint32_t *kpn,
                   float *v, uint32_t *r, uint64_t *sc, float thr, float leak, uint32_t refr,
                   uint32_t *hist, uint64_t *stats, hipStream_t s) {
  if (!pool) return hipSuccess;
  hipLaunchKernelGGL(k_seq_lif, dim3(grid_for(pool, 2048)), dim3(256), 0, s, pool, currents,
                     touched, kpn, v, r, sc, thr, leak, refr, hist,
                     (unsigned long long *)stats);
  return hipGetLastError();
}

hipError_t exact_lookup2(const TableView &t, const DeltaArgs &d, const uint64_t *q, size_t nq,
                         uint32_t *out, uint32_t *present, hipStream_t s) {
  if (!nq) return hipSuccess;
  hipLaunchKernelGGL(k_lookup2, dim3(grid_for(nq, 4096)), dim3(256), 0, s, t, d, q, (uint64_t)nq,
                     out, present);
  return hipGetLastError();
}

hipError_t exact_top_uniques(const TopCand *cand, uint32_t m, const uint32_t *kpn, uint32_t *uniq,
                             hipStream_t s) {
  if (!m) return hipSuccess;
  hipLaunchKernelGGL(k_top_uniques, dim3((m + 255) / 256), dim3(256), 0, s, cand, m, kpn, uniq);
  return hipGetLastError();
}

// ---- NK_KMER_128 table ---------------------------------------------------------
hipError_t exact_keys128(const KmerInput &in, int k, int canonical, uint64_t *keys2,
                         unsigned long long *n_keys, hipStream_t s) {
  if (!in.n_tiles) return hipSuccess;
  if (k > 64) return hipErrorInvalidValue;
  const dim3 g((unsigned)in.n_tiles), b(kXBlock);
  if (canonical) hipLaunchKernelGGL(k_keys_tile128<true>, g, b, 0, s, in, k, keys2, n_keys);
  else hipLaunchKernelGGL(k_keys_tile128<false>, g, b, 0, s, in, k, keys2, n_keys);
  return hipGetLastError();
}

size_t exact_temp_bytes128(size_t n, int end_bit) {
  size_t a = 0, b = 0;
  (void)rocprim::radix_sort_keys(nullptr, a, (const u128 *)nullptr, (u128 *)nullptr, n, 0, end_bit);
  (void)rocprim::run_length_encode(nullptr, b, (const u128 *)nullptr, n, (u128 *)nullptr,
                                   (uint32_t *)nullptr, (unsigned long long *)nullptr);
  return (a > b ? a : b) + 256;
}

hipError_t exact_sort_rle128(uint64_t *keys2, uint64_t *sorted2, size_t n, int end_bit,
                             uint64_t *uniq2, uint32_t *cnt, unsigned long long *n_uniq, void *tmp,
                             size_t tmp_bytes, hipStream_t s) {
  if (!n) return hipMemsetAsync(n_uniq, 0, sizeof(unsigned long long), s);
  const u128 *keys = reinterpret_cast<const u128 *>(keys2);
  u128 *sorted = reinterpret_cast<u128 *>(sorted2), *uniq = reinterpret_cast<u128 *>(uniq2);
  size_t tb = tmp_bytes;
  hipError_t e = rocprim::radix_sort_keys(tmp, tb, keys, sorted, n, 0, end_bit, s);
  if (e != hipSuccess) return e;
  tb = tmp_bytes;
  return rocprim::run_length_encode(tmp, tb, (const u128 *)sorted, n, uniq, cnt, n_uniq, s);
}

hipError_t exact_kpn128(const uint64_t *uniq2, const unsigned long long *n_uniq, size_t max_n,
                        uint64_t pool, uint32_t *kpn, hipStream_t s) {
  if (!pool || !max_n) return hipSuccess;
  FastMod fm;
  fm.p = pool;
  fm.magic = (~0ULL) / pool;
  hipLaunchKernelGGL(k_kpn128, dim3(grid_for(max_n, 8192)), dim3(256), 0, s,
                     reinterpret_cast<const u128 *>(uniq2), n_uniq, fm, kpn);
  return hipGetLastError();
}

hipError_t exact_lookup128(const uint64_t *uniq2, const uint32_t *cnt,
                           const unsigned long long *n_uniq, const uint64_t *q2, size_t nq,
                           uint32_t *out, uint32_t *present, hipStream_t s) {
  if (!nq) return hipSuccess;
  hipLaunchKernelGGL(k_lookup128, dim3(grid_for(nq, 4096)), dim3(256), 0, s,
                     reinterpret_cast<const u128 *>(uniq2), cnt, n_uniq, q2, (uint64_t)nq, out,
                     present);
  return hipGetLastError();
}

// ---- rows of top_abundant_neurons(n), any n ----------------------------------------
size_t rank_rows_temp_bytes(size_t pool) {
  size_t a = 0;
  (void)rocprim::radix_sort_pairs(nullptr, a, (const uint64_t *)nullptr, (uint64_t *)nullptr,
                                  (const uint32_t *)nullptr, (uint32_t *)nullptr, pool, 0, 64);
  return a + 256;
}

hipError_t rank_rows(const uint64_t *sc, uint64_t pool, uint64_t max_sc, uint64_t *keys,
                     uint64_t *keys_sorted, uint32_t *idx, uint32_t *idx_sorted, void *tmp,
                     size_t tmp_bytes, hipStream_t s) {
  if (!pool) return hipSuccess;
  if (pool > 0xFFFFFFFFull) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_rank_keys, dim3(grid_for(pool, 8192)), dim3(256), 0, s, sc, pool, max_sc,
                     keys, idx);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  int end_bit = 1;  // bits of max_sc: keys are max_sc - sc <= max_sc
  while (end_bit < 64 && (max_sc >> end_bit)) ++end_bit;
  size_t tb = tmp_bytes;
  return rocprim::radix_sort_pairs(tmp, tb, (const uint64_t *)keys, keys_sorted,
                                   (const uint32_t *)idx, idx_sorted, (size_t)pool, 0, end_bit, s);
}

}  // namespace nk
