// nk_wide.hip — the partitioned count for every key mode and pool size.
//
// k_part (nk_kernels.hip) is the fast path of the metric: k <= 32 keys rolled
// in registers, pool <= 16.7 M (bucket = neuron >> 15, 512 buckets of 32768
// bins).  This file covers the rest of SURVEY.md §8a without global atomics
// per k-mer (the direct-atomic kernels run at ~20 G adds/s chip-wide):
//
//   key modes   KM 0  k <= 32 u64 keys at a position (pools past 16.7 M)
//               KM 1  k > 32, the reference's release-build u64 semantics
//                     (NK_KMER_COMPAT, src/models.rs:188,192-194,260-266)
//               KM 2  --kmer-width=128 (u128 keys, SipHash over 16 bytes)
//   narrow      pool <= 512 * 32768: k_part_gen writes u16 bin offsets
//               straight into the 32768-bin buckets k_bucket_hist reads
//   wide        pool <= 2^31: k_part_gen sorts into <= 256 coarse buckets of
//               2^S bins (u32 offsets), k_split re-sorts each coarse bucket
//               into its 2^(S-15) fine buckets (u16 offsets), and the same
//               k_bucket_hist histograms them (two LDS counting sorts, both
//               with one HBM reservation atomic per (tile, bucket))
//
// Records past a bucket's region are counted with direct atomics (exact).  No
// positions are kept: the uniques of these modes come from the rescan pass.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <type_traits>

#include "nk_device.h"
#include "nk_kernels.h"
#include "nk_gen.h"
#include "nk_tile.h"

namespace nk {

namespace {

template <bool WIDE>
struct GenShape {
  static constexpr int kMaxB = WIDE ? kWideMaxBuckets : kMaxBuckets;
  static constexpr int kSlots = kPartTile + 7 * kMaxB;
  static constexpr int kGroups = kSlots / 8;
  static constexpr int kGroupIters = (kGroups + kPartBlock - 1) / kPartBlock;
  using Rec = typename std::conditional<WIDE, uint32_t, uint16_t>::type;
  using GMap = typename std::conditional<(kMaxB > 256), uint16_t, uint8_t>::type;
  static constexpr uint32_t kPad = WIDE ? 0xFFFFFFFFu : 0xFFFFu;
};

// LDS counting sort of one tile's records by bucket, one HBM reservation per
// (tile, bucket), 16-B stores of 8-record groups (shared by k_part_gen and
// k_split).  E[j] = bucket << 16 | rank (bucket == nb: no record), O[j] = the
// record.  Ends the kernel.
template <bool WIDE, int PER, int BLOCK = kPartBlock>
__device__ __forceinline__ void sort_and_store(const uint32_t (&E)[PER], const uint32_t (&O)[PER],
                                               uint32_t nb, uint32_t *s_cnt, uint32_t *s_start,
                                               uint32_t *s_base, uint32_t *s_fit,
                                               typename GenShape<WIDE>::Rec *s_rec,
                                               typename GenShape<WIDE>::GMap *s_gmap,
                                               unsigned long long *__restrict__ fill,
                                               uint32_t *__restrict__ overflow, uint64_t cap,
                                               typename GenShape<WIDE>::Rec *__restrict__ dst_rec,
                                               uint64_t bucket_base, int bin_bits,
                                               unsigned long long *__restrict__ currents,
                                               uint2 *__restrict__ desc = nullptr,
                                               uint64_t max_segs = 0, uint32_t tile = 0) {
  using S = GenShape<WIDE>;
  using Rec = typename S::Rec;
  const int tid = threadIdx.x;
  __syncthreads();
  if (tid < 64) {  // exclusive scan of the padded counts (one wave)
    uint32_t carry = 0;
    for (uint32_t b0 = 0; b0 < nb; b0 += 64) {
      const uint32_t b = b0 + tid;
      const uint32_t c = b < nb ? (s_cnt[b] + 7u) & ~7u : 0;
      uint32_t x = c;
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if (tid >= o) x += y;
      }
      if (b < nb) s_start[b] = carry + x - c;
      carry += __shfl(x, 63, 64);
    }
    if (tid == 0) s_start[nb] = carry;
  }
  for (uint32_t b = tid; b < nb; b += BLOCK) {
    const uint32_t c = (s_cnt[b] + 7u) & ~7u;
    uint32_t fit = 0, base = 0;
    if (c) {
      // kept records: one segment per (tile, bucket), counted in bits 40..
      const unsigned long long ret =
          atomicAdd(&fill[bucket_base + b], (unsigned long long)c | (desc ? (1ull << 40) : 0ull));
      const uint64_t eb = ret & ((1ull << 40) - 1);
      fit = eb >= cap ? 0u : (uint32_t)(cap - eb < c ? cap - eb : c);
      bool over = fit < c;
      if (desc) {
        const uint64_t seg = ret >> 40;
        if (seg < max_segs) desc[(bucket_base + b) * max_segs + seg] = make_uint2(tile, (uint32_t)eb);
        else over = true;  // (the uniques of this bucket fall back to the rescan)
      }
      if (over) overflow[bucket_base + b] = 1u;
      base = (uint32_t)eb;
    }
    s_base[b] = base;
    s_fit[b] = fit;
  }
  __syncthreads();
  {
    uint32_t st[PER];
#pragma unroll
    for (int j = 0; j < PER; ++j) st[j] = s_start[E[j] >> 16];
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const uint32_t slot = st[j] + (E[j] & 0xFFFFu);
      if (slot < (uint32_t)S::kSlots) s_rec[slot] = (Rec)O[j];  // the no-record bucket may run past
    }
  }
  for (uint32_t b = tid; b < nb; b += BLOCK) {
    const uint32_t c = s_cnt[b], st = s_start[b], cp = (c + 7u) & ~7u;
    for (uint32_t i = c; i < cp; ++i) s_rec[st + i] = (Rec)S::kPad;
    for (uint32_t g = st >> 3; g < (st + cp) >> 3; ++g) s_gmap[g] = (typename S::GMap)b;
  }
  __syncthreads();
  const uint32_t n_groups = s_start[nb] >> 3;
#pragma unroll
  for (int it = 0; it < (S::kGroups + BLOCK - 1) / BLOCK; ++it) {
    const uint32_t g = (uint32_t)tid + (uint32_t)it * BLOCK;
    if (g >= n_groups) break;
    const uint32_t b = s_gmap[g];
    const uint32_t j8 = g * 8 - s_start[b];
    const uint64_t bg = bucket_base + b;
    if (j8 < s_fit[b]) {
      Rec *d = dst_rec + bg * cap + s_base[b] + j8;
      const uint4 *src = reinterpret_cast<const uint4 *>(&s_rec[g * 8]);
      if (WIDE) {
        reinterpret_cast<uint4 *>(d)[0] = src[0];
        reinterpret_cast<uint4 *>(d)[1] = src[1];
      } else {
        reinterpret_cast<uint4 *>(d)[0] = src[0];
      }
    } else if (currents) {  // region full: count directly (exact, slow, rare; none in a table-only pass)
      for (int i = 0; i < 8; ++i) {
        const uint32_t o = (uint32_t)s_rec[g * 8 + i];
        if (o != S::kPad) atomicAdd(&currents[(bg << bin_bits) | (o & ((1u << bin_bits) - 1u))], 1ULL);
      }
    }
  }
}

}  // namespace

// k <= 32, canonical (KM 0): the lane's 16 windows rolled in registers exactly
// as K1a does it (nk_kernels.hip part_tile: the first window from the bit
// streams, the next 15 as funnel shifts of two 96-bit words per strand,
// src/models.rs:254-286) -- the generic loop extracted every window from LDS
// (window_key: six LDS words and 64-bit variable shifts per key).  Pools past
// 4.2 M take this wide count (two levels: long segments per (tile, coarse
// bucket) instead of ~13-record ones per (tile, 32768-neuron bucket)).
template <bool SMALL>
__device__ __forceinline__ void gen_rolled64(const TileLds<kPartTile, false> &L, const KmerInput &in,
                                             uint64_t T0, int q0, int k, const FastMod &fm,
                                             uint32_t nb, int bb, uint32_t omask, uint32_t ltag,
                                             uint32_t *s_cnt, uint32_t (&E)[kPer], uint32_t (&O)[kPer]) {
  const uint64_t rem = in.n_bases - T0;  // >= 1
  const uint64_t nrange = rem >= (uint64_t)k ? rem - (uint64_t)k + 1 : 0;
  uint32_t ok = ~(L.WIN[q0 >> 5] >> (q0 & 31)) & 0xFFFFu;
  if (nrange < (uint64_t)q0 + kPer) ok &= nrange > (uint64_t)q0 ? (1u << (uint32_t)(nrange - q0)) - 1u : 0u;
  const uint64_t p0 = T0 + (uint64_t)q0;
  if (in.pos_lo > p0) ok &= in.pos_lo - p0 >= (uint64_t)kPer ? 0u : ~((1u << (uint32_t)(in.pos_lo - p0)) - 1u);
  if (in.pos_hi < p0 + kPer) ok &= in.pos_hi > p0 ? (1u << (uint32_t)(in.pos_hi - p0)) - 1u : 0u;
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
  const uint32_t g0 = inF, g1 = (uint32_t)fwd, g2 = (uint32_t)(fwd >> 32);
  const unsigned __int128 X = ((unsigned __int128)inR << twok) | rev;
  const uint32_t x0 = (uint32_t)X, x1 = (uint32_t)(X >> 32), x2 = (uint32_t)(X >> 64);
  const uint32_t mlo = (uint32_t)mask2k, mhi = (uint32_t)(mask2k >> 32);
  const uint32_t pv = (uint32_t)fm.p;
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    if (j) {
      fwd = ((uint64_t)(__builtin_amdgcn_alignbit(g2, g1, 32 - 2 * j) & mhi) << 32) |
            (__builtin_amdgcn_alignbit(g1, g0, 32 - 2 * j) & mlo);
      rev = ((uint64_t)(__builtin_amdgcn_alignbit(x2, x1, 2 * j) & mhi) << 32) |
            (__builtin_amdgcn_alignbit(x1, x0, 2 * j) & mlo);
    }
    const uint64_t h = sip13_u64(fwd < rev ? fwd : rev);
    const uint32_t idx = SMALL ? fastmod32_p(h, fm, pv) : (uint32_t)fastmod(h, fm);
    const uint32_t b = ((ok >> j) & 1u) ? (idx >> bb) : nb;
    E[j] = (b << 16) | atomicAdd(&s_cnt[b], 1u);
    O[j] = (idx & omask) | ltag;
  }
}

// --kmer-width=128, canonical, 48 < k <= 64 (config 5: k = 63): the lane's 16
// windows from 6 forward and 6 complement code words read once from LDS, each
// window's two 128-bit strands by funnel shifts of constant (2j) and uniform
// (128 - 2k) amounts -- no per-window LDS reads, 64-bit variable shifts or
// dynamically indexed registers (the generic loop's cost: K1g at 0.57 of its
// 128-bit hash-only floor at a 12.5 Gbase input, profiles/r04_t3).  The same
// keys as window_key128<CANON> (nk_tile.h); every position is hashed, the
// ones that start no k-mer go to the no-record bucket nb.
// SH >= 0: 128 - 2k at compile time (k = 63: SH = 2; -1: k at run time).
template <int SH, bool SMALL>
__device__ __forceinline__ void gen_rolled128(const TileLds<kPartTile, false> &L, const KmerInput &in,
                                              uint64_t T0, int q0, int k, const FastMod &fm,
                                              uint32_t nb, int bb, uint32_t omask,
                                              uint32_t ltag, uint32_t *s_cnt, uint32_t (&E)[kPer],
                                              uint32_t (&O)[kPer]) {
  const int w = q0 >> 4;  // q0 is 16-aligned
  uint32_t Fw[6], Rw[6];
#pragma unroll
  for (int c = 0; c < 6; ++c) {
    Fw[c] = L.F[w + c];
    Rw[c] = L.R[w + c];
  }
  // windows that start a k-mer of some record, in [pos_lo, pos_hi)
  uint32_t ok = ~(L.WIN[q0 >> 5] >> (q0 & 31)) & 0xFFFFu;
  const uint64_t rem = in.n_bases - T0;
  const uint64_t nrange = rem >= (uint64_t)k ? rem - (uint64_t)k + 1 : 0;
  if (nrange < (uint64_t)q0 + kPer) ok &= nrange > (uint64_t)q0 ? (1u << (uint32_t)(nrange - q0)) - 1u : 0u;
  const uint64_t p0 = T0 + (uint64_t)q0;
  if (in.pos_lo > p0) ok &= in.pos_lo - p0 >= (uint64_t)kPer ? 0u : ~((1u << (uint32_t)(in.pos_lo - p0)) - 1u);
  if (in.pos_hi < p0 + kPer) ok &= in.pos_hi > p0 ? (1u << (uint32_t)(in.pos_hi - p0)) - 1u : 0u;
  const uint32_t sh = (uint32_t)(128 - 2 * k);  // 0 .. 30
  const uint64_t hmask = k >= 64 ? ~0ull : ((1ull << (2 * k - 64)) - 1ull);
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    uint32_t W[4], Y[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) Y[c] = j ? __builtin_amdgcn_alignbit(Rw[c + 1], Rw[c], 2 * j) : Rw[c];
    Key128 fwd, rev;
    if (SH >= 0 && 2 * j >= SH) {
      // (k compile-time) the forward strand is the stream at bit offset
      // 2j - SH, its top SH bits masked: one funnel shift per word
      constexpr uint32_t kTop = SH >= 0 ? 0xFFFFFFFFu >> (SH & 31) : 0u;
      const int o = 2 * j - SH;
#pragma unroll
      for (int c = 0; c < 4; ++c) W[c] = o ? __builtin_amdgcn_alignbit(Fw[c], Fw[c + 1], 32 - o) : Fw[c];
      fwd.lo = ((uint64_t)W[2] << 32) | W[3];
      fwd.hi = ((uint64_t)(W[0] & kTop) << 32) | W[1];
    } else {
#pragma unroll
      for (int c = 0; c < 4; ++c) W[c] = j ? __builtin_amdgcn_alignbit(Fw[c], Fw[c + 1], 32 - 2 * j) : Fw[c];
      fwd.lo = ((uint64_t)__builtin_amdgcn_alignbit(W[1], W[2], sh) << 32) |
               __builtin_amdgcn_alignbit(W[2], W[3], sh);
      fwd.hi = ((uint64_t)(W[0] >> sh) << 32) | __builtin_amdgcn_alignbit(W[0], W[1], sh);
    }
    rev.lo = ((uint64_t)Y[1] << 32) | Y[0];
    rev.hi = (((uint64_t)Y[3] << 32) | Y[2]) & hmask;
    const Key128 key = key128_less(rev, fwd) ? rev : fwd;
    const uint64_t h = sip13_u128(key.lo, key.hi);
    const uint32_t idx = SMALL ? fastmod32(h, fm) : (uint32_t)fastmod(h, fm);
    const uint32_t b = ((ok >> j) & 1u) ? (idx >> bb) : nb;
#if defined(NK_ABL_G_NORANK)  // ablation: no LDS rank atomic
    E[j] = (b << 16) | j;
#else
    E[j] = (b << 16) | atomicAdd(&s_cnt[b], 1u);
#endif
    O[j] = (idx & omask) | ltag;
  }
}

// LDS of one k_part_gen tile (and, aliased in one union, of one k_split tile:
// k_gen_split runs both in one workgroup)
template <bool WIDE, bool RAW>
struct GenLds {
  using S = GenShape<WIDE>;
  TileLds<kPartTile, RAW> L;
  uint32_t s_cnt[S::kMaxB + 1];
  uint32_t s_start[S::kMaxB + 1];
  uint32_t s_base[S::kMaxB];
  uint32_t s_fit[S::kMaxB];
  __align__(16) typename S::Rec s_rec[S::kSlots];
  typename S::GMap s_gmap[S::kGroups];
};

// K1g: hash + partition for key modes KM 0/1/2 (see the file comment) of
// tile in.tile_base + bi.  Lane = 16 consecutive positions of an 8192-position tile.
// KEYS (narrow, u64 keys: KM 0/1): each kept record's key is also written to
// ka->key at the record's slot (the grouped exact table's input, as
// K1a<KEYS> writes it for k <= 32), a record past its full region's key to
// the side list, pad slots' keys as 0.
template <int KM, bool CANON, bool WIDE, bool KEYS = false>
__device__ __forceinline__ void gen_tile(const KmerInput &in, int k, const FastMod &fm,
                                         const GenPartArgs &ga, uint64_t bi,
                                         GenLds<WIDE, !CANON> &sm, const GenKeyArgs *ka = nullptr) {
  static_assert(!KEYS || (KM < 2 && !WIDE), "keys: narrow u64-key modes");
  using S = GenShape<WIDE>;
  constexpr bool kRaw = !CANON;
  TileLds<kPartTile, kRaw> &L = sm.L;
  const int tid = threadIdx.x;
  const uint64_t tile = in.tile_base + bi;
  const uint64_t T0 = tile * (uint64_t)kPartTile;
  const uint32_t nb = ga.n_buckets;
  const int bb = ga.bin_bits;
  const bool small_pool = fm.p < (1ull << 30);  // the 32-bit modulo (nk_device.h) holds
  const uint32_t omask = (uint32_t)((1ull << bb) - 1ull);
  const uint32_t ltag = (WIDE && ga.lane_tag) ? ((uint32_t)tid << bb) : 0u;  // (GenPartArgs::lane_tag)
  for (uint32_t b = tid; b <= nb; b += kPartBlock) sm.s_cnt[b] = 0;
#if defined(NK_ABL_G_NOSTAGE)  // ablation: the tile's LDS not loaded
  __syncthreads();
#else
  stage_tile<kPartTile, kPartBlock, kRaw>(L, in, tile, k);  // syncs
#endif

  const int q0 = tid * kPer;
  uint32_t E[kPer], O[kPer];
  if constexpr (KM == 0 && CANON && !KEYS) {
    if (small_pool) gen_rolled64<true>(L, in, T0, q0, k, fm, nb, bb, omask, ltag, sm.s_cnt, E, O);
    else gen_rolled64<false>(L, in, T0, q0, k, fm, nb, bb, omask, ltag, sm.s_cnt, E, O);
    sort_and_store<WIDE, kPer>(E, O, nb, sm.s_cnt, sm.s_start, sm.s_base, sm.s_fit, sm.s_rec,
                               sm.s_gmap, ga.fill, ga.overflow, ga.cap,
                               reinterpret_cast<typename S::Rec *>(ga.rec), 0, bb, ga.currents, ga.desc,
                               ga.max_segs, (uint32_t)tile);
    return;
  }
  if constexpr (KM == 2 && CANON) {
    if (k > 48) {  // (uniform) the lane's 16 windows rolled from registers
      // (the pool's modulo a template argument too: a uniform branch per
      // window between the two forms cost K1g 1.3 %, profiles/r05_m)
      if (k == 63 && small_pool)  // config 5
        gen_rolled128<2, true>(L, in, T0, q0, k, fm, nb, bb, omask, ltag, sm.s_cnt, E, O);
      else if (k == 63)
        gen_rolled128<2, false>(L, in, T0, q0, k, fm, nb, bb, omask, ltag, sm.s_cnt, E, O);
      else if (small_pool)
        gen_rolled128<-1, true>(L, in, T0, q0, k, fm, nb, bb, omask, ltag, sm.s_cnt, E, O);
      else
        gen_rolled128<-1, false>(L, in, T0, q0, k, fm, nb, bb, omask, ltag, sm.s_cnt, E, O);
#if defined(NK_ABL_G_NOSORT)  // ablation: the records folded into one store per lane
      {
        uint32_t acc = 0;
#pragma unroll
        for (int j = 0; j < kPer; ++j) acc ^= E[j] + O[j];
        reinterpret_cast<uint32_t *>(ga.rec)[bi * kPartBlock + tid] = acc;
        return;
      }
#endif
      sort_and_store<WIDE, kPer>(E, O, nb, sm.s_cnt, sm.s_start, sm.s_base, sm.s_fit, sm.s_rec,
                                 sm.s_gmap, ga.fill, ga.overflow, ga.cap,
                                 reinterpret_cast<typename S::Rec *>(ga.rec), 0, bb, ga.currents, ga.desc,
                                 ga.max_segs, (uint32_t)tile);
      return;
    }
  }
  RecCursor rc;
  rec_cursor_init<KM>(rc, in, T0 + (uint64_t)q0, bi);
  if constexpr (KEYS) {
    uint64_t K[kPer];  // (fully unrolled: the keys stay in registers until their slots are known)
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      const int q = q0 + j;
      const bool ok = window_valid(L, T0, q, k, in.n_bases, in.pos_lo, in.pos_hi);
      K[j] = ok ? gen_key<KM, CANON>(L, in, q, T0 + (uint64_t)q, k, rc).lo : 0ull;
      const uint64_t h = ok ? gen_hash<KM>(Key128{K[j], 0}) : 0ull;
      const uint32_t idx = small_pool ? fastmod32(h, fm) : (uint32_t)fastmod(h, fm);
      const uint32_t b = ok ? (idx >> bb) : nb;
      E[j] = (b << 16) | atomicAdd(&sm.s_cnt[b], 1u);
      O[j] = idx & omask;
    }
    sort_and_store<false, kPer>(E, O, nb, sm.s_cnt, sm.s_start, sm.s_base, sm.s_fit, sm.s_rec,
                                sm.s_gmap, ga.fill, ga.overflow, ga.cap,
                                reinterpret_cast<typename S::Rec *>(ga.rec), 0, bb, ga.currents);
    // s_base / s_fit / s_cnt stay as the reservation left them (the stores only read them)
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      const uint32_t b = E[j] >> 16, r = E[j] & 0xFFFFu;
      if (b >= nb) continue;
      if (r < sm.s_fit[b]) {
        ka->key[(uint64_t)b * ga.cap + sm.s_base[b] + r] = K[j];
      } else {
        const unsigned long long at = atomicAdd(ka->n_spill, 1ull);
        if (at < ka->spill_cap) ka->spill[at] = K[j];
      }
    }
    for (uint32_t b = tid; b < nb; b += kPartBlock) {
      const uint32_t c = sm.s_cnt[b], cp = (c + 7u) & ~7u, fit = sm.s_fit[b];
      for (uint32_t i = c; i < cp && i < fit; ++i) ka->key[(uint64_t)b * ga.cap + sm.s_base[b] + i] = 0ull;
    }
    return;
  }
#pragma unroll 2
  for (int j = 0; j < kPer; ++j) {
    const int q = q0 + j;
    const bool ok = window_valid(L, T0, q, k, in.n_bases, in.pos_lo, in.pos_hi);
    uint64_t h = 0;
    if (ok) h = gen_hash<KM>(gen_key<KM, CANON>(L, in, q, T0 + (uint64_t)q, k, rc));
    const uint32_t idx = small_pool ? fastmod32(h, fm) : (uint32_t)fastmod(h, fm);
    const uint32_t b = ok ? (idx >> bb) : nb;
    E[j] = (b << 16) | atomicAdd(&sm.s_cnt[b], 1u);
    O[j] = (idx & omask) | ltag;
  }
  sort_and_store<WIDE, kPer>(E, O, nb, sm.s_cnt, sm.s_start, sm.s_base, sm.s_fit, sm.s_rec, sm.s_gmap,
                             ga.fill, ga.overflow, ga.cap, reinterpret_cast<typename S::Rec *>(ga.rec), 0,
                             bb, ga.currents, ga.desc, ga.max_segs, (uint32_t)tile);
}

template <int KM, bool CANON, bool WIDE>
__global__ __launch_bounds__(kPartBlock) void k_part_gen(KmerInput in, int k, FastMod fm,
                                                         GenPartArgs ga) {
  __shared__ GenLds<WIDE, !CANON> sm;
  gen_tile<KM, CANON, WIDE>(in, k, fm, ga, blockIdx.x, sm);
}

// K1g<KEYS>: the grouped exact table's own partition pass for k > 32
// (NK_KMER_COMPAT u64 keys; nk_table_host.cpp::build_grouped)
template <int KM, bool CANON>
__global__ __launch_bounds__(kPartBlock) void k_part_gen_keys(KmerInput in, int k, FastMod fm,
                                                              GenPartArgs ga, GenKeyArgs ka) {
  __shared__ GenLds<false, !CANON> sm;
  gen_tile<KM, CANON, false, true>(in, k, fm, ga, blockIdx.x, sm, &ka);
}

constexpr int kSplitBlock = kPartBlock;
constexpr int kSplitPer = kPartTile / kSplitBlock;  // 16
struct SplitLds {
  using S = GenShape<false>;
  uint32_t s_cnt[kMaxSplit + 1];
  uint32_t s_start[kMaxSplit + 1];
  uint32_t s_base[kMaxSplit];
  uint32_t s_fit[kMaxSplit];
  __align__(16) uint16_t s_rec[S::kSlots];
  S::GMap s_gmap[S::kGroups];
};

// K1s work item j of `items` in all: coarse bucket cb = j % nb takes the items
// j = cb, cb + nb, ... (its count: (items - cb + nb - 1) / nb); item j splits
// its bucket's records [lo, hi) from tile j / nb on, striding by that count.
// snap_lo / snap_hi (null: 0 / the whole region): one k_part_gen launch's
// records of each coarse bucket (the pipelined split, k_gen_split).  PER
// records per lane: a tile of 8192 records goes in 16 / PER rounds of
// 512 * PER records (k_gen_split: 8, half the registers of 16).
template <int PER>
__device__ __forceinline__ void split_item(const GenPartArgs &ga, const PartArgs &pa,
                                           const unsigned long long *__restrict__ snap_lo,
                                           const unsigned long long *__restrict__ snap_hi, uint64_t j,
                                           uint64_t items, SplitLds &sm) {
  static_assert(PER % 4 == 0 && kSplitPer % PER == 0, "whole 16-B loads, whole rounds per tile");
  const int tid = threadIdx.x;
  const uint32_t nb = ga.n_buckets;
  const uint32_t cb = (uint32_t)(j % nb);
  const uint64_t stride = (items - cb + nb - 1) / nb;
  // (fill bits 40..: kept segments; the region's records are [0, min(fill, cap)),
  // multiples of 8, as are the snapshots)
  uint64_t n = snap_hi ? snap_hi[cb] : ga.fill[cb] & ((1ull << 40) - 1);
  if (n > ga.cap) n = ga.cap;
  const uint64_t lo = snap_lo ? snap_lo[cb] : 0;
  const uint32_t F = 1u << (ga.bin_bits - kBinBits);
  const uint32_t cmask = (uint32_t)((1ull << ga.bin_bits) - 1ull);
  const uint32_t *src = reinterpret_cast<const uint32_t *>(ga.rec) + (uint64_t)cb * ga.cap;
  constexpr uint64_t kRound = (uint64_t)PER * kSplitBlock;
  for (uint64_t t0 = lo + (j / nb) * kPartTile; t0 < n; t0 += stride * kPartTile) {
    for (uint64_t r0 = t0; r0 < t0 + kPartTile && r0 < n; r0 += kRound) {  // (uniform)
      __syncthreads();  // (the LDS is free: the previous round's stores read it)
      for (uint32_t f = tid; f <= F; f += kSplitBlock) sm.s_cnt[f] = 0;
      __syncthreads();
      // PER records per lane: PER / 4 16-B loads (the region is a multiple of 8
      // records and 64-record aligned; records past n are ignored)
      constexpr int kL = PER / 4;
      uint4 v[kL];
      const uint64_t i0 = r0 + (uint64_t)tid * PER;
#pragma unroll
      for (int t = 0; t < kL; ++t) {
        const uint64_t i = i0 + 4 * t;
        v[t] = i < n ? *reinterpret_cast<const uint4 *>(src + i) : make_uint4(~0u, ~0u, ~0u, ~0u);
      }
      uint32_t E[PER], O[PER];
#pragma unroll
      for (int q = 0; q < PER; ++q) {
        const uint4 &w = v[q >> 2];
        const uint32_t o = (q & 3) == 0 ? w.x : (q & 3) == 1 ? w.y : (q & 3) == 2 ? w.z : w.w;
        const bool ok = o != 0xFFFFFFFFu && i0 + q < n;
        const uint32_t f = ok ? ((o & cmask) >> kBinBits) : F;  // (lane tag bits dropped)
        E[q] = (f << 16) | atomicAdd(&sm.s_cnt[f], 1u);
        O[q] = o & (kBinsPerBucket - 1);
      }
      sort_and_store<false, PER, kSplitBlock>(E, O, F, sm.s_cnt, sm.s_start, sm.s_base, sm.s_fit,
                                              sm.s_rec, sm.s_gmap, pa.fill, pa.overflow, pa.cap,
                                              pa.off, (uint64_t)cb * F, kBinBits, pa.currents);
    }
  }
}

// K1s: one 8192-record tile of a coarse bucket (u32 offsets of 2^S bins) ->
// its 2^(S-15) fine buckets (u16 offsets), the layout k_bucket_hist reads.
// 512 threads x 16 records (256 x 32 needs 119 VGPRs: the same 32 waves of
// 16-B loads in flight per CU, no gain).  Workgroup L takes item L: the
// workgroups in flight spread over every coarse bucket (bucket-major order put
// ~1000 of them on one bucket's 32 fine fill counters at a time: 131 ms at a
// 12.5 Gbase config-5 input, profiles/r04_t3), and bucket b stays on XCD b % 8
// (nb a multiple of 8), its fine regions' partial lines in one L2.
__global__ __launch_bounds__(kSplitBlock) void k_split(GenPartArgs ga, PartArgs pa,
                                                       const unsigned long long *__restrict__ snap_lo,
                                                       const unsigned long long *__restrict__ snap_hi) {
  __shared__ SplitLds sm;
  split_item<kSplitPer>(ga, pa, snap_lo, snap_hi, blockIdx.x, gridDim.x, sm);
}

// (6 waves per SIMD: three workgroups per CU, as k_part_gen's LDS allows; the
// split's registers would otherwise leave two)
#ifndef NK_GS_WAVES
#define NK_GS_WAVES 6
#endif
#ifndef NK_GS_SPLIT_PER  // records per lane per round of the fused split (8: no spills at 6 waves)
#define NK_GS_SPLIT_PER 8
#endif
// K1g of one launch's tiles fused with K1s of the previous launch's records:
// k_part_gen is VALU-bound (SipHash) and barely slowed by a third fewer
// workgroups per CU (config 5, 12.5 Gbases: +3 % at two per CU,
// profiles/r05_b), k_split is bound by its bytes, so every workgroup hashes
// its tile and then splits one item of the previous launch's records, while
// the CU's other workgroups keep the SIMDs busy.  (Two streams, one per
// kernel, hid only ~4 of the split's 18.5 ms: the hardware kept dispatching
// the hash kernel's workgroups, r05_a/r05_b.)  One LDS union: the split's
// arrays alias the hash's.
template <int KM, bool CANON>
__global__ __launch_bounds__(kPartBlock) __attribute__((amdgpu_waves_per_eu(CANON ? NK_GS_WAVES : 4))) void k_gen_split(KmerInput in, int k, FastMod fm, GenPartArgs ga,
                                                         PartArgs pa,
                                                         const unsigned long long *__restrict__ snap_lo,
                                                         const unsigned long long *__restrict__ snap_hi) {
  __shared__ union U {
    GenLds<true, !CANON> g;
    SplitLds s;
  } sm;
  // (Measured and not kept: workgroups that either hash a tile or split an
  // item, interleaved in one grid -- the count 79.3 vs 67.8 ms, profiles/r05_n;
  // the first 256 / 512 / 768 workgroups splitting every item of the launch
  // and the rest hashing -- the step equal / +3 % / +8 %, profiles/r05_s.)
  if (blockIdx.x < in.n_tiles) gen_tile<KM, CANON, true>(in, k, fm, ga, blockIdx.x, sm.g);
  if (snap_hi) {
    __syncthreads();  // (the gen tile's last stores still read its LDS)
    split_item<NK_GS_SPLIT_PER>(ga, pa, snap_lo, snap_hi, blockIdx.x, gridDim.x, sm.s);
  }
}

// the records each coarse bucket holds now (min(fill, cap)): the upper end of
// one k_part_gen launch's records for the split that runs beside the next
__global__ void k_fill_snap(const unsigned long long *__restrict__ fill, uint32_t nb, uint64_t cap,
                            unsigned long long *__restrict__ snap) {
  for (uint32_t b = blockIdx.x * blockDim.x + threadIdx.x; b < nb; b += gridDim.x * blockDim.x) {
    const uint64_t n = fill[b] & ((1ull << 40) - 1);
    snap[b] = n < cap ? n : cap;
  }
}

// U1g: the tiles that hold records of the top rows in the kept Gen/Wide
// records.  One workgroup per (top bucket, slice): the bucket's records are
// matched against its top offsets; a hit's segment (binary search of the
// descriptors by first-record index) names its tile, which goes to the list
// once per pass (mark[tile] = epoch); lane-tagged records also set their
// lane's bit (lanes[tile][16]).  The uniques rescan then runs on the listed
// tiles only (and, tagged, hashes only the marked lanes): at config 5 (0.45
// k-mers per neuron) a fraction of the 14,000 tiles.
constexpr int kTileSeen = 256;
constexpr int kHitQueue = 8192;
template <bool WIDE>
__global__ __launch_bounds__(kHistBlock) void k_uniq_tiles(GenPartArgs ga, UniqArgs u,
                                                           const uint32_t *__restrict__ tbuckets,
                                                           const uint32_t *__restrict__ n_tb,
                                                           uint32_t slices, uint32_t *__restrict__ tiles,
                                                           uint32_t *__restrict__ n_list,
                                                           uint32_t max_list, uint32_t *__restrict__ flag,
                                                           uint32_t *__restrict__ mark, uint32_t epoch,
                                                           uint32_t *__restrict__ lanes, uint32_t qcap) {
  using Rec = typename GenShape<WIDE>::Rec;
  __shared__ uint32_t t_off[kMaxTopN];
  __shared__ uint32_t s_seen[kTileSeen];
  __shared__ uint32_t t_n, h_n;
  __shared__ uint32_t h_i[kHitQueue], h_rec[kHitQueue];  // queued hits: record index, record
  if (blockIdx.y >= *n_tb) return;  // uniform
  const uint32_t b = tbuckets[blockIdx.y], r = blockIdx.x;
  if (threadIdx.x == 0) { t_n = 0; h_n = 0; }
  // (LDS left by earlier kernels holds small integers like tile ids: a
  // sentinel, never a false duplicate)
  for (int i = threadIdx.x; i < kTileSeen; i += kHistBlock) s_seen[i] = 0xFFFFFFFFu;
  __syncthreads();
  const uint32_t omask = (uint32_t)((1ull << ga.bin_bits) - 1ull);
  for (uint32_t i = threadIdx.x; i < u.n_top; i += kHistBlock) {
    const uint64_t idx = u.top[i].idx;
    if ((idx >> ga.bin_bits) == b) t_off[atomicAdd(&t_n, 1u)] = (uint32_t)idx & omask;
  }
  __syncthreads();
  const uint32_t tn = t_n;
  uint64_t n = ga.fill[b] & ((1ull << 40) - 1);
  if (n > ga.cap) n = ga.cap;
  uint64_t n_seg = ga.fill[b] >> 40;
  if (n_seg > ga.max_segs) n_seg = ga.max_segs;
  // slice bounds on 64-record boundaries (the region base is 64-aligned): only
  // the last slice's tail is not a whole 4-record group
  auto bound = [&](uint32_t q) -> uint64_t { return q >= slices ? n : ((n * q / slices) & ~63ull); };
  const uint64_t lo = bound(r), hi = bound(r + 1);
  const Rec *src = reinterpret_cast<const Rec *>(ga.rec) + (uint64_t)b * ga.cap;
  const uint2 *d = ga.desc + (uint64_t)b * ga.max_segs;
  const bool tagged = WIDE && ga.lane_tag && lanes;
  // a record -> the list entry it adds (~0u: none): a top row's record names
  // its tile (segment binary search) and, tagged, its lane; each entry once
  // per pass (tile: mark[tile] = epoch; lane: its bit)
  auto match = [&](uint32_t rec) -> bool {
    const uint32_t off = rec & omask;
    bool h = false;
    for (uint32_t t = 0; t < tn; ++t) h |= t_off[t] == off;  // (pads never match)
    return h;
  };
  auto entry = [&](uint64_t i, uint32_t rec) -> uint32_t {
    // last segment with first record <= i: every tile adds about the same
    // number of records to a bucket, so i * n_seg / n is within a few segments
    // (a gallop from there, then a binary search: ~4 dependent loads instead
    // of ~21 over 1.5 M segments at a 12.5 Gbase input)
    uint64_t a = 0, z = n_seg;
    if (n_seg > 1) {
      uint64_t g = (uint64_t)((double)i * (double)n_seg / (double)(n ? n : 1));
      if (g >= n_seg) g = n_seg - 1;
      if (d[g].y <= i) {  // gallop up: [g, z)
        a = g;
        for (uint64_t st = 1;; st <<= 1) {
          const uint64_t t = a + st;
          if (t >= n_seg) { z = n_seg; break; }
          if (d[t].y > i) { z = t; break; }
          a = t;
        }
      } else {  // gallop down: [a, g)
        z = g;
        for (uint64_t st = 1;; st <<= 1) {
          if (z <= st) { a = 0; break; }
          const uint64_t t = z - st;
          if (d[t].y <= i) { a = t; break; }
          z = t;
        }
      }
    }
    while (z - a > 1) {
      const uint64_t m = (a + z) >> 1;
      if (d[m].y <= i) a = m;
      else z = m;
    }
    const uint32_t tile = d[a].x;
    if (tagged) {
      const uint32_t lane = rec >> ga.bin_bits, bit = 1u << (lane & 31);
      if (atomicOr(&lanes[(uint64_t)tile * kLaneWords + (lane >> 5)], bit) & bit) return ~0u;
      return (tile << 9) | lane;
    }
    // a direct-mapped LDS cache of the tiles this workgroup listed (O(1); a
    // miss only costs the global mark)
    uint32_t &seen = s_seen[tile & (kTileSeen - 1)];
    if (seen == tile) return ~0u;
    seen = tile;
    return atomicExch(&mark[tile], epoch) == epoch ? ~0u : tile;
  };
  // appends of a wave's active lanes: one counter atomic per wave (the top
  // rows are hot: thousands of records each)
  const uint32_t lane_id = threadIdx.x & 63u;
  auto append = [&](uint32_t ent) {
    const bool w = ent != ~0u;
    const uint64_t m = __ballot(w);
    if (!m) return;
    const int leader = __ffsll((long long)m) - 1;
    uint32_t base = 0;
    if ((int)lane_id == leader) base = atomicAdd(n_list, (uint32_t)__popcll(m));
    base = __shfl(base, leader, 64);
    if (!w) return;
    const uint32_t g = base + (uint32_t)__popcll(m & ((1ull << lane_id) - 1ull));
    if (g < max_list) tiles[g] = ent;
    else atomicOr(flag, 1u);  // list full: the caller rescans everything
  };
  // 4 records per lane per load (16 B wide, 8 B narrow), 4 loads in flight;
  // the block steps through its range together, so the queue can be resolved
  // whenever it is half full (a planted-repeat top row of ~800 k records gave
  // a slice ~16 k hits: past the queue they were resolved in place, one
  // dependent chain per lane -- k_uniq_tiles 19 ms at a 12.5 Gbase config-5
  // input, profiles/r04_t4)
  constexpr int kU = 4;
  constexpr uint64_t kStep = 4ull * kHistBlock;
  const uint32_t flush_at = qcap > (uint32_t)kHitQueue / 2 ? (uint32_t)kHitQueue / 2 : 0u;
  for (uint64_t base = lo; base < hi; base += kU * kStep) {
    const uint64_t i0 = base + 4ull * threadIdx.x;
    uint32_t v[kU][4];
#pragma unroll
    for (int q = 0; q < kU; ++q) {
      const uint64_t ii = i0 + q * kStep;
      if (ii + 4 <= hi) {
        if (WIDE) {
          const uint4 w = *reinterpret_cast<const uint4 *>(src + ii);
          v[q][0] = w.x; v[q][1] = w.y; v[q][2] = w.z; v[q][3] = w.w;
        } else {
          const uint2 w = *reinterpret_cast<const uint2 *>(src + ii);
          v[q][0] = w.x & 0xFFFFu; v[q][1] = w.x >> 16; v[q][2] = w.y & 0xFFFFu; v[q][3] = w.y >> 16;
        }
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[q][e] = ii + e < hi ? (uint32_t)src[ii + e] : (uint32_t)GenShape<WIDE>::kPad;
      }
    }
    // hits are queued in LDS and resolved together below: a wave resolving
    // its hits one record step at a time chains 14 dependent descriptor loads
    // per hit (measured 470 us at config 5: ~9 hits per wave, 147 k hits)
#pragma unroll
    for (int q = 0; q < kU; ++q)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const uint64_t ii = i0 + q * kStep + e;
        if (ii < hi && match(v[q][e])) {
          const uint32_t at = atomicAdd(&h_n, 1u);
          if (at < qcap) {
            h_i[at] = (uint32_t)ii;
            h_rec[at] = v[q][e];
          } else {
            append(entry(ii, v[q][e]));  // queue full: resolved in place
          }
        }
      }
    __syncthreads();
    const uint32_t nh = h_n;
    __syncthreads();  // every lane has read h_n before the next round adds to it
    if (nh > flush_at) {  // (block-uniform) resolve the queued hits, all lanes together
      const uint32_t nq = nh < qcap ? nh : qcap;
      for (uint32_t j = threadIdx.x; j < nq; j += kHistBlock) append(entry(h_i[j], h_rec[j]));
      __syncthreads();
      if (threadIdx.x == 0) h_n = 0;
      __syncthreads();
    }
  }
  __syncthreads();
  const uint32_t nq = h_n < qcap ? h_n : qcap;
  for (uint32_t j = threadIdx.x; j < nq; j += kHistBlock) append(entry(h_i[j], h_rec[j]));
}

// K1k: the exact table's distinct keys -> kmer_per_neuron, as a count of a key
// array through the same partition + LDS histograms (a per-key global atomic,
// k_kpn, runs at the memory side: 4.2 ms for 113 M keys, profiles/r02_s18).
// Lane j of a tile takes keys T0 + j * kPartBlock + lane (coalesced loads; the
// record order inside a bucket does not matter to a histogram).
template <bool W128, bool WIDE>
__global__ __launch_bounds__(kPartBlock) void k_part_keys(const uint64_t *__restrict__ keys,
                                                          const unsigned long long *__restrict__ n_keys,
                                                          FastMod fm, GenPartArgs ga) {
  using S = GenShape<WIDE>;
  __shared__ uint32_t s_cnt[S::kMaxB + 1];
  __shared__ uint32_t s_start[S::kMaxB + 1];
  __shared__ uint32_t s_base[S::kMaxB];
  __shared__ uint32_t s_fit[S::kMaxB];
  __shared__ __align__(16) typename S::Rec s_rec[S::kSlots];
  __shared__ typename S::GMap s_gmap[S::kGroups];
  const uint64_t n = *n_keys;
  const uint64_t T0 = (uint64_t)blockIdx.x * kPartTile;
  if (T0 >= n) return;  // uniform: the grid is sized for the key bound
  const int tid = threadIdx.x;
  const uint32_t nb = ga.n_buckets;
  const int bb = ga.bin_bits;
  const bool small_pool = fm.p < (1ull << 30);
  const uint32_t omask = (uint32_t)((1ull << bb) - 1ull);
  for (uint32_t b = tid; b <= nb; b += kPartBlock) s_cnt[b] = 0;
  __syncthreads();
  uint32_t E[kPer], O[kPer];
#pragma unroll 4
  for (int j = 0; j < kPer; ++j) {
    const uint64_t i = T0 + (uint64_t)j * kPartBlock + (uint64_t)tid;
    const bool ok = i < n;
    uint64_t h = 0;
    if (ok) h = W128 ? sip13_u128(keys[2 * i], keys[2 * i + 1]) : sip13_u64(keys[i]);
    const uint32_t idx = small_pool ? fastmod32(h, fm) : (uint32_t)fastmod(h, fm);
    const uint32_t b = ok ? (idx >> bb) : nb;
    E[j] = (b << 16) | atomicAdd(&s_cnt[b], 1u);
    O[j] = idx & omask;
  }
  sort_and_store<WIDE, kPer>(E, O, nb, s_cnt, s_start, s_base, s_fit, s_rec, s_gmap, ga.fill,
                             ga.overflow, ga.cap, reinterpret_cast<typename S::Rec *>(ga.rec), 0,
                             bb, ga.currents);
}

__global__ void k_kpn_fold(const uint32_t *__restrict__ partials, uint32_t slices, uint64_t pool,
                           unsigned long long *__restrict__ cur, uint32_t *__restrict__ kpn) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < pool;
       i += (uint64_t)gridDim.x * blockDim.x) {
    unsigned long long s = cur[i];
    if (s) cur[i] = 0;
    for (uint32_t r = 0; r < slices; ++r) s += partials[(uint64_t)r * pool + i];
    kpn[i] = (uint32_t)s;
  }
}

// ---------------------------------------------------------------------------
hipError_t launch_part_keys(const uint64_t *keys, const unsigned long long *n_keys, uint64_t max_n,
                            int wpk, uint64_t pool, const GenPartArgs &ga, int wide, hipStream_t s) {
  if (!max_n) return hipSuccess;
  if (pool == 0 || pool > (1ull << 31) || (wpk != 1 && wpk != 2)) return hipErrorInvalidValue;
  if (wide ? (ga.n_buckets > (uint32_t)kWideMaxBuckets || ga.bin_bits < kBinBits ||
              ga.bin_bits - kBinBits > kMaxSplitBits)
           : (ga.n_buckets > (uint32_t)kMaxBuckets || ga.bin_bits != kBinBits))
    return hipErrorInvalidValue;
  const uint64_t tiles = (max_n + kPartTile - 1) / kPartTile;
  if (tiles > 0x7FFFFFFFull) return hipErrorInvalidValue;
  const FastMod fm = make_fastmod(pool);
  const dim3 g((unsigned)tiles), b(kPartBlock);
  if (wpk == 2) {
    if (wide) hipLaunchKernelGGL((k_part_keys<true, true>), g, b, 0, s, keys, n_keys, fm, ga);
    else hipLaunchKernelGGL((k_part_keys<true, false>), g, b, 0, s, keys, n_keys, fm, ga);
  } else {
    if (wide) hipLaunchKernelGGL((k_part_keys<false, true>), g, b, 0, s, keys, n_keys, fm, ga);
    else hipLaunchKernelGGL((k_part_keys<false, false>), g, b, 0, s, keys, n_keys, fm, ga);
  }
  return hipGetLastError();
}

hipError_t launch_kpn_fold(const uint32_t *partials, uint32_t slices, uint64_t pool,
                           unsigned long long *cur, uint32_t *kpn, hipStream_t s) {
  if (!pool) return hipSuccess;
  unsigned g = (unsigned)((pool + 255) / 256);
  if (g > 4096) g = 4096;
  hipLaunchKernelGGL(k_kpn_fold, dim3(g), dim3(256), 0, s, partials, slices, pool, cur, kpn);
  return hipGetLastError();
}

hipError_t launch_part_gen(const KmerInput &in, int k, int canonical, int km, uint64_t pool,
                           const GenPartArgs &ga, int wide, hipStream_t s) {
  if (!in.n_tiles) return hipSuccess;
  if (pool == 0 || pool > (1ull << 31) || km < 0 || km > 2) return hipErrorInvalidValue;
  if (wide ? (ga.n_buckets > (uint32_t)kWideMaxBuckets || ga.bin_bits < kBinBits ||
              ga.bin_bits - kBinBits > kMaxSplitBits)
           : (ga.n_buckets > (uint32_t)kMaxBuckets || ga.bin_bits != kBinBits))
    return hipErrorInvalidValue;
  if ((km == 0 && k > 32) || (km == 1 && (k <= 32 || k > 64)) || (km == 2 && k > 64) || k < 1)
    return hipErrorInvalidValue;
  const FastMod fm = make_fastmod(pool);
  const dim3 g((unsigned)in.n_tiles), b(kPartBlock);
#define NK_GEN(KM_, C_, W_) hipLaunchKernelGGL((k_part_gen<KM_, C_, W_>), g, b, 0, s, in, k, fm, ga)
#define NK_GEN_W(KM_, C_) \
  do {                    \
    if (wide) NK_GEN(KM_, C_, true); else NK_GEN(KM_, C_, false); \
  } while (0)
  if (canonical) {
    if (km == 0) NK_GEN_W(0, true);
    else if (km == 1) NK_GEN_W(1, true);
    else NK_GEN_W(2, true);
  } else {
    if (km == 0) NK_GEN_W(0, false);
    else if (km == 1) NK_GEN_W(1, false);
    else NK_GEN_W(2, false);
  }
#undef NK_GEN_W
#undef NK_GEN
  return hipGetLastError();
}

hipError_t launch_part_gen_keys(const KmerInput &in, int k, int canonical, int km, uint64_t pool,
                                const GenPartArgs &ga, const GenKeyArgs &ka, hipStream_t s) {
  if (!in.n_tiles) return hipSuccess;
  if (pool == 0 || pool > (1ull << 31) || km < 0 || km > 1 || !ka.key || !ka.n_spill) return hipErrorInvalidValue;
  if (ga.n_buckets > (uint32_t)kMaxBuckets || ga.bin_bits < 12 || ga.bin_bits > kBinBits)
    return hipErrorInvalidValue;
  if ((km == 0 && k > 32) || (km == 1 && (k <= 32 || k > 64)) || k < 1) return hipErrorInvalidValue;
  const FastMod fm = make_fastmod(pool);
  const dim3 g((unsigned)in.n_tiles), b(kPartBlock);
#define NK_GK(KM_, C_) hipLaunchKernelGGL((k_part_gen_keys<KM_, C_>), g, b, 0, s, in, k, fm, ga, ka)
  if (canonical) {
    if (km == 0) NK_GK(0, true);
    else NK_GK(1, true);
  } else {
    if (km == 0) NK_GK(0, false);
    else NK_GK(1, false);
  }
#undef NK_GK
  return hipGetLastError();
}

hipError_t launch_uniq_tiles(const GenPartArgs &ga, int wide, const UniqArgs &u,
                             const uint32_t *tbuckets, const uint32_t *n_tb, uint32_t max_tb,
                             uint32_t slices, uint32_t *tiles, uint32_t *n_list, uint32_t max_list,
                             uint32_t *flag, uint32_t *mark, uint32_t epoch, uint32_t *lanes,
                             uint32_t hit_queue, hipStream_t s) {
  if (!max_tb || !ga.desc) return hipSuccess;
  const uint32_t qcap = hit_queue < (uint32_t)kHitQueue ? hit_queue : (uint32_t)kHitQueue;
  const dim3 g(slices ? slices : 1, max_tb), b(kHistBlock);
  if (wide) hipLaunchKernelGGL(k_uniq_tiles<true>, g, b, 0, s, ga, u, tbuckets, n_tb, slices ? slices : 1,
                               tiles, n_list, max_list, flag, mark, epoch, lanes, qcap);
  else hipLaunchKernelGGL(k_uniq_tiles<false>, g, b, 0, s, ga, u, tbuckets, n_tb, slices ? slices : 1,
                          tiles, n_list, max_list, flag, mark, epoch, lanes, qcap);
  return hipGetLastError();
}

hipError_t launch_split(const GenPartArgs &ga, const PartArgs &pa, hipStream_t s,
                        const unsigned long long *snap_lo, const unsigned long long *snap_hi,
                        uint64_t est_records) {
  if (!ga.n_buckets) return hipSuccess;
  if (ga.bin_bits < kBinBits || ga.bin_bits - kBinBits > kMaxSplitBits) return hipErrorInvalidValue;
  // tiles per coarse bucket in the grid: the region (whole split), or the
  // expected share of a range (1.25x + one tile; a bucket past it loops)
  uint64_t tx = (ga.cap + kPartTile - 1) / kPartTile;
  if (snap_hi && est_records) {
    const uint64_t t = (est_records / ga.n_buckets * 5 / 4 + kPartTile - 1) / kPartTile + 1;
    if (t < tx) tx = t;
  }
  if (!tx) tx = 1;
  if (tx * ga.n_buckets > 0x7FFFFFFFull) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_split, dim3((unsigned)(tx * ga.n_buckets)), dim3(kSplitBlock), 0, s, ga, pa,
                     snap_lo, snap_hi);
  return hipGetLastError();
}

hipError_t launch_gen_split(const KmerInput &in, int k, int canonical, int km, uint64_t pool,
                            const GenPartArgs &ga, const PartArgs &pa,
                            const unsigned long long *snap_lo, const unsigned long long *snap_hi,
                            uint64_t split_records, hipStream_t s) {
  if (pool == 0 || pool > (1ull << 31) || km < 0 || km > 2) return hipErrorInvalidValue;
  if (ga.n_buckets > (uint32_t)kWideMaxBuckets || ga.bin_bits < kBinBits ||
      ga.bin_bits - kBinBits > kMaxSplitBits)
    return hipErrorInvalidValue;
  if ((km == 0 && k > 32) || (km == 1 && (k <= 32 || k > 64)) || (km == 2 && k > 64) || k < 1)
    return hipErrorInvalidValue;
  // at least the tiles to hash, and enough split items for the previous
  // launch's records (~1.1 tiles each: a bucket past its share loops)
  uint64_t grid = in.n_tiles;
  if (snap_hi) {
    const uint64_t want = (split_records / ga.n_buckets / kPartTile + 1) * ga.n_buckets;
    if (want > grid) grid = want;
  }
  if (!grid) return hipSuccess;
  if (grid > 0x7FFFFFFFull) return hipErrorInvalidValue;
  const FastMod fm = make_fastmod(pool);
  const dim3 g((unsigned)grid), b(kPartBlock);
#define NK_GS(KM_, C_) hipLaunchKernelGGL((k_gen_split<KM_, C_>), g, b, 0, s, in, k, fm, ga, pa, snap_lo, snap_hi)
  if (canonical) {
    if (km == 0) NK_GS(0, true);
    else if (km == 1) NK_GS(1, true);
    else NK_GS(2, true);
  } else {
    if (km == 0) NK_GS(0, false);
    else if (km == 1) NK_GS(1, false);
    else NK_GS(2, false);
  }
#undef NK_GS
  return hipGetLastError();
}

hipError_t launch_fill_snap(const GenPartArgs &ga, unsigned long long *snap, hipStream_t s) {
  if (!ga.n_buckets) return hipSuccess;
  hipLaunchKernelGGL(k_fill_snap, dim3((ga.n_buckets + 255) / 256), dim3(256), 0, s, ga.fill,
                     ga.n_buckets, ga.cap, snap);
  return hipGetLastError();
}

}  // namespace nk
