// nk_gen.h — keys of every key mode from a staged 8192-position tile (the
// generic partition, nk_wide.hip, and its uniques rescan, nk_kernels.hip).
//   KM 0  k <= 32: the reference's u64 key (canonical min / pack_kmer)
//   KM 1  k > 32 (<= 64), release-build u64 semantics (NK_KMER_COMPAT,
//         src/models.rs:188,192-194,260-266): forward = the last 32 bases;
//         reverse = the last k-32 inserted complements once the record's init
//         residue is shifted out (32 slides), else compat_key from HBM
//   KM 2  --kmer-width=128: u128 key (SipHash over 16 LE bytes)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "nk_device.h"
#include "nk_kernels.h"
#include "nk_tile.h"

namespace nk {

constexpr int kPer = kPartTile / kPartBlock;  // 16 consecutive positions per lane

// forward codes of the n (1..32) bases from local position q, MSB-first
template <int TILE, bool RAW>
__device__ __forceinline__ uint64_t lds_fwd(const TileLds<TILE, RAW> &L, int q, int n) {
  const int w = q >> 4, s = 2 * (q & 15);
  const uint64_t hi64 = ((uint64_t)L.F[w] << 32) | L.F[w + 1];
  const uint64_t x = (hi64 << s) | (((uint64_t)L.F[w + 2] << s) >> 32);
  return x >> (64 - 2 * n);
}

// complement codes of the n (1..32) bases from q, LSB-first (base q at bits 0-1)
template <int TILE, bool RAW>
__device__ __forceinline__ uint64_t lds_rev(const TileLds<TILE, RAW> &L, int q, int n) {
  const int w = q >> 4, s = 2 * (q & 15);
  const uint64_t lo64 = ((uint64_t)L.R[w + 1] << 32) | L.R[w];
  const uint64_t y = (lo64 >> s) | ((((uint64_t)L.R[w + 2]) << 32) << (32 - s));
  return n >= 32 ? y : y & ((1ull << (2 * n)) - 1ull);
}

// 64 invalid-byte bits of positions q .. q+63
template <int TILE, bool RAW>
__device__ __forceinline__ uint64_t lds_inv64(const TileLds<TILE, RAW> &L, int q) {
  const int iw = q >> 4, is = q & 15;
  const uint64_t z0 = ((uint64_t)L.INV[iw] | ((uint64_t)L.INV[iw + 1] << 16) |
                       ((uint64_t)L.INV[iw + 2] << 32) | ((uint64_t)L.INV[iw + 3] << 48));
  return (z0 >> is) | (is ? ((uint64_t)L.INV[iw + 4] << (64 - is)) : 0ULL);
}

// Largest r in [lo, n_recs) with offsets[r] <= p (offsets[lo] <= p): galloping
// then binary search, a few dependent loads per lane.
__device__ __forceinline__ uint64_t rec_of(const uint64_t *__restrict__ offs, uint64_t n_recs,
                                           uint64_t lo, uint64_t p) {
  uint64_t step = 1, hi = lo + 1;
  while (hi < n_recs && offs[hi] <= p) {
    lo = hi;
    step <<= 1;
    hi = lo + step;
  }
  if (hi > n_recs) hi = n_recs;
  while (hi - lo > 1) {  // offsets[lo] <= p < offsets[hi] (or hi == n_recs)
    const uint64_t m = (lo + hi) >> 1;
    if (offs[m] <= p) lo = m;
    else hi = m;
  }
  return lo;
}

struct RecCursor {  // KM 1: the record holding the lane's current position
  uint64_t r = 0, s0 = 0, e0 = 0;
};

template <int KM>
__device__ __forceinline__ void rec_cursor_init(RecCursor &c, const KmerInput &in, uint64_t p0,
                                                uint64_t ti) {  // ti: tile - in.tile_base
  if (KM != 1 || !in.n_recs) return;
  c.r = rec_of(in.offsets, in.n_recs, in.tile_rec[ti], p0);
  c.s0 = in.offsets[c.r];
  c.e0 = in.offsets[c.r + 1];
}

// Key of the valid window at local q (absolute p) of a tile staged with
// stage_tile<kPartTile, kPartBlock, !CANON>; KM 0/1 return it in .lo.
// Positions of one lane must come in increasing order (KM 1 cursor).
template <int KM, bool CANON, bool RAW>
__device__ __forceinline__ Key128 gen_key(const TileLds<kPartTile, RAW> &L, const KmerInput &in,
                                          int q, uint64_t p, int k, RecCursor &c) {
  Key128 out{0, 0};
  if (KM == 2) return window_key128<kPartTile, RAW, CANON>(L, q, k);
  if (KM == 0) {
    out.lo = window_key<kPartTile, RAW, CANON>(L, q, k);
    return out;
  }
  while (c.e0 <= p && c.r + 1 < in.n_recs) {  // lanes cross few record starts
    ++c.r;
    c.s0 = c.e0;
    c.e0 = in.offsets[c.r + 1];
  }
  if (CANON) {
    if (p - c.s0 >= 32) {  // past the init residue: both halves from LDS
      const uint64_t fwd = lds_fwd(L, q + k - 32, 32);
      const uint64_t rev = lds_rev(L, q + 32, k - 32);
      out.lo = fwd < rev ? fwd : rev;
    } else {
      out.lo = compat_key<true>(in.bases, c.s0, p, k);
    }
    return out;
  }
  const uint64_t kmask = k >= 64 ? ~0ull : ((1ull << k) - 1ull);
  if (!(lds_inv64(L, q) & kmask)) {
    out.lo = lds_fwd(L, q + k - 32, 32);  // pack_kmer keeps the last 32 bases
    return out;
  }
  const uint8_t *raw = reinterpret_cast<const uint8_t *>(L.RAWB);
  uint64_t pk = 0;
  for (int i = 0; i < k; ++i) {
    const uint8_t x = raw[q + i];
    if (valid_byte(x)) pk = (pk << 2) | code_of(x);
  }
  out.lo = pk;
  return out;
}

template <int KM>
__device__ __forceinline__ uint64_t gen_hash(const Key128 &key) {
  return KM == 2 ? sip13_u128(key.lo, key.hi) : sip13_u64(key.lo);
}

}  // namespace nk
