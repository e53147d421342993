// nk_tile.h — LDS staging of one tile of bases and per-position k-mer keys
// (k <= 32), shared by the counting, partitioning and uniques kernels.
//
// A tile covers TILE k-mer start positions [T0, T0+TILE).  Its bytes plus a
// 64-base halo are loaded with coalesced 16-B loads and converted ONCE into
//   F   forward 2-bit codes, MSB-first   (base i at bits 31-2i.. of word i/16)
//   R   complement 2-bit codes, LSB-first (base i at bits 2i.. of word i/16)
//   INV invalid-byte bits, LSB-first     (non-ACGT bytes, pack_kmer's skip set)
//   WIN invalid-window bits               (window crosses a record end)
// so that a lane extracts any window's forward value and reverse complement
// with two funnel shifts: no per-k-mer rolling, no per-lane serial chain.
// Code tables: A/a 0, C/c 1, G/g 2, T/t 3, anything else 0 on BOTH strands
// (src/models.rs:231-251) — exactly what the reference's rolling hash sees.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "nk_kernels.h"

namespace nk {

__device__ __forceinline__ uint32_t eq_bytes(uint32_t t, uint32_t c) {
  uint32_t z = t ^ c;
  return ~(((z & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | z) & 0x80808080u;  // 0x80 where byte == c
}

struct Conv4 {
  uint32_t fnib;  // 4 forward codes, first base in bits 7:6
  uint32_t rnib;  // 4 complement codes, first base in bits 1:0
  uint32_t inv;   // 4 invalid-byte bits, first base in bit 0
};

// Four bytes -> codes, in ~14 VALU ops: code = ((x>>1) ^ (x>>2)) & 3 per byte
// (A/a 0, C/c 1, G/g 2, T/t 3); a byte is valid iff (byte | 0x20) equals the
// lowercase letter of its own code, looked up with one v_perm_b32; the 2-bit
// fields are gathered into byte 3 of a product by one multiply each (the
// multipliers place field i at 30-2i / 24+2i / 28+i with no overlapping or
// carrying partial products).  Equal to the byte-compare form on all 2^32
// words (tools/conv4_check.cpp).
struct Conv4P {
  uint32_t pf;  // forward codes in bits 31:24, first base in 31:30
  uint32_t pr;  // complement codes in bits 31:24, first base in 25:24
  uint32_t pi;  // invalid-byte bits in bits 31:28, first base in 28
};

__device__ __forceinline__ Conv4P conv4p(uint32_t x, bool want_inv = true) {
  const uint32_t code = ((x >> 1) ^ (x >> 2)) & 0x03030303u;
  const uint32_t expect = __builtin_amdgcn_perm(0u, 0x74676361u, code);  // "acgt"[code]
  const uint32_t z = (x | 0x20202020u) ^ expect;
  const uint32_t valid = ~(((z & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | z) & 0x80808080u;
  const uint32_t vm3 = (valid >> 6) | (valid >> 7);  // 0x03 per valid byte
  Conv4P o;
  o.pf = (code & vm3) * 0x40100401u;
  o.pr = (~code & vm3) * 0x01041040u;
  o.pi = want_inv ? ((~valid >> 7) & 0x01010101u) * 0x10204080u : 0u;
  return o;
}

__device__ __forceinline__ Conv4 conv4(uint32_t x) {
  const Conv4P p = conv4p(x);
  return Conv4{p.pf >> 24, p.pr >> 24, p.pi >> 28};
}

__device__ __forceinline__ bool valid_byte(uint8_t b) {
  uint32_t t = b | 0x20u;
  return (t == 'a') | (t == 'c') | (t == 'g') | (t == 't');
}
__device__ __forceinline__ uint32_t code_of(uint8_t b) {
  return valid_byte(b) ? (((uint32_t)b >> 1) ^ ((uint32_t)b >> 2)) & 3u : 0u;
}
__device__ __forceinline__ uint32_t comp_of(uint8_t b) {
  return valid_byte(b) ? ((((uint32_t)b >> 1) ^ ((uint32_t)b >> 2)) & 3u) ^ 3u : 0u;
}

template <int TILE, bool RAW>
struct TileLds {
  static constexpr int kChunks = (TILE + 64) / 16;
  uint32_t F[kChunks + 2];
  uint32_t R[kChunks + 2];
  uint16_t INV[kChunks + 4];
  uint32_t WIN[TILE / 32];
  uint4 RAWB[RAW ? kChunks : 1];
};

// Loads the tile, builds F/R/INV/WIN (INV only when WANT_INV: the canonical
// partitioned count never reads it).  Ends with a __syncthreads().
template <int TILE, int BLOCK, bool RAW, bool WANT_INV = true>
__device__ __forceinline__ void stage_tile(TileLds<TILE, RAW> &L, const KmerInput &in,
                                           uint64_t tile, int k) {
  constexpr int kChunks = TileLds<TILE, RAW>::kChunks;
  const int tid = threadIdx.x;
  const uint64_t T0 = tile * (uint64_t)TILE;
  const uint64_t n_bases = in.n_bases;
  // all of this thread's 16-B loads are issued before any is consumed; the
  // input's last partial chunk takes a byte path afterwards
  constexpr int kIter = (kChunks + BLOCK - 1) / BLOCK;
  uint4 vv[kIter];
#pragma unroll
  for (int i = 0; i < kIter; ++i) {
    const int c = tid + i * BLOCK;
    const uint64_t g = T0 + 16ull * c;
    vv[i] = (c < kChunks && g + 16 <= n_bases) ? *reinterpret_cast<const uint4 *>(in.bases + g)
                                               : make_uint4(0, 0, 0, 0);
  }
#pragma unroll
  for (int i = 0; i < kIter; ++i) {
    const int c = tid + i * BLOCK;
    if (c >= kChunks) break;
    const uint64_t g = T0 + 16ull * c;
    uint4 v = vv[i];
    if (g + 16 > n_bases) {
      uint32_t w[4] = {0, 0, 0, 0};
      for (int j = 0; j < 16; ++j)
        if (g + j < n_bases) w[j >> 2] |= (uint32_t)in.bases[g + j] << (8 * (j & 3));
      v = make_uint4(w[0], w[1], w[2], w[3]);
    }
    const Conv4P a = conv4p(v.x, WANT_INV), b = conv4p(v.y, WANT_INV),
                 cc = conv4p(v.z, WANT_INV), d = conv4p(v.w, WANT_INV);
    // byte 3 of each product, MSB-first (F) / LSB-first (R): two v_perm + or
    L.F[c] = __builtin_amdgcn_perm(a.pf, b.pf, 0x07030C0Cu) |
             __builtin_amdgcn_perm(cc.pf, d.pf, 0x0C0C0703u);
    L.R[c] = __builtin_amdgcn_perm(b.pr, a.pr, 0x0C0C0703u) |
             __builtin_amdgcn_perm(d.pr, cc.pr, 0x07030C0Cu);
    if (WANT_INV)
      L.INV[c] = (uint16_t)((a.pi >> 28) | ((b.pi >> 28) << 4) | ((cc.pi >> 28) << 8) |
                            ((d.pi >> 28) << 12));
    if (RAW) L.RAWB[c] = v;
  }
  if (tid < 2) { L.F[kChunks + tid] = 0; L.R[kChunks + tid] = 0; }
  if (WANT_INV && tid < 4) L.INV[kChunks + tid] = 0;
  for (int i = tid; i < TILE / 32; i += BLOCK) L.WIN[i] = 0;
  __syncthreads();
  // windows crossing a record end (or running past the input) are not k-mers
  const uint64_t limit = T0 + TILE + (uint64_t)k - 1;
  const uint64_t r0 = in.tile_rec[tile - in.tile_base];
  for (uint64_t r = r0 + 1 + tid; r <= in.n_recs; r += BLOCK) {
    uint64_t b = in.offsets[r];
    if (b >= limit) break;
    uint64_t lo = (b + 1 > (uint64_t)k) ? b + 1 - (uint64_t)k : 0;
    if (lo < T0) lo = T0;
    uint64_t hi = b < T0 + TILE ? b : T0 + TILE;
    for (uint64_t q = lo - T0; q < hi - T0;) {
      uint32_t w = (uint32_t)(q >> 5), s = (uint32_t)(q & 31);
      uint32_t nb = (uint32_t)((hi - T0) - q);
      uint32_t take = nb < 32 - s ? nb : 32 - s;
      uint32_t bits = (take == 32 ? 0xFFFFFFFFu : ((1u << take) - 1u)) << s;
      atomicOr(&L.WIN[w], bits);
      q += take;
    }
  }
  __syncthreads();
}

// true if local position q starts a k-mer of some record
template <int TILE, bool RAW>
__device__ __forceinline__ bool window_valid(const TileLds<TILE, RAW> &L, uint64_t T0, int q,
                                             int k, uint64_t n_bases, uint64_t pos_lo = 0,
                                             uint64_t pos_hi = ~0ull) {
  const uint64_t p = T0 + (uint64_t)q;
  return p + (uint64_t)k <= n_bases && p >= pos_lo && p < pos_hi &&
         !((L.WIN[q >> 5] >> (q & 31)) & 1u);
}

// The reference's key for the window at local position q (k <= 32):
// canonical = min(forward, reverse complement) (src/models.rs:284-286,
// src/spiking_hash.rs:108,121-122); otherwise pack_kmer, which skips
// non-ACGT bytes (src/utils.rs:26-39).
template <int TILE, bool RAW, bool CANON>
__device__ __forceinline__ uint64_t window_key(const TileLds<TILE, RAW> &L, int q, int k) {
  const int twok = 2 * k;
  const int w = q >> 4;
  const int s = 2 * (q & 15);
  uint64_t hi64 = ((uint64_t)L.F[w] << 32) | L.F[w + 1];
  uint64_t x = (hi64 << s) | (((uint64_t)L.F[w + 2] << s) >> 32);
  uint64_t fwd = x >> (64 - twok);
  if (CANON) {
    const uint64_t mask2k = (k >= 32) ? ~0ULL : ((1ULL << twok) - 1ULL);
    uint64_t lo64 = ((uint64_t)L.R[w + 1] << 32) | L.R[w];
    uint64_t y = (lo64 >> s) | (((uint64_t)L.R[w + 2] << 32) << (32 - s));
    uint64_t rev = y & mask2k;
    return fwd < rev ? fwd : rev;
  } else {
    const uint32_t kmask = (k >= 32) ? 0xFFFFFFFFu : ((1u << k) - 1u);
    const int iw = q >> 4, is = q & 15;
    uint64_t z = ((uint64_t)L.INV[iw] | ((uint64_t)L.INV[iw + 1] << 16) |
                  ((uint64_t)L.INV[iw + 2] << 32) | ((uint64_t)L.INV[iw + 3] << 48)) >> is;
    if (!((uint32_t)z & kmask)) return fwd;
    const uint8_t *raw = reinterpret_cast<const uint8_t *>(L.RAWB);
    uint64_t pk = 0;
    for (int i = 0; i < k; ++i) {
      uint8_t bb = raw[q + i];
      if (valid_byte(bb)) pk = (pk << 2) | code_of(bb);
    }
    return pk;
  }
}

// --kmer-width=128 key of the window at local position q (k <= 64): the 128
// bases from q out of five code words, fwd = the top 2k bits (MSB-first
// stream), rev = the low 2k bits of the LSB-first complement stream;
// canonical = min as u128.  Non-canonical: pack_kmer in 128 bits.
struct Key128 {
  uint64_t lo, hi;
};
// (non-short-circuit: three 64-bit compares whose masks combine on the scalar
// unit; the ?: form cost five more VALU instructions per key, v_cndmask
// chains over booleans)
__device__ __forceinline__ bool key128_less(const Key128 &a, const Key128 &b) {
  return (a.hi < b.hi) | ((a.hi == b.hi) & (a.lo < b.lo));
}
template <int TILE, bool RAW, bool CANON>
__device__ __forceinline__ Key128 window_key128(const TileLds<TILE, RAW> &L, int q, int k) {
  const int w = q >> 4, s = 2 * (q & 15);
  uint32_t W[4];  // bases q .. q+63, MSB-first, W[0] most significant
#pragma unroll
  for (int c = 0; c < 4; ++c)
    W[c] = (uint32_t)(((((uint64_t)L.F[w + c] << 32) | L.F[w + c + 1]) << s) >> 32);
  uint64_t vhi = ((uint64_t)W[0] << 32) | W[1], vlo = ((uint64_t)W[2] << 32) | W[3];
  // fwd = V >> (128 - 2k)
  const int sh = 128 - 2 * k;  // 0 .. 126
  Key128 fwd;
  if (sh >= 64) {
    fwd.lo = vhi >> (sh - 64);
    fwd.hi = 0;
  } else if (sh == 0) {
    fwd.lo = vlo;
    fwd.hi = vhi;
  } else {
    fwd.lo = (vlo >> sh) | (vhi << (64 - sh));
    fwd.hi = vhi >> sh;
  }
  if (CANON) {
    uint32_t Y[4];  // LSB-first complement stream from bit s: Y[0] least significant
#pragma unroll
    for (int c = 0; c < 4; ++c)
      Y[c] = (uint32_t)(((((uint64_t)L.R[w + c + 1] << 32) | L.R[w + c]) >> s));
    Key128 rev;
    rev.lo = ((uint64_t)Y[1] << 32) | Y[0];
    rev.hi = ((uint64_t)Y[3] << 32) | Y[2];
    if (k < 32) {
      rev.lo &= (1ULL << (2 * k)) - 1ULL;
      rev.hi = 0;
    } else if (k < 64) {
      rev.hi &= (1ULL << (2 * k - 64)) - 1ULL;
    }
    return key128_less(rev, fwd) ? rev : fwd;
  } else {
    const int iw = q >> 4, is = q & 15;
    const uint64_t z0 = ((uint64_t)L.INV[iw] | ((uint64_t)L.INV[iw + 1] << 16) |
                         ((uint64_t)L.INV[iw + 2] << 32) | ((uint64_t)L.INV[iw + 3] << 48));
    const uint64_t z = (z0 >> is) | (is ? ((uint64_t)L.INV[iw + 4] << (64 - is)) : 0ULL);
    const uint64_t kmask = k >= 64 ? ~0ULL : ((1ULL << k) - 1ULL);
    if (!(z & kmask)) return fwd;
    const uint8_t *raw = reinterpret_cast<const uint8_t *>(L.RAWB);
    Key128 pk{0, 0};
    for (int i = 0; i < k; ++i) {
      uint8_t bb = raw[q + i];
      if (valid_byte(bb)) {
        pk.hi = (pk.hi << 2) | (pk.lo >> 62);
        pk.lo = (pk.lo << 2) | code_of(bb);
      }
    }
    return pk;
  }
}

// k > 32, NK_KMER_COMPAT: the reference's release-build key of the window at
// absolute position p of the record starting at s0 (src/models.rs:188,
// 192-194,260-266; src/utils.rs:36): forward = the last 32 bases; reverse =
// the masked-shift residue of init for the first 32 slides plus the last
// <= 31 inserted complements at bit (2(k-1) & 63) - 2t.
template <bool CANON>
__device__ __forceinline__ uint64_t compat_key(const uint8_t *b, uint64_t s0, uint64_t p, int k) {
  if (CANON) {
    const uint32_t sh = (uint32_t)((2 * (k - 1)) & 63);
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
    return fwd < rev ? fwd : rev;
  }
  uint64_t pk = 0;
  for (int i = 0; i < k; ++i) {
    const uint8_t bb = b[p + i];
    if (valid_byte(bb)) pk = (pk << 2) | code_of(bb);
  }
  return pk;
}

// Same key straight from global memory (rare: uniques hits only).
template <bool CANON>
__device__ __forceinline__ uint64_t global_window_key(const uint8_t *b, uint64_t p, int k) {
  if (CANON) {
    uint64_t fwd = 0, rev = 0;
    for (int i = 0; i < k; ++i) {
      fwd = (fwd << 2) | code_of(b[p + i]);
      rev |= (uint64_t)comp_of(b[p + i]) << (2 * i);
    }
    return fwd < rev ? fwd : rev;
  } else {
    uint64_t pk = 0;
    for (int i = 0; i < k; ++i) {
      uint8_t bb = b[p + i];
      if (valid_byte(bb)) pk = (pk << 2) | code_of(bb);
    }
    return pk;
  }
}

// --kmer-width=128 key straight from global memory (window_key128's value;
// uniques hits only): canonical = min(fwd, reverse complement) as u128,
// otherwise pack_kmer over the valid bytes
template <bool CANON>
__device__ __forceinline__ Key128 global_window_key128(const uint8_t *b, uint64_t p, int k) {
  Key128 fwd{0, 0}, rev{0, 0};
  for (int i = 0; i < k; ++i) {
    const uint8_t x = b[p + i];
    if (!CANON && !valid_byte(x)) continue;  // pack_kmer skips the byte
    const uint64_t c = code_of(x);
    fwd.hi = (fwd.hi << 2) | (fwd.lo >> 62);
    fwd.lo = (fwd.lo << 2) | c;
    if (CANON) {
      const uint64_t r = comp_of(x);
      if (i < 32) rev.lo |= r << (2 * i);
      else rev.hi |= r << (2 * i - 64);
    }
  }
  if (!CANON) return fwd;
  return key128_less(rev, fwd) ? rev : fwd;
}

}  // namespace nk
