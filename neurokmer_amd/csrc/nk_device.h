// nk_device.h — device-side building blocks shared by the NeuroKmer gfx950 kernels.
//
// Everything here is the MI355X restatement of the reference's per-k-mer math:
//   * SipHash-1-3, key (0,0), over the 8 little-endian bytes of a u64 k-mer
//     (siphasher 1.0.2 SipHasher13, src/spiking_hash.rs:78-82);
//   * exact u64 `hash % pool` without a hardware 64-bit divide;
//   * the LIF update `v = v*leak + c` with two f32 roundings, never fused
//     (src/models.rs:34-51), solved in closed form per neuron.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace nk {

// Cost model measured on gfx950 (tools/isabench.hip): VOP2 xor/add and
// v_bitop3 issue at ~2.4 clk per wave64 instruction; v_alignbit, 64-bit ops
// (v_lshl_add_u64), carry adds and multiplies at ~4.2.  So a 64-bit add is one
// v_lshl_add_u64, a rotate is two v_alignbit on the 32-bit halves (a rotate by
// 32 is a free register swap), and xors stay 32-bit VOP2: 70 clk per SipRound.
// (Building the swapped v0/v2 pairs with one v_pk_mov_b32 instead of two
// v_mov_b32 is 4 % faster in isolation, tools/sipbench.hip V3, but made the
// count kernel 6 % slower in an A/B on one box, tools/ab_run.sh: not used.
// Likewise adding a swapped operand as v_mad_u64_u32(w.hi, 1, x) plus a 32-bit
// add on the high word, in inline asm, removes 12 of the 21 v_mov_b32 per
// k-mer but made K1a 7 % slower in an A/B: not used.)
__device__ __forceinline__ uint64_t rotl64(uint64_t x, int r) {
  const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  const uint32_t nlo = __builtin_amdgcn_alignbit(lo, hi, 32 - r);
  const uint32_t nhi = __builtin_amdgcn_alignbit(hi, lo, 32 - r);
  return ((uint64_t)nhi << 32) | nlo;
}
__device__ __forceinline__ uint64_t swap32(uint64_t x) { return (x << 32) | (x >> 32); }

#define NK_SIP_V2(x) (x)  // (the held form of v2 between rounds)
#define NK_SIPROUND                                                  \
  do {                                                               \
    v0 += v1; v1 = rotl64(v1, 13); v1 ^= v0; v0 = swap32(v0);        \
    v2 += v3; v3 = rotl64(v3, 16); v3 ^= v2;                         \
    v0 += v3; v3 = rotl64(v3, 21); v3 ^= v0;                         \
    v2 += v1; v1 = rotl64(v1, 17); v1 ^= v2; v2 = swap32(v2);        \
  } while (0)

// The last SipRound fused with the output v0 ^ v1 ^ v2 ^ v3.  In that round
// v3' = rotl(v3, 21) ^ v0' and the output xors v0' in again, so v0' (its swap,
// its add) cancels and is never computed; v2' ^ swap32(v2') has equal halves:
//   out = rotl(v1, 17) ^ v2' ^ swap32(v2') ^ rotl(v3, 21)   (v1, v3 mid-round)
// (tests/test_oracle.py::test_sip13_last_round_model).  The compiler already
// cancelled the output xors of the plain form; this drops the dead 64-bit add
// of v0' (1 of 18 v_lshl_add_u64 per hash).
__device__ __forceinline__ uint64_t sip_last_round_out(uint64_t v0, uint64_t v1, uint64_t v2,
                                                       uint64_t v3) {
  v0 += v1; v1 = rotl64(v1, 13); v1 ^= v0;
  v2 += v3; v3 = rotl64(v3, 16); v3 ^= v2;
  v3 = rotl64(v3, 21);
  v2 += v1; v1 = rotl64(v1, 17);
  const uint32_t x = (uint32_t)v2 ^ (uint32_t)(v2 >> 32);  // both halves of v2' ^ swap32(v2')
  const uint32_t lo = (uint32_t)v1 ^ (uint32_t)v3 ^ x;
  const uint32_t hi = (uint32_t)(v1 >> 32) ^ (uint32_t)(v3 >> 32) ^ x;
  return ((uint64_t)hi << 32) | lo;
}

// SipHash-1-3 with key (0,0) of one u64 written as 8 LE bytes:
// one compression round for the message block, one for the length block
// (b = 8 << 56), three finalization rounds.  Constants of the first round
// fold at compile time.
__device__ __forceinline__ uint64_t sip13_u64(uint64_t m) {
  uint64_t v0 = 0x736f6d6570736575ULL;
  uint64_t v1 = 0x646f72616e646f6dULL;
  uint64_t v2 = NK_SIP_V2(0x6c7967656e657261ULL);
  uint64_t v3 = 0x7465646279746573ULL ^ m;
  NK_SIPROUND;
  v0 ^= m;
  const uint64_t b = 8ULL << 56;
  v3 ^= b;
  NK_SIPROUND;
  v0 ^= b;
  v2 ^= NK_SIP_V2(0xffULL);
  NK_SIPROUND;
  NK_SIPROUND;
#if defined(NK_SIP_FULL_LAST)  // A/B only: the plain last round and output xor
  NK_SIPROUND;
  return v0 ^ v1 ^ v2 ^ v3;
#else
  return sip_last_round_out(v0, v1, NK_SIP_V2(v2), v3);
#endif
}

// --kmer-width=128: SipHash-1-3 (key 0) over the 16 LE bytes of a u128 key:
// two message blocks (lo, hi), then the length block (16 << 56), three
// finalization rounds (oracle/nk_oracle.c nko_sip13_u128).
__device__ __forceinline__ uint64_t sip13_u128(uint64_t lo, uint64_t hi) {
  uint64_t v0 = 0x736f6d6570736575ULL;
  uint64_t v1 = 0x646f72616e646f6dULL;
  uint64_t v2 = NK_SIP_V2(0x6c7967656e657261ULL);
  uint64_t v3 = 0x7465646279746573ULL ^ lo;
  NK_SIPROUND;
  v0 ^= lo;
  v3 ^= hi;
  NK_SIPROUND;
  v0 ^= hi;
  const uint64_t b = 16ULL << 56;
  v3 ^= b;
  NK_SIPROUND;
  v0 ^= b;
  v2 ^= NK_SIP_V2(0xffULL);
  NK_SIPROUND;
  NK_SIPROUND;
#if defined(NK_SIP_FULL_LAST)  // A/B only: the plain last round and output xor
  NK_SIPROUND;
  return v0 ^ v1 ^ v2 ^ v3;
#else
  return sip_last_round_out(v0, v1, NK_SIP_V2(v2), v3);
#endif
}

// Exact h % P for any P >= 1 given magic = floor((2^64-1)/P):
// q = mulhi(h, magic) is floor(h/P) - {0,1,2}, so at most two corrections.
struct FastMod {
  uint64_t p;
  uint64_t magic;
};

inline FastMod make_fastmod(uint64_t p) {
  FastMod f;
  f.p = p;
  f.magic = p ? (~0ULL) / p : 0;
  return f;
}

__device__ __forceinline__ uint64_t fastmod(uint64_t h, FastMod fm) {
  uint64_t q = __umul64hi(h, fm.magic);
  uint64_t r = h - q * fm.p;
  if (r >= fm.p) r -= fm.p;
  if (r >= fm.p) r -= fm.p;
  return r;
}

// Exact h % P for P < 2^30 in 32-bit arithmetic.  magic = floor((2^64-1)/P)
// satisfies 2^64/P - 1 <= magic <= 2^64/P, so q = mulhi64(h, magic) lies in
// (h/P - 1 - h/2^64, h/P], i.e. q = floor(h/P) - {0, 1}: r = h - q*P < 2P <
// 2^31 and ONE branch-free correction min(r, r - P) is exact.  Only the low
// word of q is needed (one mul_hi + two v_mad_u64_u32 + one mul_lo).  Model
// and edge cases: tests/test_oracle.py::test_fastmod32_model.
// (p: the modulus, possibly a VGPR copy of fm.p)
__device__ __forceinline__ uint32_t fastmod32_p(uint64_t h, FastMod fm, uint32_t p) {
  const uint32_t h0 = (uint32_t)h, h1 = (uint32_t)(h >> 32);
  const uint32_t m0 = (uint32_t)fm.magic, m1 = (uint32_t)(fm.magic >> 32);
  const uint32_t ahi = __umulhi(h0, m0);
  uint64_t mid = (uint64_t)h1 * m0 + ahi;
  mid = (uint64_t)h0 * m1 + mid;
  const uint32_t qlo = h1 * m1 + (uint32_t)(mid >> 32);
  const uint32_t r = h0 - qlo * p;
  return min(r, r - p);
}
__device__ __forceinline__ uint32_t fastmod32(uint64_t h, FastMod fm) {
  return fastmod32_p(h, fm, (uint32_t)fm.p);
}

// ---- LIF -------------------------------------------------------------------
// One LifNeuron::update with input c (src/models.rs:34-51); f32 ops rounded
// separately (__fmul_rn/__fadd_rn are never contracted into an FMA).
__device__ __forceinline__ float lif_step(float v, float leak, float c) {
  return __fadd_rn(__fmul_rn(v, leak), c);
}

// Exactly `steps` calls of LifNeuron::update starting from (v, r), with
// c = (count as f64 / steps as f64) as f32.  The map v -> v*leak + c is a
// function of v alone, so (a) a repeated value means every later step repeats
// it, and (b) after a spike the state is always (0, refractory): the rest is
// periodic with period refractory + m, m = steps from 0 to the next spike.
// Returns the spikes fired; updates v and r in place.  Cost O(m + tail).
__device__ __forceinline__ uint64_t lif_closed(float c, uint64_t steps, float thr, float leak,
                                               uint32_t refr, float &v, uint32_t &r) {
  uint64_t t = 0;
  uint64_t spikes = 0;
  // refractory drain
  {
    uint64_t d = (uint64_t)r < steps ? (uint64_t)r : steps;
    r -= (uint32_t)d;
    t += d;
  }
  // integrate from the current voltage
  bool fired = false;
  while (t < steps) {
    ++t;
    float nv = lif_step(v, leak, c);
    if (nv >= thr) {
      v = 0.0f;
      r = refr;
      spikes = 1;
      fired = true;
      break;
    }
    if (nv == v) {  // fixed point below threshold: nothing changes any more
      v = nv;
      t = steps;
      break;
    }
    v = nv;
  }
  if (!fired || t == steps) return spikes;
  uint64_t remaining = steps - t;  // state (0, refr)
  if (remaining <= (uint64_t)refr) {
    r = refr - (uint32_t)remaining;
    return spikes;
  }
  // m: integrate steps from 0 to the next spike, within the steps available
  uint64_t avail = remaining - refr;
  float x = 0.0f;
  uint64_t m = 0;
  bool fires = false;
  while (m < avail) {
    ++m;
    float nx = lif_step(x, leak, c);
    if (nx >= thr) { fires = true; break; }
    if (nx == x) { x = nx; break; }
    x = nx;
  }
  if (!fires) {  // never reaches threshold again: refractory then settle at x
    v = x;
    r = 0;
    return spikes;
  }
  uint64_t period = (uint64_t)refr + m;
  uint64_t n = remaining / period;
  spikes += n;
  uint64_t rem = remaining - n * period;  // < period, starts in state (0, refr)
  if (rem <= (uint64_t)refr) {
    v = 0.0f;
    r = refr - (uint32_t)rem;
    return spikes;
  }
  r = 0;
  float y = 0.0f;
  for (uint64_t s = 0; s < rem - refr; ++s) y = lif_step(y, leak, c);  // < m steps: no spike
  v = y;
  return spikes;
}

__device__ __forceinline__ float lif_current(uint64_t count, uint64_t steps) {
  // (total_current as f64 / steps as f64) as f32  — src/spiking_hash.rs:188,193,196
  double tot = (double)count;
  return (float)(tot / (double)steps);
}

}  // namespace nk
