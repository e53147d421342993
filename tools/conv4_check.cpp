// conv4_check.cpp — exhaustive host check (all 2^32 input words) that the
// multiply/permute form of the base conversion (nk_tile.h conv4p) gives the
// same forward codes, complement codes and invalid-byte bits as the
// byte-compare form it replaced (conv4_ref below, the previous nk_tile.h).
//   g++ -O2 -fopenmp -o tools/bin/conv4_check tools/conv4_check.cpp
#include <stdint.h>
#include <stdio.h>

static uint32_t eq_bytes(uint32_t t, uint32_t c) {
  uint32_t z = t ^ c;
  return ~(((z & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | z) & 0x80808080u;
}
struct C4 { uint32_t f, r, i; };
static C4 conv4_ref(uint32_t x) {
  uint32_t t = x | 0x20202020u;
  uint32_t valid = eq_bytes(t, 0x61616161u) | eq_bytes(t, 0x63636363u) |
                   eq_bytes(t, 0x67676767u) | eq_bytes(t, 0x74747474u);
  uint32_t vm = valid >> 7, vm3 = vm * 3u;
  uint32_t code = ((x >> 1) ^ (x >> 2)) & 0x03030303u & vm3;
  uint32_t comp = (code ^ 0x03030303u) & vm3;
  C4 o;
  o.f = ((code << 6) & 0xC0u) | ((code >> 4) & 0x30u) | ((code >> 14) & 0x0Cu) | ((code >> 24) & 0x03u);
  o.r = (comp & 0x03u) | ((comp >> 6) & 0x0Cu) | ((comp >> 12) & 0x30u) | ((comp >> 18) & 0xC0u);
  uint32_t m = ~vm & 0x01010101u;
  o.i = (m & 1u) | ((m >> 7) & 2u) | ((m >> 14) & 4u) | ((m >> 21) & 8u);
  return o;
}
// v_perm_b32 for selectors 0..7 and 0x0C (the only ones used): bytes 0-3 of
// {S0, S1} are S1's, 4-7 S0's, 0x0C gives 0x00
static uint32_t perm(uint32_t s0, uint32_t s1, uint32_t sel) {
  uint64_t v = ((uint64_t)s0 << 32) | s1;
  uint32_t d = 0;
  for (int b = 0; b < 4; ++b) {
    uint32_t s = (sel >> (8 * b)) & 0xFF;
    uint32_t byte = s < 8 ? (uint32_t)(v >> (8 * s)) & 0xFF : 0;
    d |= byte << (8 * b);
  }
  return d;
}
// mirror of nk_tile.h conv4p
static C4 conv4_new(uint32_t x) {
  const uint32_t code = ((x >> 1) ^ (x >> 2)) & 0x03030303u;
  const uint32_t expect = perm(0u, 0x74676361u, code);
  const uint32_t z = (x | 0x20202020u) ^ expect;
  const uint32_t valid = ~(((z & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | z) & 0x80808080u;
  const uint32_t vm3 = (valid >> 6) | (valid >> 7);
  const uint32_t pf = (code & vm3) * 0x40100401u;
  const uint32_t pr = (~code & vm3) * 0x01041040u;
  const uint32_t pi = ((~valid >> 7) & 0x01010101u) * 0x10204080u;
  return C4{pf >> 24, pr >> 24, pi >> 28};
}

int main() {
  unsigned long long bad = 0;
#pragma omp parallel for reduction(+ : bad) schedule(static)
  for (long long hi = 0; hi < 65536; ++hi)
    for (uint32_t lo = 0; lo < 65536; ++lo) {
      const uint32_t x = ((uint32_t)hi << 16) | lo;
      const C4 a = conv4_ref(x), b = conv4_new(x);
      bad += (a.f != b.f) | (a.r != b.r) | (a.i != b.i);
    }
  // the combine: F from byte 3 of the four products, R likewise, LSB-first
  unsigned long long bad2 = 0;
  uint32_t s = 12345;
  for (int n = 0; n < 1000000; ++n) {
    uint32_t w[4], pf[4], pr[4];
    for (int j = 0; j < 4; ++j) {
      s = s * 1664525u + 1013904223u;
      w[j] = s;
      C4 c = conv4_ref(w[j]);
      pf[j] = (c.f << 24) | (s & 0xFFFFFF);  // byte 3 = nibble, garbage below
      pr[j] = (c.r << 24) | ((s >> 3) & 0xFFFFFF);
    }
    C4 a = conv4_ref(w[0]), b = conv4_ref(w[1]), c = conv4_ref(w[2]), d = conv4_ref(w[3]);
    const uint32_t F = (a.f << 24) | (b.f << 16) | (c.f << 8) | d.f;
    const uint32_t R = a.r | (b.r << 8) | (c.r << 16) | (d.r << 24);
    const uint32_t F2 = perm(pf[0], pf[1], 0x07030C0Cu) | perm(pf[2], pf[3], 0x0C0C0703u);
    const uint32_t R2 = perm(pr[1], pr[0], 0x0C0C0703u) | perm(pr[3], pr[2], 0x07030C0Cu);
    bad2 += (F != F2) | (R != R2);
  }
  printf("conv4 words checked: 4294967296, mismatches %llu; combine mismatches %llu\n", bad, bad2);
  return (bad || bad2) ? 1 : 0;
}
