// hashbench.hip — micro-benchmark of the per-k-mer arithmetic on gfx950:
// SipHash-1-3 (key 0) of a u64 + exact % pool, in several formulations.
// Each variant hashes N keys (generated in-register from the thread index),
// folds results with XOR and writes one word per thread, so the timing is
// pure VALU.  Also checks every variant against the reference formulation.
//   hipcc --offload-arch=gfx950 -O3 -o hashbench tools/hashbench.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "../neurokmer_amd/csrc/nk_device.h"

using namespace nk;

struct H2 {
  uint32_t lo, hi;
};
__device__ __forceinline__ H2 add2(H2 a, H2 b) {
  H2 r;
  r.lo = a.lo + b.lo;
  r.hi = a.hi + b.hi + (r.lo < a.lo);
  return r;
}
__device__ __forceinline__ H2 xor2(H2 a, H2 b) { return H2{a.lo ^ b.lo, a.hi ^ b.hi}; }
template <int R>
__device__ __forceinline__ H2 rotl2(H2 x) {
  if (R == 32) return H2{x.hi, x.lo};
  return H2{__builtin_amdgcn_alignbit(x.lo, x.hi, 32 - R), __builtin_amdgcn_alignbit(x.hi, x.lo, 32 - R)};
}
#define SR2                                                                 \
  do {                                                                      \
    v0 = add2(v0, v1); v1 = rotl2<13>(v1); v1 = xor2(v1, v0); v0 = rotl2<32>(v0); \
    v2 = add2(v2, v3); v3 = rotl2<16>(v3); v3 = xor2(v3, v2);               \
    v0 = add2(v0, v3); v3 = rotl2<21>(v3); v3 = xor2(v3, v0);               \
    v2 = add2(v2, v1); v1 = rotl2<17>(v1); v1 = xor2(v1, v2); v2 = rotl2<32>(v2); \
  } while (0)

__device__ __forceinline__ uint64_t sip13_32(uint64_t m) {
  H2 mm{(uint32_t)m, (uint32_t)(m >> 32)};
  H2 v0{0x70736575u, 0x736f6d65u}, v1{0x6e646f6du, 0x646f7261u}, v2{0x6e657261u, 0x6c796765u},
      v3{0x79746573u ^ mm.lo, 0x74656462u ^ mm.hi};
  SR2;
  v0 = xor2(v0, mm);
  v3.hi ^= 0x08000000u;
  SR2;
  v0.hi ^= 0x08000000u;
  v2.lo ^= 0xffu;
  SR2;
  SR2;
  SR2;
  H2 r = xor2(xor2(v0, v1), xor2(v2, v3));
  return ((uint64_t)r.hi << 32) | r.lo;
}

__device__ __forceinline__ uint64_t rotl_ab(uint64_t x, int r) {
  uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  uint32_t nlo = __builtin_amdgcn_alignbit(lo, hi, 32 - r);
  uint32_t nhi = __builtin_amdgcn_alignbit(hi, lo, 32 - r);
  return ((uint64_t)nhi << 32) | nlo;
}
__device__ __forceinline__ uint64_t swap32(uint64_t x) { return (x << 32) | (x >> 32); }
#define SR3                                                                  \
  do {                                                                       \
    v0 += v1; v1 = rotl_ab(v1, 13); v1 ^= v0; v0 = swap32(v0);               \
    v2 += v3; v3 = rotl_ab(v3, 16); v3 ^= v2;                                \
    v0 += v3; v3 = rotl_ab(v3, 21); v3 ^= v0;                                \
    v2 += v1; v1 = rotl_ab(v1, 17); v1 ^= v2; v2 = swap32(v2);               \
  } while (0)
__device__ __forceinline__ uint64_t sip13_hy(uint64_t m) {
  uint64_t v0 = 0x736f6d6570736575ULL, v1 = 0x646f72616e646f6dULL, v2 = 0x6c7967656e657261ULL,
           v3 = 0x7465646279746573ULL ^ m;
  SR3;
  v0 ^= m;
  v3 ^= 8ULL << 56;
  SR3;
  v0 ^= 8ULL << 56;
  v2 ^= 0xffULL;
  SR3; SR3; SR3;
  return v0 ^ v1 ^ v2 ^ v3;
}

// exact h % p for p < 2^32 with f64: two 32-bit-sized reductions
__device__ __forceinline__ uint32_t mod_f64(uint64_t h, uint32_t p, double invp, uint32_t t32) {
  uint32_t H = (uint32_t)(h >> 32), L = (uint32_t)h;
  double Hd = (double)H;
  double q = floor(Hd * invp);
  double r1 = fma(-q, (double)p, Hd);  // exact
  if (r1 < 0) r1 += p;
  if (r1 >= p) r1 -= p;
  double y = fma(r1, (double)t32, (double)L);  // < 2^55? r1<p, t32<p: y < p^2+2^32
  double q2 = floor(y * invp);
  double r = fma(-q2, (double)p, y);
  if (r < 0) r += p;
  if (r >= p) r -= p;
  return (uint32_t)r;
}

template <int V>
__global__ __launch_bounds__(256) void kbench(uint64_t n_per, FastMod fm, double invp, uint32_t t32,
                                              uint64_t *out) {
  uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t acc = 0;
  uint64_t key = tid * 0x9E3779B97F4A7C15ULL;
  for (uint64_t i = 0; i < n_per; ++i) {
    key += 0x632BE59BD9B4E019ULL;
    uint64_t h;
    if (V == 0 || V == 2) h = sip13_u64(key);
    else if (V == 4 || V == 5) h = sip13_hy(key);
    else h = sip13_32(key);
    uint64_t idx;
    if (V == 0 || V == 1 || V == 4) idx = fastmod(h, fm);
    else idx = mod_f64(h, (uint32_t)fm.p, invp, t32);
    acc ^= idx + i;
  }
  out[tid] = acc;
}

template <int V>
__global__ void kcheck(uint64_t n, FastMod fm, double invp, uint32_t t32, uint32_t *bad) {
  uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (tid >= n) return;
  uint64_t key = tid * 0xD1B54A32D192ED03ULL ^ (tid >> 7);
  uint64_t ref = fastmod(sip13_u64(key), fm);
  uint64_t h = (V == 0 || V == 2) ? sip13_u64(key) : (V >= 4 ? sip13_hy(key) : sip13_32(key));
  uint64_t idx = (V == 0 || V == 1 || V == 4) ? fastmod(h, fm) : mod_f64(h, (uint32_t)fm.p, invp, t32);
  if (idx != ref) atomicAdd(bad, 1u);
}

int main(int argc, char **argv) {
  uint64_t pool = argc > 1 ? strtoull(argv[1], 0, 10) : 2000000;
  FastMod fm{pool, ~0ULL / pool};
  double invp = 1.0 / (double)pool;
  uint32_t t32 = (uint32_t)((1ULL << 32) % pool);
  const int blocks = 256 * 32, threads = 256;
  const uint64_t n_per = 64;
  uint64_t *out;
  uint32_t *bad;
  hipMalloc(&out, (size_t)blocks * threads * 8);
  hipMalloc(&bad, 4);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const char *names[] = {"sip64+magicmod", "sip32alignbit+magicmod", "sip64+f64mod",
                         "sip32alignbit+f64mod", "hybrid+magicmod", "hybrid+f64mod"};
  for (int v = 0; v < 6; ++v) {
    hipMemset(bad, 0, 4);
    uint64_t nchk = 1 << 24;
#define CHK(V) hipLaunchKernelGGL(kcheck<V>, dim3(nchk / 256), dim3(256), 0, 0, nchk, fm, invp, t32, bad)
    if (v == 0) CHK(0); else if (v == 1) CHK(1); else if (v == 2) CHK(2); else if (v == 3) CHK(3); else if (v == 4) CHK(4); else CHK(5);
    uint32_t hb = 0;
    hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost);
    float best = 1e9;
    for (int rep = 0; rep < 5; ++rep) {
      hipEventRecord(a);
#define RUN(V) hipLaunchKernelGGL(kbench<V>, dim3(blocks), dim3(threads), 0, 0, n_per, fm, invp, t32, out)
      if (v == 0) RUN(0); else if (v == 1) RUN(1); else if (v == 2) RUN(2); else if (v == 3) RUN(3); else if (v == 4) RUN(4); else RUN(5);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      if (ms < best) best = ms;
    }
    double nh = (double)blocks * threads * n_per;
    printf("%-26s %8.3f ms  %8.1f G hash/s  mismatches=%u\n", names[v], best, nh / best / 1e6, hb);
  }
  return 0;
}
