// LDS out-of-range behaviour on gfx950 (round 6): is a ds_add_u32 at an
// address past the workgroup's LDS allocation (or wrapped below 0) dropped,
// and what does it cost?  Used to decide the fused count's K1b item form.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <vector>
constexpr int kWords = 12900;  // 51.6 KB allocation
constexpr int kRange = 10923;  // histogram words per pass
__global__ __launch_bounds__(512) void k_oob(const uint32_t *recs, int n, int passes, uint32_t *out,
                                             unsigned long long *cyc) {
  __shared__ uint32_t h[kWords];
  for (int i = threadIdx.x; i < kWords; i += 512) h[i] = 0;
  __syncthreads();
  const unsigned long long t0 = clock64();
  for (int p = 0; p < passes; ++p) {
    for (int i = threadIdx.x; i < n; i += 512) {
      const uint32_t off = recs[i];
      const uint32_t a = (off - (uint32_t)(p * kRange)) * 4u;  // byte address, wraps below 0
      atomicAdd(reinterpret_cast<uint32_t *>(reinterpret_cast<char *>(h) + a), 1u);
    }
  }
  __syncthreads();
  const unsigned long long t1 = clock64();
  for (int i = threadIdx.x; i < kWords; i += 512) out[blockIdx.x * kWords + i] = h[i];
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
int main() {
  const int n = 1 << 20;
  std::vector<uint32_t> r(n);
  uint64_t z = 12345;
  for (int i = 0; i < n; ++i) { z = z * 6364136223846793005ull + 1442695040888963407ull; r[i] = (uint32_t)(z >> 49); }  // 15-bit
  uint32_t *dr, *dout; unsigned long long *dc;
  hipMalloc(&dr, n * 4); hipMalloc(&dout, 256 * kWords * 4); hipMalloc(&dc, 256 * 8);
  hipMemcpy(dr, r.data(), n * 4, hipMemcpyHostToDevice);
  for (int passes = 1; passes <= 3; ++passes) {
    hipLaunchKernelGGL(k_oob, dim3(1), dim3(512), 0, 0, dr, n, passes, dout, dc);
    hipDeviceSynchronize();
    std::vector<uint32_t> h(kWords); unsigned long long c;
    hipMemcpy(h.data(), dout, kWords * 4, hipMemcpyDeviceToHost);
    hipMemcpy(&c, dc, 8, hipMemcpyDeviceToHost);
    // expected: pass p adds record off to word off - p*kRange when that is in [0, kWords)
    std::vector<uint32_t> e(kWords, 0);
    for (int p = 0; p < passes; ++p)
      for (int i = 0; i < n; ++i) { int64_t w = (int64_t)r[i] - (int64_t)p * kRange; if (w >= 0 && w < kWords) e[w]++; }
    int bad = 0; for (int i = 0; i < kWords; ++i) bad += h[i] != e[i];
    printf("passes %d: mismatching words %d, cycles %llu (%.2f clk per record-pass)\n", passes, bad, c,
           (double)c / ((double)n * passes));
  }
  // the in-range-only reference rate: every address in range
  for (int i = 0; i < n; ++i) r[i] %= kRange;
  hipMemcpy(dr, r.data(), n * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k_oob, dim3(1), dim3(512), 0, 0, dr, n, 1, dout, dc);
  hipDeviceSynchronize(); unsigned long long c; hipMemcpy(&c, dc, 8, hipMemcpyDeviceToHost);
  printf("in range only: cycles %llu (%.2f clk per record)\n", c, (double)c / n);
  hipError_t e = hipGetLastError();
  printf("last error: %s\n", hipGetErrorString(e));
  return 0;
}
