// ldsbench.hip — LDS atomic throughput on gfx950 for the histogram patterns
// the count path uses (K1b: ds_add_u32 into 32768 bins; K1a: ds_add_rtn_u32
// into ~64 bucket counters).  Reports lane-atomics per CU per shader clock.
//   hipcc --offload-arch=gfx950 -O3 -o tools/bin/ldsbench tools/ldsbench.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define ITERS 2048

__device__ __forceinline__ uint32_t xs(uint32_t x) {
  x ^= x << 13;
  x ^= x >> 17;
  x ^= x << 5;
  return x;
}

// MODE 0: random bin of NB; 1: conflict-free (lane + 64*r); 2: return-value
// atomics on NB bins; 3: all lanes same address; 4: ds_read random (no atomic)
template <int MODE, int NB, int BLOCK>
__global__ __launch_bounds__(BLOCK) void kl(uint32_t *out, uint64_t *clk) {
  extern __shared__ uint32_t h[];
  for (int i = threadIdx.x; i < NB; i += BLOCK) h[i] = 0;
  __syncthreads();
  uint32_t x = (blockIdx.x * BLOCK + threadIdx.x) * 2654435761u + 1;
  uint32_t acc = 0;
  const uint32_t lane = threadIdx.x & 63;
  uint32_t base[8];  // per-lane random addresses; each iteration adds a wave-uniform offset
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    x = xs(x);
    base[j] = MODE == 1 ? lane + 64 * (x >> 8) : MODE == 3 ? 5u : x;
  }
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < ITERS / 8; ++i) {
    const uint32_t off = MODE == 3 ? 0u : (uint32_t)i * 0x9E40u;  // multiple of 64: keeps banks
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint32_t a = (base[j] + off) & (NB - 1);
      if (MODE == 2) acc += atomicAdd(&h[a], 1u);
      else if (MODE == 4) acc += h[a];
      else atomicAdd(&h[a], 1u);
    }
  }
  __syncthreads();
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * BLOCK + threadIdx.x] = acc + h[threadIdx.x & (NB - 1)];
  if (threadIdx.x == 0 && blockIdx.x == 0) clk[0] = t1 - t0;
}

template <int MODE, int NB, int BLOCK>
static void run(const char *name, int per_cu, uint32_t *out, uint64_t *clk) {
  const int blocks = 256 * per_cu;
  const size_t lds = (size_t)NB * 4;
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  (void)hipFuncSetAttribute((const void *)kl<MODE, NB, BLOCK>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  float best = 1e9;
  for (int rep = 0; rep < 3; ++rep) {
    (void)hipEventRecord(a);
    hipLaunchKernelGGL((kl<MODE, NB, BLOCK>), dim3(blocks), dim3(BLOCK), lds, 0, out, clk);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    if (ms < best) best = ms;
  }
  uint64_t hc = 0;
  (void)hipMemcpy(&hc, clk, 8, hipMemcpyDeviceToHost);
  const double ops = (double)blocks * BLOCK * ITERS;
  const double per_cu_s = ops / 256.0 / (best * 1e-3);
  printf("%-40s %8.3f ms  %.2f G lane-ops/s/CU  %.2f per clk @2.4GHz\n", name, best,
         per_cu_s / 1e9, per_cu_s / 2.4e9);
}

int main() {
  uint32_t *out;
  uint64_t *clk;
  (void)hipMalloc(&out, 256 * 4 * 1024 * 4);
  (void)hipMalloc(&clk, 8);
  run<0, 32768, 1024>("add random 32K bins, 1x1024 thr/CU", 1, out, clk);
  run<0, 16384, 512>("add random 16K bins, 2x512 thr/CU", 2, out, clk);
  run<0, 16384, 1024>("add random 16K bins, 2x1024 thr/CU", 2, out, clk);
  run<0, 32768, 512>("add random 32K bins, 1x512 thr/CU", 1, out, clk);
  run<1, 32768, 1024>("add conflict-free 32K bins", 1, out, clk);
  run<4, 32768, 1024>("read random 32K bins", 1, out, clk);
  run<2, 32768, 1024>("add_rtn random 32K bins", 1, out, clk);
  run<0, 64, 512>("add random 64 bins, 3x512", 3, out, clk);
  run<2, 64, 512>("add_rtn random 64 bins, 3x512", 3, out, clk);
  run<2, 256, 512>("add_rtn random 256 bins, 3x512", 3, out, clk);
  run<3, 64, 512>("add same address, 3x512", 3, out, clk);
  return 0;
}
