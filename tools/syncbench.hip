// syncbench.hip — host-side latencies around a step on gfx950 / ROCm:
//   (a) gap an event marker puts between two kernels vs events attached to
//       the kernel launch itself (hipExtLaunchKernelGGL start/stop events);
//   (b) completion seen by spinning on a flag in mapped host memory vs
//       hipStreamSynchronize, and the cost of a sync after the flag is seen;
//   (c) host time of an 8-kernel launch sequence.
//   hipcc --offload-arch=gfx950 -O3 -o tools/bin/syncbench tools/syncbench.hip
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <algorithm>
#include <chrono>
#include <vector>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                            \
    }                                                                      \
  } while (0)

// ~`us` microseconds of one wave spinning per block, many blocks
__global__ void k_busy(uint64_t cycles, uint32_t *sink) {
  const uint64_t t0 = wall_clock64();
  uint32_t x = threadIdx.x;
  while (wall_clock64() - t0 < cycles) x = x * 1664525u + 1013904223u;
  if (x == 0x12345678u) sink[0] = x;
}

__global__ void k_flag(volatile uint64_t *flag, uint64_t seq) {
  if (threadIdx.x == 0) {
    __threadfence_system();
    __hip_atomic_store((uint64_t *)flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

// spin on the mapped flag, at most 2 s (then report and give up)
static bool spin(const uint64_t *f, uint64_t seq) {
  const double t0 = now_us();
  while (__atomic_load_n(f, __ATOMIC_ACQUIRE) != seq) {
    __builtin_ia32_pause();
    if (now_us() - t0 > 2e6) {
      fprintf(stderr, "flag %llu never arrived\n", (unsigned long long)seq);
      return false;
    }
  }
  return true;
}

int main() {
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  uint32_t *sink;
  CK(hipMalloc(&sink, 64));
  uint64_t *flag_h, *flag_d;
  CK(hipHostMalloc(&flag_h, 64, hipHostMallocMapped));
  CK(hipHostGetDevicePointer((void **)&flag_d, flag_h, 0));
  *flag_h = 0;
  // wall_clock64 runs at 100 MHz on gfx9
  const uint64_t c20 = 2000;  // 20 us
  hipEvent_t e[4], ef[4];
  for (auto &x : e) CK(hipEventCreate(&x));
  for (auto &x : ef) CK(hipEventCreateWithFlags(&x, hipEventDisableSystemFence));
  // warm
  for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(k_busy, dim3(1024), dim3(64), 0, s, c20, sink);
  CK(hipStreamSynchronize(s));

  const int R = 200;
  // (a) 3 kernels back to back; markers between them vs ext events vs none vs
  // markers from events without the system-scope fence
  for (int mode = 0; mode < 4; ++mode) {
    std::vector<float> v;
    for (int r = 0; r < R; ++r) {
      CK(hipEventRecord(e[0], s));
      hipLaunchKernelGGL(k_busy, dim3(1024), dim3(64), 0, s, c20, sink);
      if (mode == 0 || mode == 3) {
        CK(hipEventRecord(mode ? ef[2] : e[2], s));
        hipLaunchKernelGGL(k_busy, dim3(1024), dim3(64), 0, s, c20, sink);
        CK(hipEventRecord(mode ? ef[3] : e[3], s));
      } else if (mode == 1) {
        hipExtLaunchKernelGGL(k_busy, dim3(1024), dim3(64), 0, s, e[2], e[3], 0, c20, sink);
      } else {
        hipLaunchKernelGGL(k_busy, dim3(1024), dim3(64), 0, s, c20, sink);
      }
      hipLaunchKernelGGL(k_busy, dim3(1024), dim3(64), 0, s, c20, sink);
      CK(hipEventRecord(e[1], s));
      CK(hipStreamSynchronize(s));
      float ms = 0, mid = 0;
      CK(hipEventElapsedTime(&ms, e[0], e[1]));
      if (mode < 2) CK(hipEventElapsedTime(&mid, e[2], e[3]));
      if (mode == 3) CK(hipEventElapsedTime(&mid, ef[2], ef[3]));
      v.push_back(ms * 1000.f);
      if (r == R - 1)
        printf("(a) mode %s: 3x20us kernels (last mid-kernel event span %.1f us)\n",
               mode == 0 ? "markers" : mode == 1 ? "ext-events" : mode == 2 ? "none" : "markers-nofence",
               mid * 1000.f);
    }
    std::sort(v.begin(), v.end());
    printf("    median span %.1f us, p10 %.1f, p90 %.1f\n", v[R / 2], v[R / 10], v[R * 9 / 10]);
  }
  // (b) completion latency
  for (int mode = 0; mode < 3; ++mode) {
    std::vector<double> tl, tw, ts;
    for (int r = 0; r < R; ++r) {
      const uint64_t seq = 1000 + r + mode * 10000;
      const double t0 = now_us();
      hipLaunchKernelGGL(k_busy, dim3(1024), dim3(64), 0, s, c20, sink);
      hipLaunchKernelGGL(k_flag, dim3(1), dim3(64), 0, s, flag_d, seq);
      const double t1 = now_us();
      if (mode == 0) {
        CK(hipStreamSynchronize(s));
        tw.push_back(now_us() - t1);
      } else {
        if (!spin(flag_h, seq)) return 1;
        const double t2 = now_us();
        tw.push_back(t2 - t1);
        if (mode == 1) CK(hipStreamSynchronize(s));
        ts.push_back(now_us() - t2);
      }
      tl.push_back(t1 - t0);
      if (mode == 2) CK(hipStreamSynchronize(s));  // untimed
    }
    std::sort(tl.begin(), tl.end());
    std::sort(tw.begin(), tw.end());
    std::sort(ts.begin(), ts.end());
    printf("(b) mode %s: launch2 %.1f us, wait %.1f us (p90 %.1f), after-flag sync %.1f us\n",
           mode == 0 ? "stream-sync" : mode == 1 ? "spin+sync" : "spin", tl[R / 2], tw[R / 2],
           tw[R * 9 / 10], ts.empty() ? 0.0 : ts[R / 2]);
  }
  // (c) 8 launches + spin: whole round trip vs the 8 x 5 us of GPU work
  {
    std::vector<double> tt, tl;
    const uint64_t c5 = 500;
    for (int r = 0; r < R; ++r) {
      const uint64_t seq = 50000 + r;
      const double t0 = now_us();
      for (int j = 0; j < 7; ++j) hipLaunchKernelGGL(k_busy, dim3(1024), dim3(64), 0, s, c5, sink);
      hipLaunchKernelGGL(k_flag, dim3(1), dim3(64), 0, s, flag_d, seq);
      tl.push_back(now_us() - t0);
      if (!spin(flag_h, seq)) return 1;
      tt.push_back(now_us() - t0);
    }
    CK(hipStreamSynchronize(s));
    std::sort(tt.begin(), tt.end());
    std::sort(tl.begin(), tl.end());
    printf("(c) 7x5us + flag: launches %.1f us, round trip %.1f us (p90 %.1f)\n", tl[R / 2],
           tt[R / 2], tt[R * 9 / 10]);
  }
  return 0;
}
