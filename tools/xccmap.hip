// xccmap.hip -- which XCD (HW_REG_XCC_ID) each workgroup of a launch runs on:
// the K1a sub-regions (PartArgs::sub_shift) assume tile & 7 or read the id.
//   hipcc --offload-arch=gfx950 -O2 tools/xccmap.hip -o tools/bin/xccmap
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ void k_xcc(unsigned *o, int spin) {
  if (threadIdx.x == 0) {
    long long t0 = clock64();
    while (clock64() - t0 < spin) {
    }
    o[blockIdx.x] = __builtin_amdgcn_s_getreg((20) | (0 << 6) | (3 << 11));
  }
}

int main() {
  const int n = 4096;
  unsigned *d, h[n];
  if (hipMalloc(&d, n * sizeof(unsigned)) != hipSuccess) return 1;
  for (int spin : {0, 20000}) {
    hipLaunchKernelGGL(k_xcc, dim3(n), dim3(256), 0, 0, d, spin);
    if (hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost) != hipSuccess) return 1;
    int same = 0;
    for (int i = 0; i < n; ++i) same += h[i] == (unsigned)(i & 7);
    printf("spin %d: blocks with xcc == blockIdx & 7: %d of %d; first 24:", spin, same, n);
    for (int i = 0; i < 24; ++i) printf(" %u", h[i]);
    printf("\n");
  }
  hipFree(d);
  return 0;
}
