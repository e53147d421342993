// nk_post.h — the top-N post step shared by the selection kernels
// (nk_kernels.hip: k_top_post, the fused final step) and the pool-sliced
// adopt (nk_slice.hip): set sizing and bucket bookkeeping for the uniques pass.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "nk_kernels.h"

namespace nk {

// Set sizing and bookkeeping for the uniques pass from the final top rows
// (one block of 1024 threads).
__device__ __forceinline__ void top_post_block(const TopCand *top, const uint64_t *top_cur, uint32_t m,
                               const PostArgs &pa) {
  __shared__ unsigned long long s_sum;
  __shared__ uint32_t s_nb, s_over;
  __shared__ uint32_t s_bk[kMaxTopN];
  if (threadIdx.x == 0) { s_sum = 0; s_nb = 0; s_over = 0; *pa.n_hits = 0; }
  // a sentinel row (index ~0: a selection deferred to the host's exact redo,
  // k_slice_adopt) takes no part: no bucket, no set capacity, no hits
  constexpr uint32_t kNoBucket = 0xFFFFFFFFu;
  for (uint32_t i = threadIdx.x; i < m; i += blockDim.x)
    s_bk[i] = top[i].idx == ~0ull ? kNoBucket : (uint32_t)(top[i].idx >> pa.bin_bits);
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < m; i += blockDim.x) {
    pa.uniq[i] = 0;
    pa.special[i] = 0;
    const uint32_t b = s_bk[i];
    if (b == kNoBucket) continue;
    atomicAdd(&s_sum, (unsigned long long)top_cur[i]);
    if (pa.part) {
      if (pa.n_over && b >= pa.n_over) {  // a row outside the count's buckets: never indexed
#ifdef NK_DEBUG_ROWS
        printf("[nk top_post] row %u index %llu outside the count's %u buckets\n", i,
               (unsigned long long)top[i].idx, pa.n_over);
#endif
        s_over = 1;                          // (the host takes the rescan path)
        continue;
      }
      if (pa.overflow[b]) s_over = 1;
      bool first = true;  // first row of its bucket in the list
      for (uint32_t j = 0; j < i; ++j)
        if (s_bk[j] == b) { first = false; break; }
      if (first) pa.tbuckets[atomicAdd(&s_nb, 1u)] = b;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t cap = 64;
    while (cap < 2 * (uint64_t)s_sum + 2 && cap < (1ull << 48)) cap <<= 1;  // (bounded: a row's
    // current read before its selection was resolved must not spin the loop)
    pa.flags[0] = cap > pa.set_alloc ? 1u : 0u;  // set too small
    pa.flags[1] = s_over;                        // a top bucket overflowed
    pa.flags[2] = s_nb;                          // distinct top buckets
    pa.flags[3] = 0;
    *pa.set_mask = (cap > pa.set_alloc ? pa.set_alloc : cap) - 1;
  }
}

}  // namespace nk
