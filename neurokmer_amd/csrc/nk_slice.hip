// nk_slice.hip — the device side of the pool-sliced multi-GPU finish without
// host round trips (nk_slice_export / nk_adopt_export, include/neurokmer.h).
//
// After the reduce-scatter each rank holds the summed currents of its S
// neurons; the LIF and the top rows of that slice run on the device and
// k_slice_seg writes the slice's rows into the all-gather segment.  After the
// all-gather k_slice_adopt picks the global rows on the device (a global top
// row is always among its own slice's top rows), sums the new spikes and the
// largest spike count, and the uniques pass + the key export of the plain
// finish follow (nk_finalize_export's tail).  The reference ranks the rows by
// a stable sort on spikes, ties by index (src/spiking_hash.rs:661-673).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "nk_kernels.h"
#include "nk_post.h"

namespace nk {

namespace {

constexpr uint64_t kSegCount = kSegRefine - 1;  // (kSegRefine: nk_kernels.h)

// seg = [rows | refine << 56, new spikes, largest spike count, (global idx, spikes, current) x rows]
// A slice whose selection is not resolved on the device (spike counts past
// 4095: the exact refine; or a row the passes left unfilled, index >= n)
// exports NO rows, only the refine flag: nothing downstream may rank, adopt or
// look up rows read from buffers the selection did not finish (the r04 device
// fault: such rows reached the uniques bookkeeping); the redo
// selects exactly and rebuilds the segment.
__global__ void k_slice_seg(const TopCand *__restrict__ cand, const uint64_t *__restrict__ top_cur,
                            const TopState *__restrict__ st, const uint64_t *__restrict__ stats,
                            uint32_t m, uint64_t lo, uint64_t n, uint64_t *__restrict__ seg) {
  int bad = 0;
  for (uint32_t i = threadIdx.x; i < m; i += blockDim.x) bad |= cand[i].idx >= n ? 1 : 0;
  const bool refine = __syncthreads_or(bad) || (m && st->refine);
  const uint32_t rows = refine ? 0u : m;
  for (uint32_t i = threadIdx.x; i < rows; i += blockDim.x) {
    seg[3 + 3 * (uint64_t)i] = cand[i].idx + lo;
    seg[4 + 3 * (uint64_t)i] = cand[i].sc;
    seg[5 + 3 * (uint64_t)i] = top_cur[i];
  }
  if (threadIdx.x == 0) {
    seg[0] = (uint64_t)rows | (refine ? kSegRefine : 0ull);
    seg[1] = stats[0];
    seg[2] = stats[1];
  }
}

// One block: the global top `want` rows of the W slice segments.  A row's
// rank is the number of rows that precede it (more spikes, or as many and a
// lower index); n <= kAdoptMax rows, each thread ranks its rows against all.
constexpr int kAdoptBlock = 1024;
__global__ __launch_bounds__(kAdoptBlock) void k_slice_adopt(const uint64_t *__restrict__ all,
                                                             uint32_t W, uint64_t stride,
                                                             uint32_t want, uint64_t pool,
                                                             TopCand *__restrict__ cand,
                                                             uint64_t *__restrict__ top_cur,
                                                             TopState *__restrict__ st,
                                                             uint64_t *__restrict__ stats,
                                                             PostArgs post, int do_post) {
  __shared__ uint64_t s_idx[kAdoptMax], s_sc[kAdoptMax], s_cur[kAdoptMax];
  __shared__ uint32_t s_n;
  __shared__ unsigned long long s_new, s_max;
  __shared__ uint32_t s_ref;
  if (threadIdx.x == 0) {
    s_n = 0;
    s_new = 0;
    s_max = 0;
    s_ref = 0;
  }
  __syncthreads();
  // gather the rows (segment r's rows at a running offset)
  for (uint32_t r = threadIdx.x; r < W; r += blockDim.x) {
    const uint64_t *g = all + (uint64_t)r * stride;
    atomicAdd(&s_new, (unsigned long long)g[1]);
    atomicMax(&s_max, (unsigned long long)g[2]);
    if (g[0] & kSegRefine) atomicOr(&s_ref, 1u);
  }
  __syncthreads();
  // a segment's row count, bounded by its stride and the LDS rows (a corrupt
  // header must not drive the loops below past either)
  const uint64_t seg_max = stride >= 3 ? (stride - 3) / 3 : 0;
  auto rows_of = [&](const uint64_t *g) -> uint32_t {
    const uint64_t nr = g[0] & kSegCount;
    return (uint32_t)(nr < seg_max ? nr : seg_max);
  };
  if (threadIdx.x == 0) {
    uint32_t n = 0;
    for (uint32_t r = 0; r < W; ++r) n += rows_of(all + (uint64_t)r * stride);
    s_n = n < (uint32_t)kAdoptMax ? n : (uint32_t)kAdoptMax;
  }
  __syncthreads();
  // rows in segment order: prefix over segments (W is small), one row per thread
  uint32_t base = 0;
  for (uint32_t r = 0; r < W; ++r) {
    const uint64_t *g = all + (uint64_t)r * stride;
    uint32_t nr = rows_of(g);
    if (base + nr > (uint32_t)kAdoptMax) nr = base < (uint32_t)kAdoptMax ? (uint32_t)kAdoptMax - base : 0u;
    for (uint32_t i = threadIdx.x; i < nr; i += blockDim.x) {
      s_idx[base + i] = g[3 + 3 * (uint64_t)i];
      s_sc[base + i] = g[4 + 3 * (uint64_t)i];
      s_cur[base + i] = g[5 + 3 * (uint64_t)i];
    }
    base += nr;
  }
  __syncthreads();
  const uint32_t n = s_n;
  // a row outside the pool (a corrupt segment) is a redo too
  for (uint32_t i = threadIdx.x; i < n; i += blockDim.x)
    if (s_idx[i] >= pool) atomicOr(&s_ref, 1u);
  __syncthreads();
  if (s_ref) {  // (block-uniform) a redo: sentinel rows, so the uniques pass idles
    for (uint32_t i = threadIdx.x; i < want; i += blockDim.x) {
      cand[i] = TopCand{~0ull, 0ull};
      top_cur[i] = 0;
    }
  } else {
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
      const uint64_t sc = s_sc[i], idx = s_idx[i];
      uint32_t rank = 0;
      for (uint32_t j = 0; j < n; ++j)
        rank += (s_sc[j] > sc || (s_sc[j] == sc && s_idx[j] < idx)) ? 1u : 0u;
      if (rank < want) {
        cand[rank] = TopCand{idx, sc};
        top_cur[rank] = s_cur[i];
      }
    }
  }
  if (threadIdx.x == 0) {
    TopState z{};
    z.refine = s_ref;  // a slice needs the exact refine: the export header flags a redo
    *st = z;
    stats[0] = s_new;
    stats[1] = s_max;
  }
  if (do_post) {  // the top-N post step of the adopted rows (k_top_post's work)
    __syncthreads();  // (global cand / top_cur of this block: written above)
    __threadfence_block();
    top_post_block(cand, top_cur, want, post);
  }
}

}  // namespace

hipError_t launch_slice_seg(const TopCand *cand, const uint64_t *top_cur, const TopState *st,
                            const uint64_t *stats, uint32_t m, uint64_t lo, uint64_t n, uint64_t *seg,
                            hipStream_t s) {
  hipLaunchKernelGGL(k_slice_seg, dim3(1), dim3(256), 0, s, cand, top_cur, st, stats, m, lo, n, seg);
  return hipGetLastError();
}

hipError_t launch_slice_adopt(const uint64_t *all, uint32_t world, uint64_t stride, uint32_t want,
                              uint64_t pool, TopCand *cand, uint64_t *top_cur, TopState *st,
                              uint64_t *stats, hipStream_t s, const PostArgs *post) {
  if ((uint64_t)world * want > (uint64_t)kAdoptMax) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_slice_adopt, dim3(1), dim3(kAdoptBlock), 0, s, all, world, stride, want, pool,
                     cand, top_cur, st, stats, post ? *post : PostArgs{}, post ? 1 : 0);
  return hipGetLastError();
}

}  // namespace nk
