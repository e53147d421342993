// nk_loop.hip — the loopback transport of nk_comm: W ranks as W host threads
// of ONE process on one GPU, their collectives carried out by device copies and
// a sum kernel between host barriers (include/neurokmer.h nk_loop_group_new,
// nk_comm_new_loopback).
//
// RCCL refuses two ranks on one device ("Duplicate GPU detected"), so on a
// one-GPU box the library's multi-rank finish (nk_finalize_dist /
// nk_finalize_sliced_dist: the merge-set emptying keyed on the world size, the
// top k-mer union exchange and its redo, the slice padding of the
// reduce-scatter) could only ever run at world 1, where every collective is the
// identity.  Through this transport the same library code runs at world 2..16
// with real exchanges, so tests can compare the N-rank result with one handle
// counting the union.  It is a rehearsal transport: every collective waits for
// its stream, then for every rank (host barrier), so it overlaps nothing.
#include <hip/hip_runtime.h>
#include <stdio.h>

#include <chrono>
#include <condition_variable>
#include <mutex>
#include <vector>

#include "nk_internal.h"

namespace {

constexpr int kMaxLoopRanks = 16;

struct Srcs {
  const void *p[kMaxLoopRanks];
};

// dst[i] = sum over ranks of src_r[i] (u32 / u64 wrap like RCCL's ncclSum)
template <typename T>
__global__ void k_loop_sum(Srcs s, int W, T *__restrict__ dst, uint64_t n) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    T acc = 0;
    for (int w = 0; w < W; ++w) acc += ((const T *)s.p[w])[i];
    dst[i] = acc;
  }
}

int failf(int code, const char *what, hipError_t e = hipSuccess) {
  char buf[256];
  snprintf(buf, sizeof buf, "loopback transport: %s%s%s", what, e != hipSuccess ? ": " : "",
           e != hipSuccess ? hipGetErrorString(e) : "");
  return nk_fail_msg(code, buf);
}

}  // namespace

struct nk_loop_group {
  int world = 0;
  int device = -1;
  int joined = 0;
  std::vector<bool> member;  // rank r holds a live communicator
  std::mutex mu;
  std::condition_variable cv;
  uint64_t gen = 0;
  int arrived = 0;
  bool broken = false;
  int root_rc = NK_OK;
  std::vector<const void *> send;
  std::vector<void *> recv;
  void *scratch = nullptr;
  size_t scratch_bytes = 0;

  // every rank arrives (or the group breaks: a rank that failed or timed out
  // releases the others with an error instead of leaving them waiting)
  int barrier() {
    std::unique_lock<std::mutex> lk(mu);
    if (broken) return failf(NK_E_DEVICE, "group broken by another rank");
    const uint64_t my = gen;
    if (++arrived == world) {
      arrived = 0;
      ++gen;
      cv.notify_all();
      return NK_OK;
    }
    if (!cv.wait_for(lk, std::chrono::seconds(120), [&] { return gen != my || broken; })) {
      broken = true;
      cv.notify_all();
      return failf(NK_E_DEVICE, "a rank did not reach the collective within 120 s");
    }
    return broken ? failf(NK_E_DEVICE, "group broken by another rank") : NK_OK;
  }
  void fail_all() {
    std::lock_guard<std::mutex> lk(mu);
    broken = true;
    cv.notify_all();
  }
};

namespace nk {

int loop_world(const nk_loop_group *g) { return g->world; }

void loop_break(nk_loop_group *g) { g->fail_all(); }

int loop_join(nk_loop_group *g, int rank, int device) {
  std::lock_guard<std::mutex> lk(g->mu);
  if (rank < 0 || rank >= g->world) return failf(NK_E_INVALID, "rank out of range");
  if (g->device < 0) g->device = device;
  if (g->device != device) return failf(NK_E_INVALID, "all ranks of a loopback group use one device");
  // two communicators for one rank would overwrite each other's send/recv
  // slots and corrupt every collective
  if (g->member[rank]) return failf(NK_E_INVALID, "rank already joined this loopback group");
  g->member[rank] = true;
  ++g->joined;
  return NK_OK;
}

void loop_leave(nk_loop_group *g, int rank) {
  std::lock_guard<std::mutex> lk(g->mu);
  if (rank >= 0 && rank < g->world && g->member[rank]) {
    g->member[rank] = false;
    --g->joined;
  }
}

// One collective on rank `rank`: kind 0 all-reduce (sum; n elements), 1
// all-gather (n elements per rank), 2 reduce-scatter (sum; n per rank out of
// W*n).  elem: 4 or 8 bytes.  Blocks the calling thread until every rank's
// result is in place on its stream.
int loop_collective(nk_loop_group *g, int rank, int kind, const void *send, void *recv, size_t n,
                    int elem, hipStream_t s) {
  const size_t W = (size_t)g->world;
  hipError_t e = hipStreamSynchronize(s);  // this rank's input is complete
  if (e != hipSuccess) {
    g->fail_all();
    return failf(NK_E_DEVICE, "stream synchronize", e);
  }
  {
    std::lock_guard<std::mutex> lk(g->mu);
    g->send[rank] = send;
    g->recv[rank] = recv;
  }
  if (int rc = g->barrier()) return rc;
  const size_t out_n = kind == 0 ? n : W * n;  // elements in the scratch result
  if (rank == 0) {
    int rc = NK_OK;
    if (g->scratch_bytes < out_n * elem) {
      if (g->scratch) (void)hipFree(g->scratch);
      g->scratch = nullptr;
      g->scratch_bytes = 0;
      if ((e = hipMalloc(&g->scratch, std::max<size_t>(out_n * elem, 16))) != hipSuccess)
        rc = failf(NK_E_OOM, "scratch allocation", e);
      else
        g->scratch_bytes = std::max<size_t>(out_n * elem, 16);
    }
    if (!rc && out_n) {
      if (kind == 1) {
        for (size_t r = 0; r < W && e == hipSuccess; ++r)
          e = hipMemcpyAsync((char *)g->scratch + r * n * elem, g->send[r], n * elem,
                             hipMemcpyDeviceToDevice, s);
      } else {
        Srcs src{};
        for (size_t r = 0; r < W; ++r) src.p[r] = g->send[r];
        const unsigned blocks = (unsigned)std::min<size_t>((out_n + 255) / 256, 4096);
        if (elem == 4)
          hipLaunchKernelGGL(k_loop_sum<uint32_t>, dim3(blocks), dim3(256), 0, s, src, (int)W,
                             (uint32_t *)g->scratch, (uint64_t)out_n);
        else
          hipLaunchKernelGGL(k_loop_sum<uint64_t>, dim3(blocks), dim3(256), 0, s, src, (int)W,
                             (uint64_t *)g->scratch, (uint64_t)out_n);
        e = hipGetLastError();
      }
      if (e == hipSuccess) e = hipStreamSynchronize(s);
      if (e != hipSuccess) rc = failf(NK_E_DEVICE, "combine", e);
    }
    std::lock_guard<std::mutex> lk(g->mu);
    g->root_rc = rc;
  }
  if (int rc = g->barrier()) return rc;
  int rc = g->root_rc;
  if (rc) return failf(rc, "the root rank's combine failed");  // (every rank returns here)
  if (out_n) {
    const char *from = (const char *)g->scratch + (kind == 2 ? rank * n * elem : 0);
    const size_t bytes = (kind == 2 ? n : out_n) * elem;
    if (bytes) e = hipMemcpyAsync(recv, from, bytes, hipMemcpyDeviceToDevice, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) {
      g->fail_all();
      return failf(NK_E_DEVICE, "result copy", e);
    }
  }
  return g->barrier();  // the scratch is free for the next collective
}

}  // namespace nk

extern "C" {

nk_loop_group *nk_loop_group_new(int world) {
  if (world < 1 || world > kMaxLoopRanks) {
    failf(NK_E_INVALID, "world must be in 1 .. 16");
    return nullptr;
  }
  nk_loop_group *g = new nk_loop_group();
  g->world = world;
  g->send.assign(world, nullptr);
  g->recv.assign(world, nullptr);
  g->member.assign(world, false);
  return g;
}

void nk_loop_group_free(nk_loop_group *g) {
  if (!g) return;
  if (g->scratch) {
    (void)hipSetDevice(g->device);
    (void)hipDeviceSynchronize();
    (void)hipFree(g->scratch);
  }
  delete g;
}

}  // extern "C"
