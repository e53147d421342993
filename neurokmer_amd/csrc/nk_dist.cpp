// nk_dist.cpp — the multi-GPU finish with its collectives inside the library:
// RCCL over xGMI, one communicator per rank (include/neurokmer.h, nk_comm_*,
// nk_finalize_dist, nk_finalize_sliced_dist).
//
// The counter's split-phase entry points (nk_wire32 .. nk_merge_export,
// nk_finalize_slice / nk_adopt_slices) are enqueued on one stream together
// with the RCCL calls, so the GPU runs count -> wire -> all-reduce -> LIF +
// top-N + export -> all-gather -> merge back to back, and the host waits once,
// for the merged results (neurokmer_amd/dist.py drove the same protocol from
// Python with torch's collectives between the calls; every call was a host
// round trip the GPU idled through).  Replaces the reference's
// in-process rayon reduce of the per-record currents (src/spiking_hash.rs:
// 145-154), which is a commutative u64 sum and so shards across GPUs.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <unordered_map>
#include <vector>

#include "neurokmer.h"
#include "nk_internal.h"
#include "nk_kernels.h"

namespace {

template <typename T>
struct Buf {
  T *p = nullptr;
  size_t n = 0;
  // zero_on: zero a new allocation on that stream, ahead of the caller's work
  // there (hipMemset runs on the null stream, which does not order against
  // non-blocking streams: a rank's wire written on its stream was zeroed after
  // it, now and then -- the loopback world-3 refine case lost a whole rank's
  // counts in 3 of 40 runs, tools/loop_flake.py)
  bool ensure(size_t want, hipStream_t zero_on = nullptr, bool zero = false) {
    if (want <= n) return true;
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
    if (hipMalloc((void **)&p, std::max<size_t>(want, 1) * sizeof(T)) != hipSuccess) {
      p = nullptr;
      return false;
    }
    if (zero && hipMemsetAsync(p, 0, want * sizeof(T), zero_on) != hipSuccess) return false;
    n = want;
    return true;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
  }
};

// per handle: the wire vector, the segments and the all-gather buffers
struct HandleBufs {
  Buf<uint32_t> wire32;        // [P] u32 wire (plain) or [W*S] (sliced, zero past P)
  Buf<uint64_t> wire64;        // [W*S] u64 wire of the sliced finish (zero past P)
  Buf<uint32_t> part32;        // [S] reduce-scatter result
  Buf<uint64_t> part64;
  Buf<uint64_t> seg, all;      // export segment [stride] and all-gather [W*stride]
  Buf<uint64_t> sseg, sall;    // slice rows segment and its all-gather
  Buf<uint64_t> useg, uall;    // padded top k-mer union exchange
  Buf<uint64_t> nvec;          // [W] key counts (variable-length fallback)
  uint64_t wire_pool = 0;      // pool the sliced wires' zero padding was laid out for
  void release() {
    wire32.release(); wire64.release(); part32.release(); part64.release();
    seg.release(); all.release(); sseg.release(); sall.release();
    useg.release(); uall.release(); nvec.release();
  }
};

int failf(int code, const char *fmt, ...) __attribute__((format(printf, 2, 3)));
int failf(int code, const char *fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  return nk_fail_msg(code, buf);
}

// RCCL is bound at first use, not at link time: a process that already holds
// an RCCL (PyTorch-ROCm loads its own copy, file librccl.so, soname
// librccl.so.1) must not load a second one -- two copies in one process
// corrupt the heap at exit.  The copy already loaded is taken, else
// /opt/rocm's.
struct Rccl {
  decltype(&ncclGetUniqueId) get_unique_id = nullptr;
  decltype(&ncclCommInitRank) comm_init_rank = nullptr;
  decltype(&ncclCommDestroy) comm_destroy = nullptr;
  decltype(&ncclAllReduce) all_reduce = nullptr;
  decltype(&ncclAllGather) all_gather = nullptr;
  decltype(&ncclReduceScatter) reduce_scatter = nullptr;
  decltype(&ncclGetErrorString) error_string = nullptr;
  bool ok = false;
};

const Rccl &rccl() {
  static const Rccl r = [] {
    Rccl x;
    void *h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) return x;
    x.get_unique_id = (decltype(x.get_unique_id))dlsym(h, "ncclGetUniqueId");
    x.comm_init_rank = (decltype(x.comm_init_rank))dlsym(h, "ncclCommInitRank");
    x.comm_destroy = (decltype(x.comm_destroy))dlsym(h, "ncclCommDestroy");
    x.all_reduce = (decltype(x.all_reduce))dlsym(h, "ncclAllReduce");
    x.all_gather = (decltype(x.all_gather))dlsym(h, "ncclAllGather");
    x.reduce_scatter = (decltype(x.reduce_scatter))dlsym(h, "ncclReduceScatter");
    x.error_string = (decltype(x.error_string))dlsym(h, "ncclGetErrorString");
    x.ok = x.get_unique_id && x.comm_init_rank && x.comm_destroy && x.all_reduce &&
           x.all_gather && x.reduce_scatter && x.error_string;
    return x;
  }();
  return r;
}

int need_rccl() {
  return rccl().ok ? NK_OK : failf(NK_E_UNSUPPORTED, "RCCL (librccl.so.1) could not be loaded");
}

}  // namespace

struct nk_comm {
  ncclComm_t comm = nullptr;
  nk_loop_group *loop = nullptr;  // the loopback transport instead of RCCL (nk_loop.hip)
  int world = 0, rank = 0, device = 0;
  // per handle, keyed by its never-reused id (a handle freed and another
  // allocated at the same address must not inherit the buffers' state)
  std::unordered_map<uint64_t, HandleBufs> bufs;
  HandleBufs &of(const nk_counter *c) { return bufs[nk::counter_uid(c)]; }
};

#define NCCLCHK(expr)                                                                  \
  do {                                                                                 \
    ncclResult_t r_ = (expr);                                                          \
    if (r_ != ncclSuccess)                                                             \
      return failf(NK_E_DEVICE, "%s failed: %s", #expr, rccl().error_string(r_));     \
  } while (0)
#define RC(expr)              \
  do {                        \
    int rc_ = (expr);         \
    if (rc_) return rc_;      \
  } while (0)
#define OOM(ok, what) \
  do {                \
    if (!(ok)) return failf(NK_E_OOM, "device allocation of the %s failed", what); \
  } while (0)

namespace {

// The three collectives the finish uses, over RCCL or the loopback transport
// (n: elements per rank for the all-gather and the reduce-scatter's output)
int coll(nk_comm *m, int kind, const void *send, void *recv, size_t n, bool u64, hipStream_t s) {
  if (m->loop)
    return nk::loop_collective(m->loop, m->rank, kind, send, recv, n, u64 ? 8 : 4, s);
  const ncclDataType_t dt = u64 ? ncclUint64 : ncclUint32;
  switch (kind) {
    case 0: NCCLCHK(rccl().all_reduce(send, recv, n, dt, ncclSum, m->comm, s)); break;
    case 1: NCCLCHK(rccl().all_gather(send, recv, n, dt, m->comm, s)); break;
    default: NCCLCHK(rccl().reduce_scatter(send, recv, n, dt, ncclSum, m->comm, s)); break;
  }
  return NK_OK;
}
int all_reduce(nk_comm *m, const void *send, void *recv, size_t n, bool u64, hipStream_t s) {
  return coll(m, 0, send, recv, n, u64, s);
}
int all_gather(nk_comm *m, const void *send, void *recv, size_t n, bool u64, hipStream_t s) {
  return coll(m, 1, send, recv, n, u64, s);
}
int reduce_scatter(nk_comm *m, const void *send, void *recv, size_t n, bool u64, hipStream_t s) {
  return coll(m, 2, send, recv, n, u64, s);
}

// The top rows' uniques column from the union of every shard's distinct top
// k-mers (after a finish that left the rows set but the column per shard):
// one fixed-size all-gather of [n, keys...] segments; a segment past `cap`
// (every rank sees the same headers) redoes it with cap = the largest n.
int union_top_kmers(nk_counter *c, nk_comm *m, HandleBufs &b, size_t cap, hipStream_t s) {
  const int wpk = nk::counter_key_words(c);
  const size_t W = (size_t)m->world;
  for (int pass = 0; pass < 2; ++pass) {
    const size_t stride = 1 + (size_t)wpk * cap;
    OOM(b.useg.ensure(stride) && b.uall.ensure(W * stride), "key union buffers");
    RC(nk_top_kmers_padded(c, b.useg.p, cap, s));
    RC(all_gather(m, b.useg.p, b.uall.p, stride, true, s));
    int complete = 0;
    RC(nk_merge_top_kmers_padded(c, b.uall.p, W, stride, cap, &complete, s));
    if (complete) return NK_OK;
    if (pass) break;
    // the largest shard list sets the cap of the second exchange
    const uint64_t *dk = nullptr;
    size_t n = 0;
    RC(nk_top_kmers(c, &dk, &n));  // (host wait)
    OOM(b.nvec.ensure(2 * W), "key count buffer");
    const uint64_t mine = n;
    if (hipMemcpyAsync(b.nvec.p, &mine, 8, hipMemcpyHostToDevice, s) != hipSuccess)
      return failf(NK_E_DEVICE, "key count copy failed");
    RC(all_gather(m, b.nvec.p, b.nvec.p + W, 1, true, s));
    std::vector<uint64_t> all(W);
    if (hipMemcpyAsync(all.data(), b.nvec.p + W, W * 8, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
      return failf(NK_E_DEVICE, "key count readback failed");
    cap = std::max<size_t>(1, (size_t)*std::max_element(all.begin(), all.end()));
  }
  return failf(NK_E_DEVICE, "top k-mer union incomplete after the exact-size exchange");
}

}  // namespace

extern "C" {

int nk_comm_unique_id(uint8_t id[NK_COMM_ID_BYTES]) {
  if (!id) return failf(NK_E_INVALID, "null id");
  RC(need_rccl());
  ncclUniqueId u;
  NCCLCHK(rccl().get_unique_id(&u));
  static_assert(sizeof u == NK_COMM_ID_BYTES, "RCCL unique id size");
  memcpy(id, &u, sizeof u);
  return NK_OK;
}

nk_comm *nk_comm_new(const uint8_t id[NK_COMM_ID_BYTES], int world, int rank, int device) {
  if (!id || world < 1 || rank < 0 || rank >= world) {
    failf(NK_E_INVALID, "bad communicator arguments (world %d, rank %d)", world, rank);
    return nullptr;
  }
  if (hipSetDevice(device) != hipSuccess) {
    failf(NK_E_NO_DEVICE, "hipSetDevice(%d) failed", device);
    return nullptr;
  }
  if (need_rccl()) return nullptr;
  ncclUniqueId u;
  memcpy(&u, id, sizeof u);
  nk_comm *m = new nk_comm();
  m->world = world;
  m->rank = rank;
  m->device = device;
  const ncclResult_t r = rccl().comm_init_rank(&m->comm, world, u, rank);
  if (r != ncclSuccess) {
    failf(NK_E_DEVICE, "ncclCommInitRank failed: %s", rccl().error_string(r));
    delete m;
    return nullptr;
  }
  return m;
}

nk_comm *nk_comm_new_loopback(nk_loop_group *g, int rank, int device) {
  if (!g) {
    failf(NK_E_INVALID, "null loopback group");
    return nullptr;
  }
  if (hipSetDevice(device) != hipSuccess) {
    failf(NK_E_NO_DEVICE, "hipSetDevice(%d) failed", device);
    return nullptr;
  }
  if (nk::loop_join(g, rank, device)) return nullptr;
  nk_comm *m = new nk_comm();
  m->loop = g;
  m->world = nk::loop_world(g);
  m->rank = rank;
  m->device = device;
  return m;
}

void nk_comm_forget(nk_comm *m, const nk_counter *c) {
  if (!m || !c) return;
  auto it = m->bufs.find(nk::counter_uid(c));
  if (it == m->bufs.end()) return;
  (void)hipSetDevice(m->device);
  (void)hipDeviceSynchronize();
  it->second.release();
  m->bufs.erase(it);
}

void nk_comm_free(nk_comm *m) {
  if (!m) return;
  (void)hipSetDevice(m->device);
  (void)hipDeviceSynchronize();
  for (auto &kv : m->bufs) kv.second.release();
  if (m->comm) (void)rccl().comm_destroy(m->comm);
  if (m->loop) nk::loop_leave(m->loop, m->rank);
  delete m;
}

static int finalize_dist_impl(nk_counter *c, nk_comm *m, int streaming, uint64_t total_kmers,
                              size_t cap, void *stream) {
  if (!c || !m) return failf(NK_E_INVALID, "null argument");
  if (!cap || cap > (1u << 24)) return failf(NK_E_INVALID, "cap must be in 1 .. 2^24");
  // the library's calls and the collectives share this stream's order (a NULL
  // stream would mean the handle's private stream to the library's calls)
  if (!stream) return failf(NK_E_INVALID, "a stream is required");
  (void)hipSetDevice(m->device);
  hipStream_t s = (hipStream_t)stream;
  HandleBufs &b = m->of(c);
  const uint64_t P = nk_pool_size(c);
  const size_t W = (size_t)m->world;
  if (nk::counter_kpn_global(c)) {  // exact table adopted: u64 currents, uniques from kpn
    uint64_t *cur = nk::counter_currents_on(c, s);
    if (!cur && P) return NK_E_DEVICE;
    if (P) RC(all_reduce(m, cur, cur, P, true, s));
    return nk_finalize(c, streaming, stream);
  }
  const uint32_t *wire = nullptr;
  if (total_kmers < (1ull << 31)) {  // no summed current can leave u32
    OOM(b.wire32.ensure(std::max<uint64_t>(P, 1)), "wire vector");
    RC(nk_wire32(c, b.wire32.p, stream));
    if (P) RC(all_reduce(m, b.wire32.p, b.wire32.p, P, false, s));
    wire = b.wire32.p;
  } else {
    uint64_t *cur = nk::counter_currents_on(c, s);
    if (!cur && P) return NK_E_DEVICE;
    if (P) RC(all_reduce(m, cur, cur, P, true, s));
  }
  const size_t stride = 1 + (size_t)nk::counter_key_words(c) * cap;
  OOM(b.seg.ensure(stride) && b.all.ensure(W * stride), "export segments");
  nk::counter_merge_hint(c, (uint32_t)W);
  RC(nk_finalize_export(c, streaming, wire, b.seg.p, cap, stream));
  RC(all_gather(m, b.seg.p, b.all.p, stride, true, s));
  int redo = 0;
  RC(nk_merge_export(c, b.all.p, W, stride, cap, &redo, stream));
  if (!redo) return NK_OK;
  RC(nk_finalize_redo(c, stream));
  return union_top_kmers(c, m, b, cap, s);
}

static int finalize_sliced_dist_impl(nk_counter *c, nk_comm *m, int streaming,
                                     uint64_t total_kmers, size_t cap, void *stream) {
  if (!c || !m) return failf(NK_E_INVALID, "null argument");
  if (!cap || cap > (1u << 24)) return failf(NK_E_INVALID, "cap must be in 1 .. 2^24");
  // the library's calls and the collectives share this stream's order (a NULL
  // stream would mean the handle's private stream to the library's calls)
  if (!stream) return failf(NK_E_INVALID, "a stream is required");
  (void)hipSetDevice(m->device);
  hipStream_t s = (hipStream_t)stream;
  HandleBufs &b = m->of(c);
  const uint64_t P = nk_pool_size(c);
  const uint64_t W = (uint64_t)m->world;
  const uint64_t S = P ? (P + W - 1) / W : 0;  // neurons per slice (the last may be short)
  const uint64_t lo = std::min<uint64_t>(P, (uint64_t)m->rank * S), hi = std::min<uint64_t>(P, lo + S);
  const bool small = total_kmers < (1ull << 31);
  if (b.wire_pool != P) {  // the padding past P must be zero: lay the wires out afresh
    b.wire32.release();
    b.wire64.release();
    b.wire_pool = P;
  }
  const void *slice = nullptr;
  if (small) {
    OOM(b.wire32.ensure(std::max<uint64_t>(W * S, 1), s, true) && b.part32.ensure(std::max<uint64_t>(S, 1)),
        "slice wire");
    RC(nk_wire32(c, b.wire32.p, stream));
    if (S) RC(reduce_scatter(m, b.wire32.p, b.part32.p, S, false, s));
    slice = b.part32.p;
  } else {
    OOM(b.wire64.ensure(std::max<uint64_t>(W * S, 1), s, true) && b.part64.ensure(std::max<uint64_t>(S, 1)),
        "slice wire");
    uint64_t *cur = nk::counter_currents_on(c, s);
    if (!cur && P) return NK_E_DEVICE;
    if (P && hipMemcpyAsync(b.wire64.p, cur, P * 8, hipMemcpyDeviceToDevice, s) != hipSuccess)
      return failf(NK_E_DEVICE, "wire copy failed");
    if (S) RC(reduce_scatter(m, b.wire64.p, b.part64.p, S, true, s));
    slice = b.part64.p;
  }
  const uint64_t rows = nk::counter_rows(c);
  const size_t stride = 3 + 3 * rows;
  OOM(b.sseg.ensure(stride) && b.sall.ensure(W * stride), "slice row segments");
  if (small && W * rows <= (uint64_t)nk::kAdoptMax) {
    // no host wait before the merge: the slice's LIF + top rows, the global
    // rows and this shard's uniques all on the device (nk_slice_export ..
    // nk_merge_export); a redo takes the blocking selection without the LIF
    const size_t kstride = 1 + (size_t)nk::counter_key_words(c) * cap;
    OOM(b.seg.ensure(kstride) && b.all.ensure(W * kstride), "export segments");
    RC(nk_slice_export(c, streaming, hi > lo ? (const uint32_t *)slice : nullptr, lo, hi, b.sseg.p,
                       rows, stream));
    RC(all_gather(m, b.sseg.p, b.sall.p, stride, true, s));
    RC(nk_adopt_export(c, b.sall.p, W, stride, b.seg.p, cap, stream));
    RC(all_gather(m, b.seg.p, b.all.p, kstride, true, s));
    int redo = 0;
    RC(nk_merge_export(c, b.all.p, W, kstride, cap, &redo, stream));
    if (!redo) return NK_OK;
    RC(nk::slice_reselect(c, lo, hi, b.sseg.p, rows, s));
    RC(all_gather(m, b.sseg.p, b.sall.p, stride, true, s));
    RC(nk_adopt_slices(c, b.sall.p, W, stride, stream));
    return union_top_kmers(c, m, b, cap, s);
  }
  RC(nk_finalize_slice(c, streaming, hi > lo ? slice : nullptr, small ? 32 : 64, lo, hi, b.sseg.p,
                       rows, stream));
  RC(all_gather(m, b.sseg.p, b.sall.p, stride, true, s));
  RC(nk_adopt_slices(c, b.sall.p, W, stride, stream));
  return union_top_kmers(c, m, b, cap, s);
}

// (a loopback rank that fails releases the others at once instead of leaving
// them at the next collective until the group's timeout)
int nk_finalize_dist(nk_counter *c, nk_comm *m, int streaming, uint64_t total_kmers, size_t cap,
                     void *stream) {
  const int rc = finalize_dist_impl(c, m, streaming, total_kmers, cap, stream);
  if (rc && m && m->loop) nk::loop_break(m->loop);
  return rc;
}

int nk_finalize_sliced_dist(nk_counter *c, nk_comm *m, int streaming, uint64_t total_kmers,
                            size_t cap, void *stream) {
  const int rc = finalize_sliced_dist_impl(c, m, streaming, total_kmers, cap, stream);
  if (rc && m && m->loop) nk::loop_break(m->loop);
  return rc;
}

}  // extern "C"
