// nk_counter.cpp — host orchestrator behind the C ABI (include/neurokmer.h).
//
// Mirrors SpikingKmerCounter (src/spiking_hash.rs:16-715) with all per-neuron
// state resident in HBM of one MI355X:
//   currents u64[P] | voltage f32[P] | refractory u32[P] | spike_count u64[P]
// and drives the gfx950 kernels of nk_kernels.hip on one HIP stream.
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>
#include <string.h>
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <future>
#include <string>
#include <vector>

#include "neurokmer.h"
#include "nk_exact.h"
#include "nk_fastx.h"
#include "nk_ingest.h"
#include "nk_reader.h"
#include "nk_kernels.h"

// K1b workgroups per batch (one 128 KiB-LDS workgroup per CU: one round on 256 CUs)
#ifndef NK_K1B_WGS
#define NK_K1B_WGS 256
#endif

using namespace nk;

namespace {

thread_local std::string g_err;

int fail(int code, const char *fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

#define HIPCHK(expr)                                                                  \
  do {                                                                                \
    hipError_t e_ = (expr);                                                           \
    if (e_ != hipSuccess)                                                             \
      return fail(NK_E_DEVICE, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), \
                  __FILE__, __LINE__);                                                \
  } while (0)

template <typename T>
struct DevBuf {
  T *p = nullptr;
  size_t n = 0;
  int ensure(size_t want) {
    if (want <= n) return NK_OK;
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
    if (hipMalloc((void **)&p, std::max<size_t>(want, 1) * sizeof(T)) != hipSuccess) {
      p = nullptr;
      return fail(NK_E_OOM, "hipMalloc of %zu bytes failed", want * sizeof(T));
    }
    n = want;
    return NK_OK;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
  }
};

// pinned host memory (the file ingest's double buffer)
struct PinnedBuf {
  uint8_t *p = nullptr;
  size_t n = 0;
  int ensure(size_t want) {
    if (want <= n) return NK_OK;
    release();
    if (hipHostMalloc((void **)&p, want) != hipSuccess) {
      p = nullptr;
      return fail(NK_E_OOM, "hipHostMalloc of %zu bytes failed", want);
    }
    n = want;
    return NK_OK;
  }
  void release() {
    if (p) (void)hipHostFree(p);
    p = nullptr;
    n = 0;
  }
};

constexpr int kLifTable = 1 << 16;
constexpr int kStages = 7;
const char *kStageNames[kStages] = {"index", "count", "hist", "lif", "topn", "uniques", "total"};
// default (opts.stage_timing == 0): events only around the count kernel and at
// both ends; an event between two kernels idles the GPU for ~6 us on MI355X
constexpr int kStagesLight = 4;
const char *kStageNamesLight[kStagesLight] = {"index", "count", "post", "total"};

}  // namespace

static std::atomic<uint64_t> g_next_uid{1};

struct nk_counter {
  // never reused (nk_dist.cpp keys a communicator's per-handle buffers by it)
  const uint64_t uid = g_next_uid.fetch_add(1);
  size_t k = 0, pool = 0;
  float thr = 1.0f, leak = 0.95f;
  uint32_t refr = 2;
  double cost = 1.0;
  int canonical = 0;
  uint64_t steps = 1000;
  nk_opts opts{};
  int device = 0;
  hipStream_t own_stream = nullptr;

  // neuron state (HBM)
  DevBuf<uint64_t> cur, sc;
  DevBuf<float> v;
  DevBuf<uint32_t> r;
  // scratch
  DevBuf<uint32_t> tile_rec, hist, tie_cnt, uniq, special;
  DevBuf<uint64_t> stats;  // [0] new spikes, [1] max spike count
  DevBuf<LifEntry> lif_tbl;
  DevBuf<TopState> topst;
  DevBuf<TopCand> cand;
  DevBuf<uint64_t> top_cur;
  DevBuf<unsigned long long> set_keys;
  DevBuf<uint64_t> top_keys;
  DevBuf<unsigned long long> top_keys_n;
  DevBuf<uint32_t> trunc_d;  // a padded all-gather segment held more keys than its cap
  bool top_keys_ready = false;  // top_keys holds this shard's compacted list (padded export)
  DevBuf<uint32_t> radix_h;
  uint64_t set_cap = 0;     // capacity used by the last uniques pass
  uint64_t set_alloc = 0;   // allocated capacity of set_keys (keys)
  // set_keys[i] == kEmpty for every i >= set_dirty; set_clean: for every i (the
  // count's prep kernel empties [0, set_dirty) for the partitioned path's scan)
  uint64_t set_dirty = 0, dirty_before = 0;
  bool set_clean = false;
  bool w128 = false;        // --kmer-width=128: u128 keys, 3 set words per key
  size_t n_top_keys = 0;
  DevBuf<uint64_t> set_mask_d, set_need_d;
  DevBuf<unsigned long long> hits, n_hits;  // uniques hit records (cap = set_alloc / 2)
  DevBuf<uint32_t> post_flags;  // [0] set too small [1] top bucket overflowed [2] top buckets
  // packed finalize results: ResultHdr | cand[m] | uniq[m]
  static constexpr size_t kResBytes = sizeof(ResultHdr) + kMaxTopN * (sizeof(TopCand) + 4);
  // + a 64-B line after the results: k_gather's completion word (res_seq)
  static constexpr size_t kResFlagOff = (kResBytes + 63) & ~(size_t)63;
  uint8_t *res_h = nullptr;   // pinned, mapped: written by k_gather
  uint8_t *res_hd = nullptr;  // its device-side address
  uint64_t res_seq = 0;       // last completion word asked of k_gather
  // host copies of input (host-array entry points)
  DevBuf<uint8_t> in_bases;
  DevBuf<uint64_t> in_offs;
  // GPU FASTX ingest buffers, kept between file calls
  PinnedBuf ing_hb[3];                    // chunk i of a file in ing_hb[i % 3]
  DevBuf<uint8_t> ing_draw, ing_scratch;
  DevBuf<uint8_t> ing_draw2;              // the second raw-chunk buffer (H2D of the next chunk)
  hipStream_t ing_cs = nullptr;           // the ingest's copy stream
  hipEvent_t ing_ev[4] = {};              // copied[0..1], free[0..1]
  DevBuf<IngestState> ing_dst;
  // LIF table cache key
  bool lif_valid = false;
  LifParams lif_key{};
  // partitioned count (k <= 32, pool <= kMaxBuckets * 32768)
  DevBuf<uint16_t> p_off, p_pos;
  DevBuf<unsigned long long> p_fill;
  DevBuf<uint2> p_desc;
  DevBuf<uint32_t> p_over, partials, tbuckets;
  PartArgs last_pa{};
  // wide partition (pool > 16.7 M or big-key modes past it): coarse buckets
  DevBuf<uint32_t> w_rec, w_over;
  DevBuf<unsigned long long> w_fill;
  // pipelined split (split_pipelined): the coarse records of k_part_gen launch
  // g are split on split_s while launch g + 1 hashes; w_snap[g][bucket] = the
  // records reserved after launch g
  static constexpr int kSplitMax = 32;
  hipStream_t split_s = nullptr;
  hipEvent_t split_ev[kSplitMax + 1] = {};
  DevBuf<unsigned long long> w_snap;
  // overflow target of a write-through K1b (PartArgs::out), kept zero
  DevBuf<unsigned long long> ovf;
  size_t ovf_zeroed = 0;  // entries known zero
  uint32_t pend_slices = 0;  // K1b partials not yet folded into cur (fused into LIF)
  bool cur_in_wire = false;  // nk_wire32 moved the currents into the caller's wire vector
  // multi-GPU export (nk_finalize_export -> nk_merge_export -> [nk_finalize_redo])
  DevBuf<unsigned long long> export_n;  // key counter of k_export_keys (kept zero between uses)
  bool export_n_zeroed = false;
  uint64_t *xport_dst = nullptr;  // set while nk_finalize_export enqueues its uniques pass
  uint64_t xport_cap = 0;
  // the union of the segments (nk_merge_export), apart from this shard's set
  DevBuf<unsigned long long> mset_keys;
  DevBuf<uint64_t> mset_mask_d;
  DevBuf<uint32_t> muniq, mspecial;
  uint64_t mset_alloc = 0;
  bool export_pending = false, export_uniq = false, export_blocking = false, redo_ready = false;
  uint32_t export_want = 0;
  ResultHdr last_hdr{};
  bool lif_zeroed = false;   // hist/stats already zeroed by this call's prep kernel
  bool state_fresh = true;   // spikes/v/r are logically zero (lazy reset)
  // the last LIF ran from the reset state, so v / r / spike counts are a
  // function of each neuron's count (cur) and were not written: derived_lp
  // and the closed-form table give them back (settle_state writes them out)
  bool state_derived = false;
  LifParams derived_lp{};
  // the last accumulate's write-through K1b also ran the LIF from the reset
  // state with these parameters (sc8, hist, stats written): the next LIF of a
  // finalize is skipped while nothing else touched the currents or the state
  bool k1b_lif = false;
  LifParams k1b_lp{};
  // nk_finalize_dist: the world size of the merge that follows the next export
  // (the export's header kernel empties the merge set, nk_merge_export then
  // skips k_merge_prep for that capacity)
  uint32_t merge_world_hint = 0;
  uint64_t merge_prepped = 0;
  // min(spike count, 255) per neuron, written by a LIF whose top-N is not fused
  // (large pools): what the top-N passes read first (1 B instead of 8 per neuron)
  DevBuf<uint8_t> sc8;
  bool sc8_ok = false;
  bool cur_fresh = true;     // currents are logically zero (lazy reset)
  // exact k-mer table (opts.exact_counts, nk_exact.h)
  DevBuf<uint64_t> x_keys, x_sorted, x_uniq, x_q;
  DevBuf<uint32_t> x_cnt, x_tile_rec, kpn, x_out, x_pres, x_cs;
  // multi-GPU exact table: pairs grouped by owner rank
  DevBuf<uint64_t> xp_keys;
  DevBuf<uint32_t> xp_cnt;
  DevBuf<unsigned long long> xp_ctr;
  DevBuf<uint8_t> x_tmp;
  // [0] keys of the last input (sorted build) / of a process_sequence record,
  // [1] table entries (sorted: distinct keys; grouped: span + side part),
  // [2] grouped: first index of the side part, [3] side part's entries,
  // [4] grouped span, [5] side records, [6] grouped: distinct keys, [7] scratch
  DevBuf<unsigned long long> x_n;
  // kmer_per_neuron by partition (table_kpn): fine / coarse bucket regions,
  // K1b partials, and the overflow + slices == 1 target (all zero between uses)
  DevBuf<uint16_t> xk_off;
  DevBuf<uint32_t> xk_over, xk_wrec, xk_wover, xk_part;
  DevBuf<unsigned long long> xk_fill, xk_wfill, xk_cur;
  size_t xk_cur_zeroed = 0;
  bool exact_built = false;        // the table holds the last process/accumulate input
  // the grouped table (nk_table.hip): ent per neuron; the count's K1a<KEYS>
  // keys (p_key, kept_keys: the count arena holds this input's keyed records)
  // or the table's own K1a<KEYS> arena (xg_*), the regrouped records, the side list
  bool x_grouped = false;
  bool kept_keys = false;
  DevBuf<uint64_t> x_ent, p_key, xg_key, xg_key2, xg_side;
  DevBuf<uint16_t> xg_off;
  DevBuf<uint32_t> xg_over, xg_cnt, xg_gst, xg_trec;
  DevBuf<unsigned long long> xg_fill, xg_bctr;
  DevBuf<uint8_t> xg_bin2;
  // process_sequence: delta counts on top of the sorted table, kmer_per_neuron
  DevBuf<unsigned long long> d_keys, d_meta;
  DevBuf<uint32_t> d_vals;
  DevBuf<uint8_t> touched;
  uint64_t d_cap = 0, d_bound = 0;  // delta capacity, upper bound of its distinct keys
  bool d_dirty = true;              // delta must be cleared before use
  bool kpn_valid = false;           // kpn holds kmer_per_neuron (else it is all zero)
  bool kpn_global = false;          // table adopted across ranks: nk_finalize's uniques from kpn
  // without opts.exact_counts the table of the last process/accumulate input is
  // built on demand (get_count, kmer_per_neuron, top rows past top_n,
  // process_sequence) from that input, while it is still resident
  bool x_lazy = false;              // the table is the last input's, not built yet
  bool slice_ready = false;         // nk_finalize_slice ran; nk_adopt_slices next
  // since nk_finalize_slice the neuron state is authoritative on this rank's
  // slice only: whole-pool readers and LIF passes are refused until nk_reset
  bool sliced = false;
  uint64_t max_sc = 0;              // largest spike count of the pool (last LIF readback)
  bool input_owned = false;         // last_in is the handle's own copy (host/file entry points)
  // top_abundant_neurons(n) past the rows the last call selected
  DevBuf<uint64_t> rk_keys;         // [2P]: keys | sorted keys
  DevBuf<uint32_t> rk_idx;          // [2P]: indices | sorted indices
  DevBuf<uint8_t> rk_tmp;
  DevBuf<TopCand> rk_cand;          // the rows as TopCand (uniques gather)
  DevBuf<uint32_t> rk_uniq;
  // top-N selection fused into the LIF kernel (TopFuse)
  DevBuf<uint64_t> bcand;
  DevBuf<uint32_t> bcnt;
  bool part_used = false;
  int gen_km = -1;  // key mode of the last count when it ran k_part_gen (Gen/Wide), else -1
  // Gen/Wide count of one batch: its k_part_gen records and segment
  // descriptors are kept, so the uniques pass rescans only the tiles holding
  // the top rows' records (k_uniq_tiles) instead of the whole input
  bool gen_keep = false;
  bool gen_wide = false;
  GenPartArgs last_ga{};
  DevBuf<uint32_t> u_tiles, u_nt;
  DevBuf<uint32_t> u_mark;  // per tile: the last pass that listed it (zeroed when allocated)
  DevBuf<uint32_t> u_lanes;  // per tile: lanes with a top row's record (lane-tagged records)
  size_t u_mark_zeroed = 0;
  uint32_t u_epoch = 0;
  // input of the last accumulate (for the uniques pass)
  KmerInput last_in{};
  bool have_input = false;
  // energy (src/models.rs:145-173)
  uint64_t total_spikes = 0, total_energy = 0;
  // top rows of the last finalize
  std::vector<nk_top_row> top;
  bool top_valid = false;
  // timings
  hipEvent_t ev[kStages + 1] = {};  // see collect_timings
  float stage_ms[kStages] = {};
  int n_stage = 0;
  hipStream_t last_s = nullptr;  // stream of the previous enqueue (pick_stream)
  hipEvent_t order_ev = nullptr;
  bool order_eager = false;  // order_ev marks the end of the last call (record_order)
  int timing_pending = 0;  // 0: stage_ms is current; 1/2: collect (without/with count) on demand
  // ev[1]/ev[2] (around the count kernel) rotate through a ring, one pair per
  // accumulate call, so every call's K1 time stays readable (nk_count_history)
  static constexpr int kCountRing = 256;
  hipEvent_t cnt_ev[kCountRing][2] = {};
  uint64_t cnt_calls = 0;
  // in-kernel [start, end] s_memrealtime words of the partitioned count kernel,
  // one pair per launch in a ring (nk_count_spans): its duration with no event
  // between kernels (stage_timing 2)
  DevBuf<unsigned long long> span;
  uint64_t span_calls = 0;
};

// ev[i] for the stage timings; the inner stage boundaries only in full mode
// (stage_timing 0: also around the count kernel; 1: every stage; 2: the ends
// of a call only, so no event sits between two kernels)
static bool full_timing(const nk_counter *c) { return c->opts.stage_timing == 1; }
static bool count_timing(const nk_counter *c) { return c->opts.stage_timing < 2; }
static hipError_t mark(nk_counter *c, int i, hipStream_t s) {
  if (c->opts.stage_timing == 3) return hipSuccess;  // no events at all
  if (full_timing(c) || i == 0 || i == 6 || i == 7 || (count_timing(c) && (i == 1 || i == 2)))
    return hipEventRecord(c->ev[i], s);
  return hipSuccess;
}

static uint64_t cost_fixed(double cost) {  // Rust `(cost * 1000.0) as u64`
  double x = cost * 1000.0;
  if (!(x > 0.0)) return 0;
  if (x >= 18446744073709551616.0) return UINT64_MAX;
  return (uint64_t)x;
}

// The stream an entry point enqueues on (NULL: the handle's own stream).  When
// it differs from the previous call's, it first waits for that call's work:
// the calls of one handle stay ordered whatever streams the caller mixes.
// The wait is on an event recorded when the switch happens -- or, after
// nk_accumulate_device, on the one recorded at the end of that call
// (order_eager): by the time of the switch the caller may have queued other
// work behind it (another handle's count on a stream that shares the hardware
// queue), which a marker recorded then would wait for as well.
static hipStream_t pick_stream(nk_counter *c, void *s) {
  hipStream_t t = s ? (hipStream_t)s : c->own_stream;
  if (c->last_s && c->last_s != t && c->order_ev &&
      (c->order_eager || hipEventRecord(c->order_ev, c->last_s) == hipSuccess))
    (void)hipStreamWaitEvent(t, c->order_ev, 0);
  c->order_eager = false;
  c->last_s = t;
  return t;
}

// the end of this call's work, for the next call's pick_stream
static void record_order(nk_counter *c, hipStream_t s) {
  c->order_eager = c->order_ev && hipEventRecord(c->order_ev, s) == hipSuccess;
}

// Reset is lazy: the neuron state (spikes, v, r) and the currents are only
// marked fresh.  The next LIF takes fresh state as zero without reading it and
// writes every neuron; the next accumulate zeroes the currents in its prep
// kernel; the copy-out / pointer entry points materialise zeros on demand.
static int zero_state_on(nk_counter *c, hipStream_t) {
  c->total_spikes = c->total_energy = 0;
  c->pend_slices = 0;
  c->cur_in_wire = false;
  c->export_pending = c->redo_ready = false;
  c->top_valid = false;
  c->have_input = false;
  c->state_fresh = true;
  c->cur_fresh = true;
  c->exact_built = false;  // a fresh counter's `counts` is empty
  c->kpn_global = false;
  c->d_dirty = true;
  c->d_bound = 0;
  c->kpn_valid = false;
  c->x_lazy = false;
  c->sliced = false;
  c->max_sc = 0;
  c->state_derived = false;
  c->sc8_ok = false;
  c->k1b_lif = false;
  return NK_OK;
}

// The derived state written out: before anything reads the v / refractory /
// spike count arrays or changes the counts it is a function of.
static int settle_state(nk_counter *c, hipStream_t s) {
  if (!c->state_derived) return NK_OK;
  c->state_derived = false;
  HIPCHK(launch_lif_derive(c->cur.p, c->v.p, c->r.p, c->sc.p, c->pool, c->derived_lp, c->lif_tbl.p,
                           kLifTable, s));
  return NK_OK;
}

// spike counts of neurons [lo, ...) as the top-N passes read them
static SpikeSrc spike_src(const nk_counter *c, uint64_t lo) {
  SpikeSrc x{};
  if (c->sc8_ok) x.sc8 = c->sc8.p + lo;
  if (c->state_derived) {
    x.cur = c->cur.p + lo;
    x.tbl = c->lif_tbl.p;
    x.tbl_n = kLifTable;
    x.lp = c->derived_lp;
  } else {
    x.sc = c->sc.p + lo;
  }
  return x;
}

// LIF passes and readers of the whole pool need the whole pool's state on this
// handle: not after the pool-sliced finish (nk_finalize_slice), which leaves a
// rank authoritative on its slice only, until nk_reset
static int whole_pool(nk_counter *c) {
  if (c->sliced)
    return fail(NK_E_UNSUPPORTED,
                "the neuron state is sharded across ranks since nk_finalize_slice (this rank "
                "holds its slice only): nk_reset first, or gather the state");
  return NK_OK;
}

// materialise the lazily-zero buffers (what != 0: currents; what == 0: state)
static int materialize(nk_counter *c, bool currents, hipStream_t s) {
  ZeroList z{};
  if (currents && c->cur_fresh) {
    z.ptr[z.n] = c->cur.p; z.bytes[z.n++] = c->pool * 8;
    c->cur_fresh = false;
  }
  if (!currents && c->state_fresh) {
    c->sc8_ok = false;
    z.ptr[z.n] = c->sc.p; z.bytes[z.n++] = c->pool * 8;
    z.ptr[z.n] = c->v.p;  z.bytes[z.n++] = c->pool * 4;
    z.ptr[z.n] = c->r.p;  z.bytes[z.n++] = c->pool * 4;
    c->state_fresh = false;
  }
  if (z.n && c->pool) HIPCHK(launch_zero(z, s));
  return NK_OK;
}

// the K1b partials of an nk_accumulate_device not yet folded into the currents
// (the LIF of nk_finalize folds them itself): for every other reader
static int fold_pending(nk_counter *c, hipStream_t s) {
  if (!c->pend_slices) return NK_OK;
  HIPCHK(launch_partials_add(c->partials.p, c->pend_slices, c->pool, c->cur.p, s));
  c->pend_slices = 0;
  return NK_OK;
}

static int zero_state(nk_counter *c) {
  hipStream_t s = pick_stream(c, nullptr);
  int rc = zero_state_on(c, s);
  if (rc) return rc;
  HIPCHK(hipStreamSynchronize(s));
  c->total_spikes = c->total_energy = 0;
  c->top_valid = false;
  c->have_input = false;
  return NK_OK;
}

template <typename T>
static int copy_out(nk_counter *c, const DevBuf<T> &b, T *out, size_t n) {
  if (!c || (!out && n)) return fail(NK_E_INVALID, "null argument");
  if (n != c->pool) return fail(NK_E_INVALID, "n (%zu) must equal pool_size (%zu)", n, c->pool);
  if (!n) return NK_OK;
  (void)hipSetDevice(c->device);
  const bool is_cur = (const void *)&b == (const void *)&c->cur;
  if (is_cur && c->cur_in_wire)
    return fail(NK_E_INVALID, "the currents are in the wire vector until nk_finalize_export");
  hipStream_t s = pick_stream(c, nullptr);
  int rc = materialize(c, is_cur, s);
  if (rc) return rc;
  if (is_cur && (rc = fold_pending(c, s))) return rc;
  if (!is_cur && (rc = settle_state(c, s))) return rc;
  HIPCHK(hipStreamSynchronize(s));
  HIPCHK(hipMemcpy(out, b.p, n * sizeof(T), hipMemcpyDeviceToHost));
  return NK_OK;
}

// error text for the other translation units of the library (nk_assoc.hip)
int nk_fail_msg(int code, const char *msg) { return fail(code, "%s", msg); }

// nk_internal.h: what the multi-GPU driver (nk_dist.cpp) reads of a handle
namespace nk {
uint64_t counter_rows(const nk_counter *c) { return std::min<uint64_t>(c->opts.top_n, c->pool); }
int counter_key_words(const nk_counter *c) { return c->w128 ? 2 : 1; }
bool counter_kpn_global(const nk_counter *c) {
  return c->opts.exact_counts && c->exact_built && c->kpn_global;
}
void counter_merge_hint(nk_counter *c, uint32_t world) { c->merge_world_hint = world; }
uint64_t counter_uid(const nk_counter *c) { return c->uid; }
uint64_t *counter_currents_on(nk_counter *c, hipStream_t stream) {
  if (c->cur_in_wire) {
    fail(NK_E_INVALID, "the currents are in the wire vector until nk_finalize_export");
    return nullptr;
  }
  (void)hipSetDevice(c->device);
  hipStream_t s = pick_stream(c, stream);
  if (settle_state(c, s) || materialize(c, true, s) || fold_pending(c, s)) return nullptr;
  c->k1b_lif = false;  // the caller may change the counts
  return c->cur.p;
}
}  // namespace nk

extern "C" {

void nk_opts_default(nk_opts *o) {
  memset(o, 0, sizeof *o);
  o->device = 0;
  o->kmer_width = NK_KMER_COMPAT;
  o->top_n = 20;
}

const char *nk_last_error(void) { return g_err.c_str(); }
const char *nk_version(void) { return "neurokmer-mi355x 0.1.0 (abi 1, gfx950)"; }

nk_counter *nk_new(size_t k, float threshold, float leak, uint32_t refractory, double spike_cost,
                   size_t pool_size, int use_canonical, const nk_opts *opts) {
  if (k == 0) {
    fail(NK_E_INVALID, "k must be >= 1 (the reference panics on k == 0)");
    return nullptr;
  }
  nk_opts o;
  if (opts) o = *opts;
  else nk_opts_default(&o);
  if (o.kmer_width != NK_KMER_COMPAT && o.kmer_width != NK_KMER_128) {
    fail(NK_E_INVALID, "kmer_width %d unknown", o.kmer_width);
    return nullptr;
  }
  if (o.kmer_width == NK_KMER_128 && k > 64) {
    fail(NK_E_INVALID, "kmer_width 128 needs k <= 64 (k = %zu)", k);
    return nullptr;
  }
  if (o.top_n > (uint32_t)kMaxTopN) {
    fail(NK_E_INVALID, "top_n %u exceeds %d", o.top_n, kMaxTopN);
    return nullptr;
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
    fail(NK_E_NO_DEVICE, "no HIP device available (this library has no CPU fallback)");
    return nullptr;
  }
  if (o.device < 0 || o.device >= ndev) {
    fail(NK_E_NO_DEVICE, "device %d out of range (%d devices)", o.device, ndev);
    return nullptr;
  }
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, o.device) != hipSuccess ||
      strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
    fail(NK_E_NO_DEVICE, "device %d is %s, this build targets gfx950 only", o.device,
         prop.gcnArchName);
    return nullptr;
  }
  if (hipSetDevice(o.device) != hipSuccess) {
    fail(NK_E_NO_DEVICE, "hipSetDevice(%d) failed", o.device);
    return nullptr;
  }
  nk_counter *c = new nk_counter();
  c->k = k;
  c->pool = pool_size;
  c->thr = threshold;
  c->leak = leak;
  c->refr = refractory;
  c->cost = spike_cost;
  c->canonical = use_canonical ? 1 : 0;
  c->opts = o;
  c->w128 = o.kmer_width == NK_KMER_128;
  c->device = o.device;
  bool ok = hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking) == hipSuccess &&
            hipEventCreateWithFlags(&c->order_ev, hipEventDisableTiming) == hipSuccess;
  // timing-only markers: no system-scope fence (a fenced marker between two
  // kernels writes back L2 and idles the GPU ~2.5 us; tools/syncbench.hip)
  for (int i = 0; ok && i <= kStages; ++i)
    if (i != 1 && i != 2)
      ok = hipEventCreateWithFlags(&c->ev[i], hipEventDisableSystemFence) == hipSuccess;
  for (int i = 0; ok && i < nk_counter::kCountRing; ++i)
    for (int j = 0; ok && j < 2; ++j)
      ok = hipEventCreateWithFlags(&c->cnt_ev[i][j], hipEventDisableSystemFence) == hipSuccess;
  c->ev[1] = c->cnt_ev[0][0];
  c->ev[2] = c->cnt_ev[0][1];
  size_t P = pool_size ? pool_size : 1;
  ok = ok && !c->cur.ensure(P) && !c->sc.ensure(P) && !c->v.ensure(P) && !c->r.ensure(P) &&
       !c->hist.ensure(kHistBins * kHistCopies) && !c->stats.ensure(2) && !c->topst.ensure(1) &&
       !c->cand.ensure(kMaxTopN) && !c->top_cur.ensure(kMaxTopN) &&
       !c->uniq.ensure(kMaxTopN) && !c->special.ensure(kMaxTopN) &&
       !c->top_keys_n.ensure(1) && !c->radix_h.ensure(256) && !c->set_mask_d.ensure(1) &&
       !c->set_need_d.ensure(1) && !c->post_flags.ensure(4) && !c->set_keys.ensure((o.kmer_width == NK_KMER_128 ? 3 : 1) << 20) &&
       !c->n_hits.ensure(1) && !c->span.ensure(2 * nk_counter::kCountRing) &&
       hipHostMalloc((void **)&c->res_h, nk_counter::kResFlagOff + 64,
                     hipHostMallocMapped | hipHostMallocCoherent) == hipSuccess &&
       hipHostGetDevicePointer((void **)&c->res_hd, c->res_h, 0) == hipSuccess;
  c->set_alloc = 1 << 20;
  c->set_dirty = c->set_alloc;  // uninitialised memory
  if (!ok || zero_state(c) != NK_OK) {
    std::string e = g_err.empty() ? "device allocation failed" : g_err;
    nk_free(c);
    fail(NK_E_OOM, "%s", e.c_str());
    return nullptr;
  }
  return c;
}

void nk_free(nk_counter *c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  if (c->last_s) (void)hipStreamSynchronize(c->last_s);
  if (c->own_stream) (void)hipStreamSynchronize(c->own_stream);
  c->cur.release(); c->sc.release(); c->v.release(); c->r.release();
  c->sc8.release(); c->ovf.release();
  c->w_rec.release(); c->w_over.release(); c->w_fill.release();
  c->x_cs.release(); c->xp_keys.release(); c->xp_cnt.release(); c->xp_ctr.release();
  c->xk_off.release(); c->xk_over.release(); c->xk_wrec.release(); c->xk_wover.release();
  c->xk_part.release(); c->xk_fill.release(); c->xk_wfill.release(); c->xk_cur.release();
  c->u_tiles.release(); c->u_nt.release(); c->u_mark.release(); c->u_lanes.release();
  c->p_off.release(); c->p_pos.release(); c->p_fill.release(); c->p_desc.release();
  c->p_over.release(); c->partials.release(); c->tbuckets.release();
  c->bcand.release(); c->bcnt.release();
  c->x_keys.release(); c->x_sorted.release(); c->x_uniq.release(); c->x_q.release();
  c->x_cnt.release(); c->x_tile_rec.release(); c->kpn.release(); c->x_out.release();
  c->x_pres.release(); c->x_tmp.release(); c->x_n.release();
  c->x_ent.release(); c->p_key.release(); c->xg_key.release(); c->xg_key2.release();
  c->xg_side.release(); c->xg_off.release(); c->xg_over.release(); c->xg_cnt.release();
  c->xg_gst.release(); c->xg_trec.release(); c->xg_fill.release(); c->xg_bin2.release();
  c->xg_bctr.release();
  c->d_keys.release(); c->d_meta.release(); c->d_vals.release(); c->touched.release();
  c->tile_rec.release(); c->hist.release(); c->tie_cnt.release(); c->uniq.release();
  c->span.release();
  c->rk_keys.release(); c->rk_idx.release(); c->rk_tmp.release(); c->rk_cand.release();
  c->rk_uniq.release();
  for (PinnedBuf &b : c->ing_hb) b.release();
  c->ing_draw.release();
  c->ing_draw2.release(); c->ing_scratch.release(); c->ing_dst.release();
  if (c->ing_cs) (void)hipStreamSynchronize(c->ing_cs);
  for (hipEvent_t &e : c->ing_ev)
    if (e) (void)hipEventDestroy(e);
  if (c->ing_cs) (void)hipStreamDestroy(c->ing_cs);
  if (c->split_s) (void)hipStreamSynchronize(c->split_s);
  for (hipEvent_t &e : c->split_ev)
    if (e) (void)hipEventDestroy(e);
  if (c->split_s) (void)hipStreamDestroy(c->split_s);
  c->w_snap.release();
  c->special.release(); c->stats.release(); c->lif_tbl.release(); c->topst.release();
  c->cand.release(); c->top_cur.release(); c->set_keys.release(); c->top_keys.release();
  c->top_keys_n.release(); c->radix_h.release(); c->set_mask_d.release();
  c->set_need_d.release(); c->post_flags.release(); c->hits.release(); c->n_hits.release();
  c->trunc_d.release(); c->export_n.release();
  c->mset_keys.release(); c->mset_mask_d.release(); c->muniq.release(); c->mspecial.release();
  if (c->res_h) (void)hipHostFree(c->res_h); c->in_bases.release(); c->in_offs.release();
  for (int i = 0; i <= kStages; ++i)
    if (c->ev[i] && i != 1 && i != 2) (void)hipEventDestroy(c->ev[i]);
  for (auto &pr : c->cnt_ev)
    for (auto &e : pr)
      if (e) (void)hipEventDestroy(e);
  if (c->order_ev) (void)hipEventDestroy(c->order_ev);
  if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
  delete c;
}

int nk_reset(nk_counter *c) {
  if (!c) return fail(NK_E_INVALID, "null counter");
  (void)hipSetDevice(c->device);
  return zero_state(c);
}

int nk_reset_async(nk_counter *c, void *stream) {
  if (!c) return fail(NK_E_INVALID, "null counter");
  (void)hipSetDevice(c->device);
  return zero_state_on(c, pick_stream(c, stream));
}

// ---------------------------------------------------------------------------
// accumulate: currents = histogram of H(kmer) % pool over this input
// ---------------------------------------------------------------------------
// kmer_per_neuron[i] = distinct keys of the table with H(key) % pool == i
// (src/spiking_hash.rs:467-473), from the table's key array (*n_uniq keys of
// wpk words, at most max_n).  The keys are hashed and partitioned exactly like
// the count (k_part_keys, then k_split for pools past 16.7 M, k_bucket_hist
// and one fold into kpn): no global atomic per key.  The per-key atomic kernel
// (k_kpn) took 4.2 ms of an 11.4 ms table build at 113 M keys
// (profiles/r02_s18); it remains only for pools past 2^31.
static int table_kpn(nk_counter *c, const uint64_t *uniq, const unsigned long long *n_uniq,
                     uint64_t max_n, int wpk, hipStream_t s) {
  const uint64_t P = c->pool;
  int rc;
  if ((rc = c->kpn.ensure(std::max<uint64_t>(P, 1)))) return rc;
  if (!P) return NK_OK;
  const char *force = getenv("NK_KPN_ATOMIC");  // tests / A/B: the per-key atomic kernel
  if (!max_n || P > (1ull << 31) || (force && atoi(force))) {
    HIPCHK(hipMemsetAsync(c->kpn.p, 0, P * 4, s));
    if (!max_n) return NK_OK;
    HIPCHK(wpk == 2 ? exact_kpn128(uniq, n_uniq, max_n, P, c->kpn.p, s)
                    : exact_kpn(uniq, n_uniq, max_n, P, c->kpn.p, s));
    return NK_OK;
  }
  const uint64_t B0 = (P + kBinsPerBucket - 1) >> kBinBits;
  const bool wide = B0 > (uint64_t)kMaxBuckets;
  GenPartArgs ga{};
  PartArgs pa{};
  uint64_t B = B0, cap;
  if (wide) {
    int bits = kBinBits;
    while (((P + (1ull << bits) - 1) >> bits) > (uint64_t)kWideMaxBuckets) ++bits;
    const uint64_t C = (P + (1ull << bits) - 1) >> bits;
    // distinct keys hash uniformly: 1.25x the fair share + a tile overflows
    // only in theory (and stays exact: the excess is counted with atomics)
    const uint64_t cap_c = (max_n / C * 5 / 4 + kPartTile + 63) & ~63ull;
    if ((rc = c->xk_wrec.ensure(C * cap_c)) || (rc = c->xk_wfill.ensure(C)) ||
        (rc = c->xk_wover.ensure(C)))
      return rc;
    ga = GenPartArgs{(uint32_t)C, bits, cap_c, c->xk_wrec.p, c->xk_wfill.p, c->xk_wover.p, nullptr};
    B = C << (bits - kBinBits);
    cap = max_n / B * 5 / 4 + 8 * ((cap_c + kPartTile - 1) / kPartTile) + 1024;
    HIPCHK(hipMemsetAsync(c->xk_wfill.p, 0, C * 8, s));
    HIPCHK(hipMemsetAsync(c->xk_wover.p, 0, C * 4, s));
  } else {
    cap = max_n / B * 5 / 4 + kPartTile;
  }
  cap = (cap + 63) & ~63ull;
  const uint32_t slices = (uint32_t)std::max<uint64_t>(1, NK_K1B_WGS / B);
  // xk_cur is zero between calls (k_kpn_fold clears what it read) unless it was
  // (re)allocated (its size grows) or a call failed half-way (xk_cur_zeroed is
  // set again only once the fold is enqueued)
  const size_t clean_n = c->xk_cur_zeroed;
  c->xk_cur_zeroed = 0;
  if ((rc = c->xk_off.ensure(B * cap)) || (rc = c->xk_fill.ensure(B)) || (rc = c->xk_over.ensure(B)) ||
      (rc = c->xk_cur.ensure(P)) || (slices > 1 && (rc = c->xk_part.ensure(slices * P))))
    return rc;
  if (!clean_n || clean_n != c->xk_cur.n) HIPCHK(hipMemsetAsync(c->xk_cur.p, 0, c->xk_cur.n * 8, s));
  HIPCHK(hipMemsetAsync(c->xk_fill.p, 0, B * 8, s));
  HIPCHK(hipMemsetAsync(c->xk_over.p, 0, B * 4, s));
  pa.n_buckets = (uint32_t)B;
  pa.cap = cap;
  pa.off = c->xk_off.p;
  pa.fill = c->xk_fill.p;
  pa.overflow = c->xk_over.p;
  pa.currents = c->xk_cur.p;
  pa.bin_bits = kBinBits;
  if (wide) {
    ga.currents = c->xk_cur.p;
  } else {
    ga = GenPartArgs{(uint32_t)B, kBinBits, cap, c->xk_off.p, c->xk_fill.p, c->xk_over.p, c->xk_cur.p};
  }
  HIPCHK(launch_part_keys(uniq, n_uniq, max_n, wpk, P, ga, wide ? 1 : 0, s));
  if (wide) HIPCHK(launch_split(ga, pa, s));
  HIPCHK(launch_bucket_hist(pa, P, slices, slices > 1 ? c->xk_part.p : nullptr, s));
  HIPCHK(launch_kpn_fold(c->xk_part.p, slices > 1 ? slices : 0, P, c->xk_cur.p, c->kpn.p, s));
  c->xk_cur_zeroed = c->xk_cur.n;
  return NK_OK;
}

// the table as the lookup kernels read it (n null: no table)
static TableView table_view(const nk_counter *c) {
  TableView t{};
  if (!c->exact_built) return t;
  t.uniq = c->x_uniq.p;
  t.cnt = c->x_cnt.p;
  t.n = c->x_n.p + 1;
  if (c->x_grouped) {
    t.ent = c->x_ent.p;
    t.fm = make_fastmod(c->pool);
  }
  return t;
}

// The exact k-mer table of this input sorted by key (nk_exact.h "sorted"
// layout): every key extracted, rocPRIM radix sort + RLE, kmer_per_neuron by
// partition.  One host synchronisation (the key count sizes the sort).  For
// 128-bit keys, k > 32, pools past 16.7 M, inputs past one count batch, and
// the grouped build's fallback.
static int build_sorted(nk_counter *c, const KmerInput &in0, hipStream_t s) {
  int rc;
  // NK_KMER_128: u128 keys (two u64 words each) over their 2k significant bits
  const int w = c->w128 ? 2 : 1;
  const int end_bit = c->w128 ? (int)(2 * c->k) : (c->k <= 32 ? (int)(2 * c->k) : 64);
  KmerInput in = in0;
  in.n_tiles = n_tiles_for(in.n_bases, kTile);
  if ((rc = c->x_n.ensure(8)) || (rc = c->x_tile_rec.ensure(std::max<uint64_t>(in.n_tiles, 1))) ||
      (rc = c->x_keys.ensure(w * std::max<uint64_t>(in.n_bases, 1))) || (rc = c->kpn.ensure(c->pool)))
    return rc;
  in.tile_rec = c->x_tile_rec.p;
  HIPCHK(hipMemsetAsync(c->x_n.p, 0, 16, s));
  HIPCHK(launch_tile_rec(in, kTile, c->x_tile_rec.p, s));
  if (c->w128)
    HIPCHK(exact_keys128(in, (int)c->k, c->canonical, c->x_keys.p, c->x_n.p, s));
  else
    HIPCHK(exact_keys(in, (int)c->k, c->canonical, c->x_keys.p, c->x_n.p, s));
  unsigned long long n = 0;
  HIPCHK(hipMemcpyAsync(&n, c->x_n.p, 8, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  const uint64_t nn = std::max<uint64_t>(n, 1);
  if ((rc = c->x_sorted.ensure(w * nn)) || (rc = c->x_uniq.ensure(w * nn)) ||
      (rc = c->x_cnt.ensure(nn)) ||
      (rc = c->x_tmp.ensure(c->w128 ? exact_temp_bytes128(nn, end_bit) : exact_temp_bytes(nn, end_bit))))
    return rc;
  if (c->w128)
    HIPCHK(exact_sort_rle128(c->x_keys.p, c->x_sorted.p, n, end_bit, c->x_uniq.p, c->x_cnt.p,
                             c->x_n.p + 1, c->x_tmp.p, c->x_tmp.n, s));
  else
    HIPCHK(exact_sort_rle(c->x_keys.p, c->x_sorted.p, n, end_bit, c->x_uniq.p, c->x_cnt.p,
                          c->x_n.p + 1, c->x_tmp.p, c->x_tmp.n, s));
  if ((rc = table_kpn(c, c->x_uniq.p, c->x_n.p + 1, n, w, s))) return rc;
  c->x_grouped = false;
  c->x_lazy = false;
  c->exact_built = true;
  c->kpn_valid = true;
  c->kpn_global = false;
  c->d_dirty = true;  // counts.clear() (src/spiking_hash.rs:157,426)
  c->d_bound = 0;
  return NK_OK;
}

static uint64_t count_chunk(uint64_t n_bases = 0, uint64_t pool = 0, bool wide = false,
                            uint64_t held = 0);
static uint32_t env_u32(const char *name, uint32_t dflt);

// neurons per K1a<KEYS> bucket (log2): kXMinBinBits; NK_XBIN_BITS (A/B,
// 13..15) trades K1a's bucket count against passes per group in k_xgroup
static uint32_t xbin_bits() {
  static const uint32_t b = [] {
    const uint32_t v = env_u32("NK_XBIN_BITS", kXMinBinBits);
    return v < (uint32_t)kXMinBinBits ? (uint32_t)kXMinBinBits : v > (uint32_t)kBinBits ? (uint32_t)kBinBits : v;
  }();
  return b;
}

// The grouped table (nk_table.hip) applies: u64 keys of k <= 32, a pool the
// partitioned count covers, one count batch, and few enough keys per neuron
// for a group's distinct keys to fit the LDS table.  NK_EXACT_SORT=1 (tests,
// A/B) takes the sorted build.
static bool grouped_ok(const nk_counter *c, uint64_t n_bases) {
  if (c->w128 || c->k > 32 || !c->pool || !n_bases) return false;
  const char *e = getenv("NK_EXACT_SORT");
  if (e && atoi(e)) return false;
  if (((c->pool + kBinsPerBucket - 1) >> kBinBits) > (uint64_t)kMaxBuckets) return false;
  if (n_bases > count_chunk()) return false;
  return xgroup_fits(n_bases, c->pool, xgroup_bits(n_bases, c->pool));
}

// side list capacity: records that leave the grouped path (overflowed K1a
// regions, groups with too many distinct keys); past it the sorted build runs
static uint64_t side_cap_for(uint64_t n_bases) {
  const uint64_t e = env_u32("NK_XSIDE_CAP", 0);
  return e ? e : std::max<uint64_t>(n_bases / 8, 1ull << 20);
}

// the K1a<KEYS> arguments whose records feed the grouped table: the key
// array (the count's p_key, or the table's own) and the side list
static int keyed_args(nk_counter *c, uint64_t n_bases, PartArgs &pa, bool own, hipStream_t s) {
  int rc;
  const uint64_t sc = side_cap_for(n_bases);
  DevBuf<uint64_t> &kb = own ? c->xg_key : c->p_key;
  if ((rc = c->x_n.ensure(8)) || (rc = c->xg_side.ensure(sc)) ||
      (rc = kb.ensure((uint64_t)pa.n_buckets * pa.cap)))
    return rc;
  HIPCHK(hipMemsetAsync(c->x_n.p + 5, 0, 8, s));  // [5] side records
  pa.key = kb.p;
  pa.spill = c->xg_side.p;
  pa.n_spill = c->x_n.p + 5;
  pa.spill_cap = sc;
  return NK_OK;
}

// The grouped table from the keyed records of a K1a<KEYS> pass: the count's
// own (keyed: its PartArgs) or, without one, a K1a<KEYS> pass of the table's
// own over the input (no currents touched).  One host synchronisation (the
// side list's size); the sorted build when the side list overflowed.
static int build_grouped(nk_counter *c, const KmerInput &in0, const PartArgs *keyed, hipStream_t s) {
  int rc;
  const uint64_t P = c->pool, n_bases = in0.n_bases;
  PartArgs pa{};
  if (keyed) {
    pa = *keyed;
  } else {
    uint32_t bits = xbin_bits();
    while (bits < kBinBits && ((P + (1ull << bits) - 1) >> bits) > 256) ++bits;
    const uint64_t B = (P + (1ull << bits) - 1) >> bits;
    pa.n_buckets = (uint32_t)B;
    // 1.25x the fair share + the 8-record padding of each (tile, bucket) segment
    pa.cap = ((n_bases / B * 5 / 4 + kPartTile + 4 * n_tiles_for(n_bases, kPartTile)) + 63) & ~63ull;
    pa.bin_bits = bits;
    KmerInput in = in0;
    in.n_tiles = n_tiles_for(n_bases, kPartTile);
    if ((rc = c->xg_off.ensure(B * pa.cap)) || (rc = c->xg_fill.ensure(B)) ||
        (rc = c->xg_over.ensure(B)) || (rc = c->xg_trec.ensure(std::max<uint64_t>(in.n_tiles, 1))))
      return rc;
    pa.off = c->xg_off.p;
    pa.fill = c->xg_fill.p;
    pa.overflow = c->xg_over.p;
    pa.currents = nullptr;  // the table only: the currents are the count's
    if ((rc = keyed_args(c, n_bases, pa, /*own=*/true, s))) return rc;
    in.tile_rec = c->xg_trec.p;
    HIPCHK(hipMemsetAsync(c->xg_fill.p, 0, B * 8, s));
    HIPCHK(hipMemsetAsync(c->xg_over.p, 0, B * 4, s));
    HIPCHK(launch_tile_rec(in, kPartTile, c->xg_trec.p, s));
    HIPCHK(launch_part(in, (int)c->k, c->canonical, P, pa, s));
  }
  XGroupArgs t{};
  t.n_buckets = pa.n_buckets;
  t.cap = pa.cap;
  t.bin_bits = pa.bin_bits;
  t.off = pa.off;
  t.key = pa.key;
  t.fill = pa.fill;
  t.overflow = pa.overflow;
  t.gbits = xgroup_bits(n_bases, P);
  t.ggbits = xgroup_group_bits(t.gbits, pa.bin_bits);
  t.n_groups = 1u << (pa.bin_bits - t.ggbits);
  t.n_slices = (uint32_t)((pa.cap + kXSlice - 1) / kXSlice);
  const uint64_t B = pa.n_buckets, slots = B * pa.cap;
  const uint64_t n_tab = std::max<uint64_t>(n_bases, 1) + pa.spill_cap;  // grouped span + side part
  if ((rc = c->xg_cnt.ensure(B * t.n_slices * t.n_groups)) ||
      (rc = c->xg_gst.ensure(B * (t.n_groups + 1))) || (rc = c->xg_key2.ensure(slots)) ||
      (rc = c->xg_bin2.ensure(slots)) || (rc = c->xg_bctr.ensure(2 * B)) ||
      (rc = c->x_uniq.ensure(n_tab)) || (rc = c->x_cnt.ensure(n_tab)) ||
      (rc = c->x_ent.ensure(P)) || (rc = c->kpn.ensure(P)))
    return rc;
  t.xcnt = c->xg_cnt.p;
  t.gstart = c->xg_gst.p;
  t.key2 = c->xg_key2.p;
  t.bin2 = c->xg_bin2.p;
  t.side = pa.spill;
  t.n_side = pa.n_spill;
  t.side_cap = pa.spill_cap;
  t.pool = P;
  t.uniq = c->x_uniq.p;
  t.cnt = c->x_cnt.p;
  t.bbase = c->xg_bctr.p;
  t.bdist = c->xg_bctr.p + B;
  t.span = c->x_n.p + 4;
  t.ent = c->x_ent.p;
  t.kpn = c->kpn.p;
  t.hash_max = env_u32("NK_XHASH_MAX", 0);
  t.hash_bits = xgroup_hash_bits();
  HIPCHK(xgroup_build(t, s));
  unsigned long long cnt[2] = {0, 0};  // grouped span, side records
  HIPCHK(hipMemcpyAsync(cnt, c->x_n.p + 4, 16, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  if (cnt[1] > t.side_cap) return build_sorted(c, in0, s);
  if (cnt[1]) {  // the side part: sorted, run-length encoded after the grouped span
    const int end_bit = (int)(2 * c->k);
    if ((rc = c->x_sorted.ensure(cnt[1])) || (rc = c->x_tmp.ensure(exact_temp_bytes(cnt[1], end_bit))))
      return rc;
    HIPCHK(exact_sort_rle(t.side, c->x_sorted.p, cnt[1], end_bit, c->x_uniq.p + cnt[0],
                          c->x_cnt.p + cnt[0], c->x_n.p + 3, c->x_tmp.p, c->x_tmp.n, s));
    HIPCHK(exact_kpn(c->x_uniq.p + cnt[0], c->x_n.p + 3, cnt[1], P, c->kpn.p, s));
    HIPCHK(xgroup_finish(t, c->x_n.p + 1, c->x_n.p + 3, s));
  } else {
    HIPCHK(xgroup_finish(t, c->x_n.p + 1, nullptr, s));
  }
  c->x_grouped = true;
  c->x_lazy = false;
  c->exact_built = true;
  c->kpn_valid = true;
  c->kpn_global = false;
  c->d_dirty = true;  // counts.clear() (src/spiking_hash.rs:157,426)
  c->d_bound = 0;
  return NK_OK;
}

// The exact k-mer table of this input (opts.exact_counts; nk_exact.h):
// grouped by neuron where it applies (keyed: the count's K1a<KEYS> records of
// this input), else sorted by key.
static int build_exact(nk_counter *c, const KmerInput &in, hipStream_t s,
                       const PartArgs *keyed = nullptr) {
  if (keyed || grouped_ok(c, in.n_bases)) return build_grouped(c, in, keyed, s);
  return build_sorted(c, in, s);
}

// A process/accumulate call replaces `counts` and `kmer_per_neuron` with its
// input's (src/spiking_hash.rs:157-172,426-427,467-473): built now with
// opts.exact_counts, else marked to be built from that input on demand.
static int table_for_input(nk_counter *c, const KmerInput &in, hipStream_t s,
                           const PartArgs *keyed = nullptr) {
  if (c->opts.exact_counts) return build_exact(c, in, s, keyed);
  c->exact_built = false;
  c->kpn_valid = false;
  c->kpn_global = false;
  c->d_dirty = true;
  c->d_bound = 0;
  c->x_lazy = true;
  return NK_OK;
}

// The table on demand (no opts.exact_counts): built from the last input, which
// must still be resident.  Device input passed by pointer is the caller's and
// may be gone: such a handle needs opts.exact_counts (eager build).
static int ensure_table(nk_counter *c, hipStream_t s) {
  if (!c->x_lazy) return NK_OK;
  if (!c->input_owned)
    return fail(NK_E_UNSUPPORTED,
                "the last input was device memory of the caller (not kept by the handle): "
                "set nk_opts.exact_counts = 1 for counts / kmer_per_neuron / rows past top_n");
  return build_exact(c, c->last_in, s);
}

// How one count batch runs:
//   Part   k <= 32 keys, pool <= 16.7 M: k_part (rolled keys) + k_bucket_hist;
//          the records are kept for the uniques scan
//   Gen    k > 32 compat / 128-bit keys, pool <= 16.7 M: k_part_gen (narrow)
//          + k_bucket_hist
//   Wide   pool <= 2^31, k <= 64: k_part_gen (coarse) + k_split + k_bucket_hist
//   Atomic the direct-atomic kernels (k > 64 compat keys, pool > 2^31)
enum class CountPath { Atomic, Part, Gen, Wide };
struct CountPlan {
  CountPath path = CountPath::Atomic;
  int km = 0;               // key mode of k_part_gen
  uint64_t tile = kTile;
  uint32_t slices = 0;      // K1b slices (Part, or > 1: partials; else adds into cur)
  PartArgs pa{};            // the 32768-bin buckets k_bucket_hist reads
  GenPartArgs ga{};         // Gen: same arrays as pa; Wide: the coarse buckets
};

// tests: NK_WIDE_BITS=b forces the wide path with coarse buckets of 2^b bins
static int wide_bits_forced() {
  const char *e = getenv("NK_WIDE_BITS");
  return e ? atoi(e) : 0;
}

// tests: NK_FORCE_ATOMIC=1 forces the direct-atomic count kernels (k_kmers,
// k_kmers_compat, k_kmers128), which otherwise run only past the partitions
static bool atomic_forced() {
  const char *e = getenv("NK_FORCE_ATOMIC");
  return e && atoi(e) != 0;
}

// Positions counted per partition launch.  An input up to this size keeps its
// records (4-5 B per k-mer; 7.5 B on the wide path) for the uniques scan,
// which then reads only the top rows' buckets; a larger one is counted in
// batches whose records are histogrammed and dropped batch by batch, and the
// top rows' uniques come from a rescan of the WHOLE input (a full re-hash:
// ~115 ms of a 166 ms step at a 12.5 Gbase config-4 shard, profiles/r04_side).
// So an input past the default batch is counted in ONE launch whenever its
// arena fits in kKeepFrac of the free HBM (a 12.5 Gbase shard: ~63 GB Part,
// ~95 GB wide, of 288 GB); batches remain for inputs that do not fit.
// NK_COUNT_CHUNK (tests) forces a batch size, rounded to whole tiles.
#ifndef NK_COUNT_CHUNK_DEFAULT
#define NK_COUNT_CHUNK_DEFAULT (1ull << 31)
#endif
constexpr double kKeepFrac = 0.6;
// (pool: a bucket region of one launch stays below 2^31 records, so K1b's u32
// bins and partials cannot wrap whatever the input; held: the arena bytes
// this handle already holds, free for it to reuse -- without them a handle's
// second count of the same input measured its own arena as taken and fell
// back to batches, profiles/r04_t3)
static uint64_t count_chunk(uint64_t n_bases, uint64_t pool, bool wide, uint64_t held) {
  const char *e = getenv("NK_COUNT_CHUNK");
  uint64_t v = e ? strtoull(e, nullptr, 10) : 0;
  if (!v) {
    v = NK_COUNT_CHUNK_DEFAULT;
    const uint64_t B = std::max<uint64_t>(1, (pool + kBinsPerBucket - 1) >> kBinBits);
    // arena bytes per position: Part u16 offset + u16 position; Gen/Wide u32
    // coarse + u16 fine records; x1.25 region slack, + segment descriptors
    const double per = (wide || B > (uint64_t)kMaxBuckets) ? 8.5 : 5.5;
    size_t fr = 0, tot = 0;
    if (n_bases > v && pool && n_bases / B * 5 / 4 < (1ull << 31) - (1ull << 24) &&
        !getenv("NK_COUNT_BATCHED") && hipMemGetInfo(&fr, &tot) == hipSuccess &&
        (double)n_bases * per <= kKeepFrac * (double)(fr + held))
      v = (n_bases + kPartTile - 1) / kPartTile * kPartTile;
  }
  return std::max<uint64_t>(kPartTile, v / kPartTile * kPartTile);
}

// device bytes of the partition arena this handle holds (reused by a count)
static uint64_t arena_bytes(const nk_counter *c) {
  return c->p_off.n * 2 + c->p_pos.n * 2 + c->p_desc.n * 8 + c->w_rec.n * 4;
}

// Sizes the buffers for a batch of about est_bases bases (slack: extra
// records per bucket region; max_segs: Part's descriptors per bucket) and
// lists the arrays to zero before the first batch.
// part_bits: the narrowest Part buckets to try (the exact table's K1a<KEYS>
// count takes 4096-neuron buckets, up to 512 of them: nk_table.hip)
static int plan_count(nk_counter *c, uint64_t est_bases, uint64_t slack, uint64_t max_segs,
                      CountPlan &cp, ZeroList &z, bool keep_gen = false, int part_bits = 0) {
  cp = CountPlan{};
  const uint64_t P = c->pool;
  if (!P) return NK_OK;
  const int k = (int)c->k;
  uint64_t B = (P + kBinsPerBucket - 1) >> kBinBits;
  cp.km = c->w128 ? 2 : (k > 32 ? 1 : 0);
  const bool keys_ok = cp.km == 0 || k <= 64;
  const bool wide_ok = keys_ok && P <= (1ull << 31);
  const int forced = wide_bits_forced();
  if (atomic_forced()) return NK_OK;  // tests: the direct-atomic kernels at any size
  if (forced > 0 && wide_ok) cp.path = CountPath::Wide;
  else if (cp.km == 0 && B <= (uint64_t)kMaxBuckets) cp.path = CountPath::Part;
  else if (keys_ok && B <= (uint64_t)kMaxBuckets) cp.path = CountPath::Gen;
  else if (wide_ok) cp.path = CountPath::Wide;
  if (cp.path == CountPath::Atomic) return NK_OK;
#ifndef NK_PART_MIN_BITS
#define NK_PART_MIN_BITS 15  // A/B: 13 (245 buckets at P = 2 M) costs K1a +20 us and the histogram +20 us
#endif
  int pbits = kBinBits;
  if (cp.path == CountPath::Part) {
    // bucket width: the narrowest from NK_PART_MIN_BITS that fits K1a's 256
    // bucket counters.  Narrower buckets would need no histogram slices and a
    // shorter uniques scan, but measured slower overall (more K1a segments and
    // reservations, hotter LDS histogram bins): the default keeps 32768 bins
    pbits = part_bits ? part_bits : NK_PART_MIN_BITS;
    while (pbits < kBinBits && ((P + (1ull << pbits) - 1) >> pbits) > 256) ++pbits;
    B = (P + (1ull << pbits) - 1) >> pbits;
  }
  cp.tile = kPartTile;
  const uint64_t est = std::max<uint64_t>(est_bases, 1);
  int rc;
  uint64_t cap;
  if (cp.path == CountPath::Wide) {
    int bits = kBinBits;
    while (((P + (1ull << bits) - 1) >> bits) > (uint64_t)kWideMaxBuckets) ++bits;
    if (forced > bits) bits = std::min(forced, kBinBits + kMaxSplitBits);
    const uint64_t C = (P + (1ull << bits) - 1) >> bits;
    uint64_t cap_c = est / C * 5 / 4 + slack;
    cap_c = (cap_c + 63) & ~63ull;
    if ((rc = c->w_rec.ensure(C * cap_c)) || (rc = c->w_fill.ensure(C)) || (rc = c->w_over.ensure(C)))
      return rc;
    cp.ga = GenPartArgs{(uint32_t)C, bits, cap_c, c->w_rec.p, c->w_fill.p, c->w_over.p,
                        (unsigned long long *)c->cur.p};
    z.ptr[z.n] = c->w_fill.p; z.bytes[z.n++] = C * 8;
    z.ptr[z.n] = c->w_over.p; z.bytes[z.n++] = C * 4;
    // a fine bucket takes up to 7 pad records per split tile of its coarse bucket
    cap = est / B * 5 / 4 + 8 * ((cap_c + kPartTile - 1) / kPartTile) + 1024;
  } else {
    cap = est / B * 5 / 4 + slack;
    // narrow buckets: K1a pads each (tile, bucket) segment to 8 records, ~3.5
    // records per tile (at 245 buckets about 10 % of the records)
    if (part_bits) cap += 4 * n_tiles_for(est, kPartTile);
  }
  cap = (cap + 63) & ~63ull;
  // one round of 1-per-CU workgroups (128 KiB LDS each) on 256 CUs
  cp.slices = (uint32_t)std::max<uint64_t>(1, NK_K1B_WGS / B);
  if ((rc = c->p_off.ensure(B * cap)) || (rc = c->p_fill.ensure(B)) || (rc = c->p_over.ensure(B)) ||
      ((cp.path == CountPath::Part || cp.slices > 1) && (rc = c->partials.ensure(cp.slices * P))))
    return rc;
  PartArgs &pa = cp.pa;
  pa.n_buckets = (uint32_t)B;
  pa.cap = cap;
  pa.off = c->p_off.p;
  pa.fill = c->p_fill.p;
  pa.overflow = c->p_over.p;
  pa.currents = (unsigned long long *)c->cur.p;
  pa.bin_bits = (uint32_t)pbits;
  if (cp.path == CountPath::Part) {
    if ((rc = c->p_pos.ensure(B * cap)) || (rc = c->p_desc.ensure(B * max_segs))) return rc;
    pa.pos = c->p_pos.p;
    pa.desc = c->p_desc.p;
    pa.max_segs = max_segs;
  }
  if (cp.path == CountPath::Gen)
    cp.ga = GenPartArgs{(uint32_t)B, kBinBits, cap, c->p_off.p, c->p_fill.p, c->p_over.p,
                        (unsigned long long *)c->cur.p};
  if (keep_gen && (cp.path == CountPath::Gen || cp.path == CountPath::Wide)) {
    // segment descriptors of k_part_gen's buckets (coarse ones when wide)
    if ((rc = c->p_desc.ensure((uint64_t)cp.ga.n_buckets * max_segs))) return rc;
    cp.ga.desc = c->p_desc.p;
    cp.ga.max_segs = max_segs;
    cp.ga.lane_tag = (cp.path == CountPath::Wide && cp.ga.bin_bits <= kLaneTagMaxBits &&
                      !getenv("NK_NO_LANE_TAG")) ? 1u : 0u;
  }
  z.ptr[z.n] = c->p_fill.p; z.bytes[z.n++] = B * 8;
  z.ptr[z.n] = c->p_over.p; z.bytes[z.n++] = B * 4;
  return NK_OK;
}

// K1b of a Gen/Wide batch: partials (several slices per bucket) or straight
// into the currents
static hipError_t gen_hist(nk_counter *c, const CountPlan &cp, bool defer_partials, hipStream_t s) {
  if (cp.slices > 1) {
    hipError_t e = launch_bucket_hist(cp.pa, c->pool, cp.slices, c->partials.p, s);
    if (e != hipSuccess) return e;
    if (defer_partials) {
      c->pend_slices = cp.slices;
      return hipSuccess;
    }
    return launch_partials_add(c->partials.p, cp.slices, c->pool, c->cur.p, s);
  }
  return launch_bucket_hist(cp.pa, c->pool, 1, nullptr, s);
}

// k_part_gen launches of a pipelined wide count: G launches of at least
// kSplitMinTiles tiles each (NK_SPLIT_LAUNCHES: tests / A/B; 1 = one launch,
// the split after it)
constexpr uint64_t kSplitMinTiles = 2048;
static uint32_t split_launches(uint64_t n_tiles) {
  const char *e = getenv("NK_SPLIT_LAUNCHES");
  uint64_t g = e ? strtoull(e, nullptr, 10) : std::min<uint64_t>(16, n_tiles / kSplitMinTiles);
  g = std::min<uint64_t>(std::min<uint64_t>(g, nk_counter::kSplitMax), n_tiles);
  return (uint32_t)std::max<uint64_t>(g, 1);
}

// The wide count with its split pipelined: k_part_gen is VALU-bound (SipHash)
// and k_split is bound by its bytes, so the input's tiles go in G launches on
// s and the split of launch g's records (each coarse bucket's records reserved
// between the fill snapshots after launches g - 1 and g) runs on split_s while
// launch g + 1 hashes.  s waits for the last split before K1b.
static hipError_t split_pipelined(nk_counter *c, const CountPlan &cp, const KmerInput &in, uint32_t G,
                                  hipStream_t s) {
  hipError_t e;
  if (!c->split_s) {
    if ((e = hipStreamCreateWithFlags(&c->split_s, hipStreamNonBlocking)) != hipSuccess) return e;
    for (hipEvent_t &ev : c->split_ev)
      if ((e = hipEventCreateWithFlags(&ev, hipEventDisableTiming)) != hipSuccess) return e;
  }
  const uint64_t nb = cp.ga.n_buckets;
  if (c->w_snap.ensure(G * nb)) return hipErrorOutOfMemory;
  const uint64_t per = (in.n_tiles + G - 1) / G;
  const bool wide = true;
  uint32_t g = 0;
  for (uint64_t t0 = 0; t0 < in.n_tiles; t0 += per, ++g) {
    KmerInput bi = in;
    bi.tile_base = in.tile_base + t0;
    bi.tile_rec = in.tile_rec + t0;
    bi.n_tiles = std::min<uint64_t>(per, in.n_tiles - t0);
    unsigned long long *hi = c->w_snap.p + (uint64_t)g * nb;
    if ((e = launch_part_gen(bi, (int)c->k, c->canonical, cp.km, c->pool, cp.ga, wide ? 1 : 0, s)) ||
        (e = launch_fill_snap(cp.ga, hi, s)) || (e = hipEventRecord(c->split_ev[g], s)) ||
        (e = hipStreamWaitEvent(c->split_s, c->split_ev[g], 0)) ||
        (e = launch_split(cp.ga, cp.pa, c->split_s, g ? hi - nb : nullptr, hi, bi.n_tiles * kPartTile)))
      return e;
  }
  if ((e = hipEventRecord(c->split_ev[nk_counter::kSplitMax], c->split_s))) return e;
  return hipStreamWaitEvent(s, c->split_ev[nk_counter::kSplitMax], 0);
}

// Gen/Wide count kernels of one batch (before K1b)
static hipError_t gen_count(nk_counter *c, const CountPlan &cp, const KmerInput &in, hipStream_t s,
                            bool pipeline = false) {
  const bool wide = cp.path == CountPath::Wide;
  if (wide && pipeline) {
    const uint32_t G = split_launches(in.n_tiles);
    if (G > 1) return split_pipelined(c, cp, in, G, s);
  }
  hipError_t e = launch_part_gen(in, (int)c->k, c->canonical, cp.km, c->pool, cp.ga, wide ? 1 : 0, s);
  if (e != hipSuccess || !wide) return e;
  return launch_split(cp.ga, cp.pa, s);
}

// One batch whose records are not kept (Gen/Wide always; Part past
// count_chunk()): count, histogram into the currents, empty the regions for
// the next batch.
static hipError_t batch_count(nk_counter *c, const CountPlan &cp, const KmerInput &in, hipStream_t s) {
  hipError_t e = cp.path == CountPath::Part
                     ? launch_part(in, (int)c->k, c->canonical, c->pool, cp.pa, s)
                     : gen_count(c, cp, in, s);
  if (e == hipSuccess) e = gen_hist(c, cp, false, s);
  if (e != hipSuccess) return e;
  ZeroList z{};
  z.ptr[z.n] = cp.pa.fill; z.bytes[z.n++] = (uint64_t)cp.pa.n_buckets * 8;
  if (cp.path == CountPath::Wide) {
    z.ptr[z.n] = cp.ga.fill; z.bytes[z.n++] = (uint64_t)cp.ga.n_buckets * 8;
  }
  return launch_zero(z, s);
}

// a positive integer from the environment (tests: force the rare branches)
static uint32_t env_u32(const char *name, uint32_t dflt) {
  const char *e = getenv(name);
  const unsigned long v = e ? strtoul(e, nullptr, 10) : 0;
  return v ? (uint32_t)v : dflt;
}

// defer_partials: leave K1c (currents += partials) to the LIF kernel of the
// same process call instead of a separate pass
static bool top_fused(const nk_counter *c, uint64_t want);
static LifParams lif_params(const nk_counter *c, int streaming);
static int lif_table(nk_counter *c, const LifParams &lp, hipStream_t s);

static int accumulate(nk_counter *c, const uint8_t *d_bases, const uint64_t *d_offs,
                      size_t n_recs, size_t n_bases, void *stream, bool defer_partials,
                      uint64_t first_pos = 0) {
  if (!c) return fail(NK_E_INVALID, "null counter");
  if (n_bases && ((uintptr_t)d_bases & 15))
    return fail(NK_E_INVALID, "device bases must be 16-byte aligned");
  if (n_bases && !n_recs) return fail(NK_E_INVALID, "bases without records");
  if (c->pool == 0 && n_bases >= c->k)
    return fail(NK_E_INVALID, "pool_size 0 with k-mers present (the reference panics on % 0)");
  (void)hipSetDevice(c->device);
  hipStream_t s = pick_stream(c, stream);
  // a derived state is a function of the counts this call replaces
  if (int rc0 = settle_state(c, s)) return rc0;
  c->pend_slices = 0;  // this call zeroes the currents: earlier partials are void
  c->cur_in_wire = false;
  c->k1b_lif = false;
  c->export_pending = c->redo_ready = false;
  KmerInput in{};
  in.bases = d_bases;
  in.offsets = d_offs;
  in.n_recs = n_recs;
  in.n_bases = n_bases;
  in.pos_lo = first_pos;
  // one prep kernel: tile -> first record index, and every buffer the count
  // (and, for a process call, the LIF) accumulates into zeroed
  ZeroList z{};
  CountPlan cp;
  // bucket regions: 1.25x the fair share + one tile of slack (overflow is
  // still exact: the excess is counted with direct atomics); past
  // count_chunk() positions the regions hold one batch at a time
  uint64_t chunk = count_chunk(n_bases, c->pool, c->w128 || c->k > 32, arena_bytes(c));
  uint64_t est = std::min<uint64_t>(n_bases, chunk);
  // the exact table grouped by neuron from this count's own records (K1a also
  // writes each record's key, nk_table.hip), in 4096-neuron buckets
  const bool want_keyed = c->opts.exact_counts && grouped_ok(c, n_bases);
  int rc = plan_count(c, est, kPartTile, n_tiles_for(est, kPartTile), cp, z,
                     /*keep_gen=*/n_bases <= chunk, want_keyed ? xbin_bits() : 0);
  if (rc == NK_E_OOM && chunk > count_chunk()) {
    // the one-launch arena did not fit after all (other handles took the
    // memory since the estimate): count in batches instead
    z = ZeroList{};
    chunk = count_chunk();
    est = std::min<uint64_t>(n_bases, chunk);
    rc = plan_count(c, est, kPartTile, n_tiles_for(est, kPartTile), cp, z, n_bases <= chunk,
                    want_keyed ? xbin_bits() : 0);
  }
  if (rc) return rc;
  in.n_tiles = n_tiles_for(n_bases, cp.tile);
  const bool batched = cp.path != CountPath::Atomic && n_bases > chunk;
  const uint64_t batch_tiles = chunk / kPartTile;  // cp.tile == kPartTile on the partitioned paths
  // Gen/Wide with one K1b workgroup per bucket and one batch: K1b writes every
  // bin of the currents (write-through), so they are neither zeroed nor read;
  // region overflow goes to the kept-zero ovf array, which K1b folds back
  const bool wt = !batched && (cp.path == CountPath::Gen || cp.path == CountPath::Wide) &&
                  cp.slices == 1 && in.n_tiles > 0 && !getenv("NK_NO_WRITE_THROUGH");
  if (wt) {
    if (c->ovf.n < c->pool || c->ovf_zeroed < c->pool) {
      if ((rc = c->ovf.ensure(c->pool))) return rc;
      HIPCHK(hipMemsetAsync(c->ovf.p, 0, c->pool * 8, s));
      c->ovf_zeroed = c->pool;
    }
    cp.pa.currents = cp.ga.currents = c->ovf.p;
    cp.pa.out = (unsigned long long *)c->cur.p;
    // from the reset state with the hist/stats zeroed by this prep (a split
    // accumulate or a process call) and a finish that does not fuse its top-N
    // into the LIF kernel: K1b runs the LIF too (a function of the counts)
    const uint64_t want = std::min<uint64_t>(c->opts.top_n, c->pool);
    if (defer_partials && c->state_fresh && !top_fused(c, want) && c->pool &&
        !getenv("NK_NO_K1B_LIF")) {
      const LifParams lp = lif_params(c, 0 /* skip_zero: the in-memory finish */);
      if ((rc = lif_table(c, lp, s)) || (rc = c->sc8.ensure(c->pool))) return rc;
      cp.pa.lif.sc8 = c->sc8.p;
      cp.pa.lif.tbl = c->lif_tbl.p;
      cp.pa.lif.tbl_n = kLifTable;
      cp.pa.lif.lp = lp;
      cp.pa.lif.hist = c->hist.p;
      cp.pa.lif.stats = (unsigned long long *)c->stats.p;
      c->k1b_lif = true;
      c->k1b_lp = lp;
    }
    if (cp.path == CountPath::Wide) {
      cp.pa.over_coarse = cp.ga.overflow;
      cp.pa.coarse_shift = (uint32_t)(cp.ga.bin_bits - kBinBits);
    }
  } else {
    z.ptr[z.n] = c->cur.p; z.bytes[z.n++] = c->pool * 8;
  }
  if ((rc = c->tile_rec.ensure(std::max<uint64_t>(batched ? batch_tiles : in.n_tiles, 1)))) return rc;
  in.tile_rec = c->tile_rec.p;
  const bool counted = cp.path != CountPath::Atomic && in.n_tiles > 0;
  if (count_timing(c)) {  // level 2 records no count-kernel events
    const int slot = (int)(c->cnt_calls++ % nk_counter::kCountRing);
    c->ev[1] = c->cnt_ev[slot][0];
    c->ev[2] = c->cnt_ev[slot][1];
  }
  if (batched) {
    // prep (the zero list) with the first batch's tile index, then batch by
    // batch; the records are dropped, so the uniques pass rescans the input
    if (defer_partials) {
      z.ptr[z.n] = c->hist.p;  z.bytes[z.n++] = kHistBins * kHistCopies * 4;
      z.ptr[z.n] = c->stats.p; z.bytes[z.n++] = 16;
      c->lif_zeroed = true;
    }
    HIPCHK(mark(c, 0, s));
    for (uint64_t t0 = 0; t0 < in.n_tiles; t0 += batch_tiles) {
      KmerInput bi = in;
      bi.tile_base = t0;
      bi.n_tiles = std::min<uint64_t>(batch_tiles, in.n_tiles - t0);
      if (t0 == 0) {
        HIPCHK(launch_prep(bi, cp.tile, c->tile_rec.p, z, s));
        HIPCHK(mark(c, 1, s));
      } else {
        HIPCHK(launch_tile_rec(bi, cp.tile, c->tile_rec.p, s));
      }
      HIPCHK(batch_count(c, cp, bi, s));
    }
    HIPCHK(mark(c, 2, s));
    c->cur_fresh = false;
    c->part_used = false;
    c->gen_keep = false;
    c->gen_km = cp.path == CountPath::Part ? -1 : cp.km;
    c->pend_slices = 0;
    HIPCHK(mark(c, 3, s));
    c->last_in = in;
    c->have_input = true;
    c->top_valid = false;
    c->input_owned = d_bases == c->in_bases.p;
    return table_for_input(c, in, s);
  }
  c->part_used = counted && cp.path == CountPath::Part;
  c->gen_km = (cp.path == CountPath::Gen || cp.path == CountPath::Wide) ? cp.km : -1;
  c->gen_keep = counted && c->gen_km >= 0 && cp.ga.desc && !getenv("NK_NO_GEN_KEEP");
  c->gen_wide = cp.path == CountPath::Wide;
  c->last_ga = cp.ga;
  if (cp.path == CountPath::Part && c->set_dirty && !c->w128 && z.n < kZeroMax) {
    // the uniques set, empty for this input's scan (k_uniq_scan inserts as it goes)
    z.ptr[z.n] = c->set_keys.p; z.bytes[z.n] = c->set_dirty * 8; z.fill[z.n++] = 0xFF;
    c->set_dirty = 0;
    c->set_clean = true;
  } else if (cp.path == CountPath::Part && !c->set_dirty) {
    c->set_clean = true;
  }
  if (defer_partials) {  // the LIF of this process call accumulates into these
    z.ptr[z.n] = c->hist.p;  z.bytes[z.n++] = kHistBins * kHistCopies * 4;
    z.ptr[z.n] = c->stats.p; z.bytes[z.n++] = 16;
    c->lif_zeroed = !c->k1b_lif;  // (K1b adds into them: a LIF that runs after all re-zeroes)
  }
  unsigned long long *span = nullptr;
  if (c->part_used) {
    span = c->span.p + 2 * (c->span_calls++ % nk_counter::kCountRing);
    cp.pa.span = span;
  }
  const bool keyed = c->part_used && want_keyed;
  if (keyed && (rc = keyed_args(c, n_bases, cp.pa, /*own=*/false, s))) return rc;
  HIPCHK(mark(c, 0, s));
  HIPCHK(launch_prep(in, cp.tile, c->tile_rec.p, z, s, span));
  c->cur_fresh = false;
  HIPCHK(mark(c, 1, s));
  if (c->part_used) {
    HIPCHK(launch_part(in, (int)c->k, c->canonical, c->pool, cp.pa, s));
    HIPCHK(mark(c, 2, s));
    HIPCHK(launch_bucket_hist(cp.pa, c->pool, cp.slices, c->partials.p, s));
    if (defer_partials)
      c->pend_slices = cp.slices;
    else
      HIPCHK(launch_partials_add(c->partials.p, cp.slices, c->pool, c->cur.p, s));
    c->last_pa = cp.pa;
  } else if (counted) {
    HIPCHK(gen_count(c, cp, in, s, /*pipeline=*/true));
    HIPCHK(mark(c, 2, s));
    HIPCHK(gen_hist(c, cp, defer_partials, s));
  } else {
    if (c->w128)
      HIPCHK(launch_count128(in, (int)c->k, c->canonical, c->pool, c->cur.p, s));
    else
      HIPCHK(launch_count(in, (int)c->k, c->canonical, c->pool, c->cur.p, s));
    HIPCHK(mark(c, 2, s));
  }
  HIPCHK(mark(c, 3, s));
  c->last_in = in;
  c->have_input = true;
  c->top_valid = false;
  c->input_owned = d_bases == c->in_bases.p;
  if ((rc = table_for_input(c, in, s, keyed ? &cp.pa : nullptr))) return rc;
  return NK_OK;
}

// The split entry points (a finish usually follows on another stream: the
// multi-GPU step, or batches in flight on two handles) mark their end for the
// next call's pick_stream.
int nk_accumulate_device(nk_counter *c, const uint8_t *d_bases, const uint64_t *d_offs,
                         size_t n_recs, size_t n_bases, void *stream) {
  // the partials stay pending: nk_finalize's LIF (or nk_wire32) folds them,
  // nk_device_currents / nk_copy_currents fold them first
  const int rc = accumulate(c, d_bases, d_offs, n_recs, n_bases, stream, true);
  if (!rc) record_order(c, c->last_s);
  return rc;
}

int nk_accumulate_device_from(nk_counter *c, const uint8_t *d_bases, const uint64_t *d_offs,
                              size_t n_recs, size_t n_bases, size_t first_pos, void *stream) {
  const int rc = accumulate(c, d_bases, d_offs, n_recs, n_bases, stream, true, first_pos);
  if (!rc) record_order(c, c->last_s);
  return rc;
}

// ---------------------------------------------------------------------------
// exact radix refine of the top-N threshold (spike counts >= 4095; rare)
// ---------------------------------------------------------------------------
// (sc, n): the spike counts ranked — the whole pool, or a rank's slice of it
// (nk_finalize_slice); sc == nullptr means the handle's own pool
static int refine_threshold(nk_counter *c, uint64_t want, uint64_t max_sc, TopState &st,
                            hipStream_t s, uint64_t lo = 0, uint64_t n = ~0ull) {
  if (n == ~0ull) n = c->pool;
  const SpikeSrc sc = spike_src(c, lo);
  int top_bit = 63;
  while (top_bit > 0 && !((max_sc >> top_bit) & 1)) --top_bit;
  int shift = (top_bit / 8) * 8;
  uint64_t prefix = 0, above = 0;
  for (;;) {
    HIPCHK(hipMemsetAsync(c->radix_h.p, 0, 256 * 4, s));
    HIPCHK(launch_radix_hist(sc, n, shift, prefix, c->radix_h.p, s));
    uint32_t h[256];
    HIPCHK(hipMemcpyAsync(h, c->radix_h.p, sizeof h, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    int d = 255;
    for (; d >= 0; --d) {
      if (above + h[d] >= want) break;
      above += h[d];
    }
    if (d < 0) d = 0;
    prefix = (prefix << 8) | (uint64_t)d;
    if (shift == 0) break;
    shift -= 8;
  }
  st.T = prefix;
  st.n_above = above;
  st.need = want - above;
  st.emit_above = 0;
  st.refine = 0;
  return NK_OK;
}

// fuse_want > 0: the LIF kernel also selects the top rows and runs the
// uniques post step (part: the partitioned count's records are used)
// wire != nullptr: the currents are the (all-reduced) u32 wire vector of
// nk_wire32; the LIF reads them from it and writes the u64 currents
// LIF parameters of a finalize, the closed-form table for them (cached), and
// the spike histogram + stats zeroed unless this call's prep already did it
static LifParams lif_params(const nk_counter *c, int streaming) {
  LifParams lp{};
  lp.steps = c->steps;
  lp.thr = c->thr;
  lp.leak = c->leak;
  lp.refr = c->refr;
  lp.skip_zero = streaming ? 0 : 1;  // process_parallel skips zero currents (:189-191)
  return lp;
}

// closed-form results for fresh neurons with count < 65536, cached per params
static int lif_table(nk_counter *c, const LifParams &lp, hipStream_t s) {
  if (!c->lif_valid || c->lif_key.steps != lp.steps || c->lif_key.refr != lp.refr ||
      memcmp(&c->lif_key.thr, &lp.thr, 4) || memcmp(&c->lif_key.leak, &lp.leak, 4)) {
    if (int rc = c->lif_tbl.ensure(kLifTable)) return rc;
    HIPCHK(launch_lif_table(c->lif_tbl.p, kLifTable, lp, s));
    c->lif_key = lp;
    c->lif_valid = true;
  }
  return NK_OK;
}

static int lif_prepare(nk_counter *c, int streaming, LifParams &lp, hipStream_t s) {
  lp = lif_params(c, streaming);
  if (int rc = lif_table(c, lp, s)) return rc;
  if (!c->lif_zeroed) {
    ZeroList z{};
    z.ptr[0] = c->hist.p;  z.bytes[0] = kHistBins * kHistCopies * 4;
    z.ptr[1] = c->stats.p; z.bytes[1] = 16;
    z.n = 2;
    HIPCHK(launch_zero(z, s));
  }
  c->lif_zeroed = false;
  return NK_OK;
}

// the LIF the write-through K1b already ran (K1bLif) holds for this finalize
static bool k1b_lif_holds(const nk_counter *c, const LifParams &lp, uint32_t fuse_want,
                          const uint32_t *wire) {
  if (!c->k1b_lif || wire || fuse_want || !c->state_fresh || c->pend_slices || c->cur_fresh ||
      c->cur_in_wire || !c->pool)
    return false;
  const LifParams &k = c->k1b_lp;
  if (k.steps != lp.steps || k.refr != lp.refr || memcmp(&k.thr, &lp.thr, 4) ||
      memcmp(&k.leak, &lp.leak, 4))
    return false;
  // skip_zero differs (a streaming finalize): the same outcome when a zero
  // count cannot spike from the reset state (thr > 0: v stays 0)
  return k.skip_zero == lp.skip_zero || lp.thr > 0.0f;
}

static int enqueue_lif(nk_counter *c, int streaming, uint32_t fuse_want, bool part,
                       hipStream_t s, const uint32_t *wire = nullptr) {
  LifParams lp;
  // (a LIF with no count since the last one: that one's derived state first)
  int rc = settle_state(c, s);
  if (rc) return rc;
  const bool k1b = k1b_lif_holds(c, lif_params(c, streaming), fuse_want, wire);
  c->k1b_lif = false;
  if (k1b) {  // sc8, hist and stats are this LIF's: the state is derived
    c->lif_zeroed = false;
    c->sc8_ok = true;
    c->state_derived = true;
    c->derived_lp = lif_params(c, streaming);
    c->state_fresh = false;
    return NK_OK;
  }
  if ((rc = lif_prepare(c, streaming, lp, s))) return rc;
  TopFuse tf{};
  if (fuse_want) {
    const uint32_t nb = lif_blocks(c->pool);
    if ((rc = c->bcand.ensure((uint64_t)nb * fuse_want)) || (rc = c->bcnt.ensure(nb)) ||
        (rc = c->tbuckets.ensure(fuse_want)))
      return rc;
    tf.want = fuse_want;
    tf.bcand = c->bcand.p;
    tf.bcnt = c->bcnt.p;
    tf.st = c->topst.p;
    tf.cand = c->cand.p;
    tf.top_cur = c->top_cur.p;
    // kept records (Part, or Gen/Wide): the top buckets and their overflow
    const bool gk = part && !c->part_used;
    tf.post = PostArgs{c->set_alloc, part ? (gk ? c->last_ga.overflow : c->p_over.p) : nullptr,
                       part ? 1 : 0, c->set_mask_d.p, c->tbuckets.p, c->post_flags.p, c->uniq.p,
                       c->special.p, c->n_hits.p,
                       gk ? (uint32_t)c->last_ga.bin_bits : c->last_pa.bin_bits,
                       part ? (gk ? c->last_ga.n_buckets : c->last_pa.n_buckets) : 0u};
  }
  // steps == 0: the kernel leaves every neuron as it is (streaming returns early,
  // src/spiking_hash.rs:549-551; in-memory runs zero iterations)
  if (wire) {
    c->pend_slices = 0;
    c->cur_fresh = false;
    c->cur_in_wire = false;
  } else if ((rc = materialize(c, true, s))) {  // finalize right after a reset
    return rc;
  }
  // partitioned count with its partials pending: the prep zeroed the currents and
  // only overflowed buckets added into them, so only those buckets are read
  const uint32_t *over = (!wire && c->pend_slices && c->part_used) ? c->p_over.p : nullptr;
  if (!fuse_want && (rc = c->sc8.ensure(c->pool))) return rc;
  HIPCHK(launch_lif_apply(c->cur.p, wire ? wire : c->partials.p, wire ? 1u : c->pend_slices,
                          wire ? 1 : 0, over, (int)c->last_pa.bin_bits, c->state_fresh ? 1 : 0,
                          /*derive=*/1, c->v.p, c->r.p, c->sc.p, c->pool, lp, c->lif_tbl.p, kLifTable,
                          c->hist.p, c->stats.p, tf, s, fuse_want ? nullptr : c->sc8.p));
  c->pend_slices = 0;
  c->sc8_ok = !fuse_want;
  if (c->pool && c->state_fresh) {  // from the reset state: v / r / spike counts derived
    c->state_derived = true;
    c->derived_lp = lp;
  }
  if (c->pool) c->state_fresh = false;
  return NK_OK;
}

// (lo, n): as refine_threshold; candidate indices are relative to lo
static int enqueue_select(nk_counter *c, uint64_t want, hipStream_t s, uint64_t lo = 0,
                          uint64_t n = ~0ull) {
  if (n == ~0ull) n = c->pool;
  const SpikeSrc sc = spike_src(c, lo);
  const uint64_t *cur = c->cur.p + lo;
  const unsigned nb = (unsigned)((n + 2047) / 2048);
  int rc;
  if ((rc = c->tie_cnt.ensure(nb))) return rc;
  // rows the passes leave unfilled (a threshold inconsistent with the counts)
  // read back as index ~0, never as stale rows
  HIPCHK(hipMemsetAsync(c->cand.p, 0xFF, want * sizeof(TopCand), s));
  HIPCHK(launch_topn_count(sc, n, c->topst.p, c->tie_cnt.p, c->cand.p, s));
  HIPCHK(launch_topn_emit(sc, n, c->topst.p, c->tie_cnt.p, c->cand.p, s));
  HIPCHK(launch_topn_sort(c->cand.p, (uint32_t)want, n, cur, c->top_cur.p, s));
  return NK_OK;
}

#ifndef NK_U1_SLICE_BUDGET
#define NK_U1_SLICE_BUDGET 1024  // scan workgroups per launch (A/B: 1024 with 4 loads in flight best)
#endif
static int enqueue_uniques(nk_counter *c, uint32_t m, bool rescan, bool post_done,
                           hipStream_t s) {
  const bool part = c->part_used && !rescan;
  const bool genk = c->gen_keep && !rescan;  // kept Gen/Wide records: rescan the hit tiles only
  int rc;
  if ((rc = c->tbuckets.ensure(m))) return rc;
  if (!post_done)
    HIPCHK(launch_top_post(c->cand.p, c->top_cur.p, m, c->set_alloc,
                           part ? c->p_over.p : genk ? c->last_ga.overflow : nullptr,
                           (part || genk) ? 1 : 0, c->set_mask_d.p, c->tbuckets.p, c->post_flags.p,
                           c->uniq.p, c->special.p, c->n_hits.p,
                           genk ? (uint32_t)c->last_ga.bin_bits : c->last_pa.bin_bits, s,
                           part ? c->last_pa.n_buckets : genk ? c->last_ga.n_buckets : 0u));
  // the set must be empty up to the pass's mask: after the count's prep it is
  c->dirty_before = c->set_clean ? 0 : c->set_alloc;
  if (!part || !c->set_clean)
    HIPCHK(c->w128 ? launch_set_fill128(c->set_keys.p, c->set_mask_d.p, c->set_alloc, s)
                   : launch_set_fill(c->set_keys.p, c->set_mask_d.p, c->set_alloc, s));
  c->set_clean = false;
  c->set_dirty = c->set_alloc;  // until a readback tells the mask the pass used
  UniqArgs u{};
  u.top = c->cand.p;
  u.n_top = m;
  u.tbl_size = (uint32_t)top_tbl_size(m);
  u.set_keys = c->set_keys.p;
  u.set_mask = c->set_mask_d.p;
  u.uniq = c->uniq.p;
  u.special = c->special.p;
  if (c->xport_dst) {  // nk_finalize_export: new keys also go to the segment
    u.xdst = c->xport_dst;
    u.xn = c->export_n.p;
    u.xcap = c->xport_cap;
  }
  if (part) {
    const uint32_t slices = std::max<uint32_t>(1, NK_U1_SLICE_BUDGET / m);
    HIPCHK(launch_part_uniques(c->last_in, (int)c->k, c->canonical, c->last_pa, u, c->tbuckets.p,
                               c->post_flags.p + 2, m, slices, s));
  } else {
    KmerInput in = c->last_in;
    const uint64_t tile = c->gen_km >= 0 ? kPartTile : kTile;
    in.n_tiles = n_tiles_for(in.n_bases, tile);
    if ((rc = c->tile_rec.ensure(std::max<uint64_t>(in.n_tiles, 1)))) return rc;
    in.tile_rec = c->tile_rec.p;
    HIPCHK(launch_tile_rec(in, tile, c->tile_rec.p, s));
    if (genk) {
      // the tiles holding the top rows' records, then the rescan of those only;
      // a full list sets post flag 1 (-> settle_top redoes a full rescan)
      // list capacity: 2^20 entries, or 1/16 of the input's lanes when that is
      // more (a 12.5 Gbase config-5 input: planted repeats give the top rows
      // ~800 k records each, 16 M lanes, past 2^20 -> the full rescan, 70 ms,
      // profiles/r04_t3); a list past 1/16 of the lanes would hash as much as
      // half a rescan anyway.  NK_UNIQ_TILE_LIST (tests): a small list overflows.
      const uint32_t kTileList = [&] {
        const char *e = getenv("NK_UNIQ_TILE_LIST");
        const unsigned long v = e ? strtoul(e, nullptr, 10) : 0;
        const uint64_t lanes16 = in.n_tiles * kPartBlock / 16;  // k_part_gen: one lane per 16 positions
        return v ? (uint32_t)v
                 : (uint32_t)std::min<uint64_t>(std::max<uint64_t>(1u << 20, lanes16), 1u << 30);
      }();
      if ((rc = c->u_tiles.ensure(kTileList)) || (rc = c->u_nt.ensure(1))) return rc;
      if (c->u_mark.n < in.n_tiles || c->u_mark_zeroed < in.n_tiles || ++c->u_epoch == 0) {
        if ((rc = c->u_mark.ensure(in.n_tiles))) return rc;
        HIPCHK(hipMemsetAsync(c->u_mark.p, 0, c->u_mark.n * 4, s));
        c->u_mark_zeroed = c->u_mark.n;
        c->u_epoch = 1;
      }
      HIPCHK(hipMemsetAsync(c->u_nt.p, 0, 4, s));
      const bool tagged = c->last_ga.lane_tag != 0;
      if (tagged) {
        if ((rc = c->u_lanes.ensure(in.n_tiles * kLaneWords))) return rc;
        HIPCHK(hipMemsetAsync(c->u_lanes.p, 0, in.n_tiles * kLaneWords * 4, s));
      }
      const uint32_t slices = std::max<uint32_t>(1, NK_U1_SLICE_BUDGET / m);
      HIPCHK(launch_uniq_tiles(c->last_ga, c->gen_wide ? 1 : 0, u, c->tbuckets.p, c->post_flags.p + 2,
                               m, slices, c->u_tiles.p, c->u_nt.p, kTileList, c->post_flags.p + 1,
                               c->u_mark.p, c->u_epoch, tagged ? c->u_lanes.p : nullptr,
                               env_u32("NK_UNIQ_HIT_QUEUE", ~0u), s));
      if (tagged)  // the list holds lanes: their windows, keyed from global memory
        HIPCHK(launch_uniq_lanes(in, (int)c->k, c->canonical, c->gen_km, c->pool, u, c->u_tiles.p,
                                 c->u_nt.p, kTileList, s));
      else
        HIPCHK(launch_uniq_gen(in, (int)c->k, c->canonical, c->gen_km, c->pool, u, s, c->u_tiles.p,
                               c->u_nt.p, kTileList));
    } else if (c->gen_km >= 0)
      HIPCHK(launch_uniq_gen(in, (int)c->k, c->canonical, c->gen_km, c->pool, u, s));
    else if (c->w128)
      HIPCHK(launch_uniques128(in, (int)c->k, c->canonical, c->pool, u, s));
    else
      HIPCHK(launch_uniques(in, (int)c->k, c->canonical, c->pool, u, s));
  }
  return NK_OK;
}

// flag3: a device word copied into ResultHdr.flags[3] (the merge's reasons to redo)
static int enqueue_readback(nk_counter *c, uint32_t m, bool uniq, hipStream_t s,
                            const uint32_t *flag3 = nullptr, const uint32_t *uniq_src = nullptr) {
  HIPCHK(launch_gather(c->topst.p, c->stats.p, uniq ? c->set_mask_d.p : nullptr,
                       uniq ? c->post_flags.p : nullptr, flag3, c->cand.p,
                       uniq ? (uniq_src ? uniq_src : c->uniq.p) : nullptr, m,
                       c->res_hd, reinterpret_cast<uint64_t *>(c->res_hd + nk_counter::kResFlagOff),
                       ++c->res_seq, s));  // straight into pinned host memory: no copy
  return NK_OK;
}

// Wait for the k_gather of enqueue_readback: spin on its completion word in
// mapped host memory (the results are complete once it shows res_seq; the
// kernel does no memory access after it), which sees completion ~5 us sooner
// than hipStreamSynchronize (tools/syncbench.hip).  Past kSpinUs the wait
// falls back to hipStreamSynchronize, which also reports a failed launch.
static int wait_readback(nk_counter *c, hipStream_t s) {
  constexpr double kSpinUs = 20000.0;
  const uint64_t *flag = reinterpret_cast<const uint64_t *>(c->res_h + nk_counter::kResFlagOff);
  const auto t0 = std::chrono::steady_clock::now();
  for (uint32_t i = 0;; ++i) {
    if (__atomic_load_n(flag, __ATOMIC_ACQUIRE) == c->res_seq) return NK_OK;
    __builtin_ia32_pause();
    if ((i & 1023) == 1023 &&
        std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() >
            kSpinUs)
      break;
  }
  HIPCHK(hipStreamSynchronize(s));
  if (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != c->res_seq)
    return fail(NK_E_DEVICE, "result readback did not complete");
  return NK_OK;
}

// LIF + exact top-N + uniques with ONE host synchronisation in the common
// case; the rare corrections (spike counts past the histogram, a hash set too
// small for the top rows, an overflowed top bucket) are redone after it.
// use_kpn: the uniques column comes from the exact table's kmer_per_neuron
// (a process call with opts.exact_counts) instead of the uniques pass
static int finish_top(nk_counter *c, uint64_t want, bool fused, bool uniq, bool use_kpn,
                      hipStream_t s);
static int settle_top(nk_counter *c, uint64_t want, bool uniq, bool use_kpn, bool account,
                      hipStream_t s);

static bool top_fused(const nk_counter *c, uint64_t want) {
  return want && want <= kFuseMaxTopN && lif_blocks(c->pool) <= kFuseMaxBlocks &&
         c->pool <= (1ull << 24);
}

static int lif_top_uniques(nk_counter *c, int streaming, bool use_kpn, hipStream_t s,
                           const uint32_t *wire = nullptr) {
  int rc = whole_pool(c);
  if (rc) return rc;
  c->top_keys_ready = false;
  const uint64_t want = std::min<uint64_t>(c->opts.top_n, c->pool);
  const bool uniq = want && c->have_input && c->last_in.n_tiles;
  // top-N selection (and the uniques post step) inside the LIF kernel
  const bool fused = top_fused(c, want);
  if ((rc = enqueue_lif(c, streaming, fused ? (uint32_t)want : 0u,
                        uniq && (c->part_used || c->gen_keep), s, wire)))
    return rc;
  HIPCHK(mark(c, 4, s));
  return finish_top(c, want, fused, uniq, use_kpn, s);
}

// After a LIF pass (hist, stats and, when fused, the selected rows on the
// device): exact top-N, uniques, one readback, energy and c->top.
static int finish_top(nk_counter *c, uint64_t want, bool fused, bool uniq, bool use_kpn,
                      hipStream_t s) {
  int rc;
  if (want && !fused) {
    HIPCHK(launch_topn_threshold(c->hist.p, want, c->pool, c->topst.p, s));
    if ((rc = enqueue_select(c, want, s))) return rc;
  }
  HIPCHK(mark(c, 5, s));
  auto uniques = [&](bool post_done) -> int {
    if (!uniq) return NK_OK;
    if (use_kpn) {
      HIPCHK(exact_top_uniques(c->cand.p, (uint32_t)want, c->kpn.p, c->uniq.p, s));
      return NK_OK;
    }
    return enqueue_uniques(c, (uint32_t)want, false, post_done, s);
  };
  if ((rc = uniques(fused))) return rc;
  if ((rc = enqueue_readback(c, (uint32_t)want, uniq, s))) return rc;
  HIPCHK(mark(c, 6, s));  // may still be pending on return: timings are collected on demand
  if ((rc = wait_readback(c, s))) return rc;
  return settle_top(c, want, uniq, use_kpn, true, s);
}

// After the readback in c->res_h: energy (account), the rare corrections
// (each with its own synchronisation) and c->top.
static int settle_top(nk_counter *c, uint64_t want, bool uniq, bool use_kpn, bool account,
                      hipStream_t s) {
  int rc;
  auto uniques = [&](bool post_done) -> int {
    if (!uniq) return NK_OK;
    if (use_kpn) {
      HIPCHK(exact_top_uniques(c->cand.p, (uint32_t)want, c->kpn.p, c->uniq.p, s));
      return NK_OK;
    }
    return enqueue_uniques(c, (uint32_t)want, false, post_done, s);
  };
  const ResultHdr *h = reinterpret_cast<const ResultHdr *>(c->res_h);
  const TopCand *hc = reinterpret_cast<const TopCand *>(c->res_h + sizeof(ResultHdr));
  const uint32_t *hu =
      reinterpret_cast<const uint32_t *>(c->res_h + sizeof(ResultHdr) + want * sizeof(TopCand));
  if (account) {
    c->total_spikes += h->stats[0];
    c->total_energy += h->stats[0] * cost_fixed(c->cost);
    c->max_sc = h->stats[1];
  }
  if (want && h->st.refine) {  // spike counts >= 4095: exact radix refine, redo
    TopState st = h->st;
    if ((rc = refine_threshold(c, want, h->stats[1], st, s))) return rc;
    HIPCHK(hipMemcpyAsync(c->topst.p, &st, sizeof st, hipMemcpyHostToDevice, s));
    if ((rc = enqueue_select(c, want, s))) return rc;
    if ((rc = uniques(false))) return rc;
    if ((rc = enqueue_readback(c, (uint32_t)want, uniq, s))) return rc;
    HIPCHK(hipStreamSynchronize(s));
  }
  if (uniq && !use_kpn) {
    // set too small: grow to the capacity the top rows need, redo the pass
    if (h->flags[0]) {
      uint64_t cap = c->set_alloc;
      uint64_t sum = 0;
      std::vector<uint64_t> tc(want);
      HIPCHK(hipMemcpyAsync(tc.data(), c->top_cur.p, want * 8, hipMemcpyDeviceToHost, s));
      HIPCHK(hipStreamSynchronize(s));
      for (uint64_t x : tc) sum += x;
      while (cap < 2 * sum + 2) cap <<= 1;
      if ((rc = c->set_keys.ensure(c->w128 ? 3 * cap : cap))) return rc;
      c->set_alloc = cap;
      c->set_dirty = cap;
      c->set_clean = false;
    }
    if (h->flags[0] || h->flags[1]) {
      if ((rc = enqueue_uniques(c, (uint32_t)want, h->flags[1] != 0, false, s))) return rc;
      if ((rc = enqueue_readback(c, (uint32_t)want, uniq, s))) return rc;
      HIPCHK(hipStreamSynchronize(s));
    }
    c->set_cap = h->mask + 1;
    c->set_dirty = std::max(c->dirty_before, c->set_cap);  // the last pass wrote below its mask
  } else {
    c->set_cap = 0;
  }
  c->top.resize(want);
  for (uint64_t i = 0; i < want; ++i) {
    c->top[i].idx = hc[i].idx;
    c->top[i].spikes = hc[i].sc;
    c->top[i].uniques = uniq ? hu[i] : 0;
    c->top[i]._pad = 0;
  }
  return NK_OK;
}

static void collect_timings_now(nk_counter *c, bool with_count);

// The stage markers of the last call may still be pending when it returns
// (the results are awaited on k_gather's completion word, not on the stream):
// the timings are read when asked for.
static void collect_timings(nk_counter *c, bool with_count) {
  if (c->opts.stage_timing == 3) {  // nothing was recorded
    c->timing_pending = 0;
    c->n_stage = 0;
    return;
  }
  c->timing_pending = with_count ? 2 : 1;
  c->n_stage = full_timing(c) ? kStages : kStagesLight;
}

static void collect_timings_now(nk_counter *c, bool with_count) {
  // ev[0] start | ev[1] after index | ev[2] after K1 count (K1a) | ev[3] after
  // K1b/K1c | ev[4] after lif | ev[5] after topn | ev[6] after uniques |
  // ev[7] finalize start
  auto el = [](hipEvent_t a, hipEvent_t b) {
    float ms = 0;
    return hipEventElapsedTime(&ms, a, b) == hipSuccess ? ms : 0.0f;
  };
  if (!full_timing(c)) {
    const bool wc = with_count && count_timing(c);  // no count markers at level 2
    c->stage_ms[0] = wc ? el(c->ev[0], c->ev[1]) : (with_count ? -1.0f : 0.0f);
    c->stage_ms[1] = wc ? el(c->ev[1], c->ev[2]) : (with_count ? -1.0f : 0.0f);
    c->stage_ms[2] = with_count && !wc ? -1.0f : el(with_count ? c->ev[2] : c->ev[7], c->ev[6]);
    c->stage_ms[3] = el(with_count ? c->ev[0] : c->ev[7], c->ev[6]);
    c->n_stage = kStagesLight;
    return;
  }
  c->stage_ms[0] = with_count ? el(c->ev[0], c->ev[1]) : 0.0f;
  c->stage_ms[1] = with_count ? el(c->ev[1], c->ev[2]) : 0.0f;
  c->stage_ms[2] = with_count ? el(c->ev[2], c->ev[3]) : 0.0f;
  c->stage_ms[3] = el(with_count ? c->ev[3] : c->ev[7], c->ev[4]);
  c->stage_ms[4] = el(c->ev[4], c->ev[5]);
  c->stage_ms[5] = el(c->ev[5], c->ev[6]);
  c->stage_ms[6] = el(with_count ? c->ev[0] : c->ev[7], c->ev[6]);
  c->n_stage = kStages;
}

int nk_finalize(nk_counter *c, int streaming, void *stream) {
  if (!c) return fail(NK_E_INVALID, "null counter");
  (void)hipSetDevice(c->device);
  hipStream_t s = pick_stream(c, stream);
  HIPCHK(mark(c, 7, s));
  // after nk_exact_adopt (+ the caller's all-reduce) kmer_per_neuron is global:
  // the uniques column comes from it; else from this shard's k-mers
  int rc = lif_top_uniques(c, streaming, c->opts.exact_counts && c->exact_built && c->kpn_global, s);
  if (rc) return rc;
  c->top_valid = true;
  // an accumulate on this handle precedes: report its stages too
  collect_timings(c, c->have_input);
  return NK_OK;
}

// SpikingKmerCounter::simulate_spikes_auto (src/spiking_hash.rs:697-714).  On
// x86-64 with AVX2 (the reference's target, and the host of an MI355X node) it
// is simulate_spikes_simd (:544-659): `steps` LifNeuron updates of EVERY neuron,
// zero currents included, from the currents the counter holds (neuron_currents:
// the last process call's, :175/:464; zero after process_sequence, :271); the
// spikes go to the neurons' counts and the energy tracker; steps == 0 returns
// before touching anything (:549-551).  The same closed-form LIF kernel as a
// process call with the streaming rule, then the top rows again: their uniques
// column is kmer_per_neuron when the handle holds the table (exact_counts,
// process_sequence), else the distinct k-mers of the last input (which must
// still be resident, as for nk_finalize), else 0 (no input since new/reset).
int nk_simulate_spikes_auto(nk_counter *c) {
  if (!c) return fail(NK_E_INVALID, "null counter");
  int rc = whole_pool(c);
  if (rc) return rc;
  if (c->cur_in_wire)
    return fail(NK_E_INVALID, "the currents are in the wire vector until nk_finalize_export");
  if (c->steps == 0 || c->pool == 0) return NK_OK;
  (void)hipSetDevice(c->device);
  hipStream_t s = pick_stream(c, nullptr);
  HIPCHK(mark(c, 7, s));
  if (c->kpn_valid) {
    const uint64_t want = std::min<uint64_t>(c->opts.top_n, c->pool);
    const bool fused = top_fused(c, want);
    if ((rc = enqueue_lif(c, 1, fused ? (uint32_t)want : 0u, false, s))) return rc;
    HIPCHK(mark(c, 4, s));
    if ((rc = finish_top(c, want, fused, want != 0, true, s))) return rc;
  } else if ((rc = lif_top_uniques(c, 1, false, s))) {
    return rc;
  }
  c->top_valid = true;
  collect_timings(c, false);
  return NK_OK;
}

static int process_device(nk_counter *c, const uint8_t *d_bases, const uint64_t *d_offs,
                          size_t n_recs, size_t n_bases, void *stream, int streaming) {
  if (int rc0 = whole_pool(c)) return rc0;
  int rc = accumulate(c, d_bases, d_offs, n_recs, n_bases, stream, true);
  if (rc) {
    c->pend_slices = 0;
    c->lif_zeroed = false;
    return rc;
  }
  hipStream_t s = pick_stream(c, stream);
  if ((rc = lif_top_uniques(c, streaming, c->opts.exact_counts && c->exact_built, s))) return rc;
  c->top_valid = true;
  collect_timings(c, true);
  return NK_OK;
}

int nk_process_parallel_device(nk_counter *c, const uint8_t *d_bases, const uint64_t *d_offs,
                               size_t n_recs, size_t n_bases, void *stream) {
  return process_device(c, d_bases, d_offs, n_recs, n_bases, stream, 0);
}

static int check_offsets(const uint64_t *offs, size_t n_recs) {
  if (!offs) return fail(NK_E_INVALID, "null offsets");
  if (offs[0] != 0) return fail(NK_E_INVALID, "rec_offsets[0] must be 0");
  for (size_t i = 0; i < n_recs; ++i)
    if (offs[i + 1] < offs[i]) return fail(NK_E_INVALID, "rec_offsets not monotone at %zu", i);
  return NK_OK;
}

static bool any_kmer(const uint64_t *offs, size_t n_recs, size_t k) {
  for (size_t i = 0; i < n_recs; ++i)
    if (offs[i + 1] - offs[i] >= k) return true;
  return false;
}

static int process_host(nk_counter *c, const uint8_t *bases, const uint64_t *offs, size_t n_recs,
                        int streaming) {
  if (!c) return fail(NK_E_INVALID, "null counter");
  int rc = check_offsets(offs, n_recs);
  if (rc) return rc;
  const size_t n_bases = (size_t)offs[n_recs];
  if (c->pool == 0) {
    if (any_kmer(offs, n_recs, c->k))
      return fail(NK_E_INVALID, "pool_size 0 with k-mers present (the reference panics on % 0)");
    // nothing to do: no neurons, no k-mers
    c->top.clear();
    c->top_valid = true;
    return NK_OK;
  }
  (void)hipSetDevice(c->device);
  hipStream_t s = pick_stream(c, nullptr);
  if ((rc = c->in_bases.ensure(n_bases + 16))) return rc;
  if ((rc = c->in_offs.ensure(n_recs + 1))) return rc;
  if (n_bases) HIPCHK(hipMemcpyAsync(c->in_bases.p, bases, n_bases, hipMemcpyHostToDevice, s));
  HIPCHK(hipMemcpyAsync(c->in_offs.p, offs, (n_recs + 1) * 8, hipMemcpyHostToDevice, s));
  return process_device(c, c->in_bases.p, c->in_offs.p, n_recs, n_bases, s, streaming);
}

int nk_process_parallel(nk_counter *c, const uint8_t *bases, const uint64_t *offs, size_t n_recs) {
  return process_host(c, bases, offs, n_recs, 0);
}

static int ingest_file(nk_counter *c, const char *path, bool *fallback);

// A FASTA/FASTQ file through the GPU ingest (nk_ingest.h), then the LIF rule of
// process_file_streaming (streaming = 1, src/spiking_hash.rs:277-486) or of
// process_parallel over the file's records (streaming = 0, src/main.rs:45-46).
static int process_file(nk_counter *c, const char *path, int streaming) {
  if (!c) return fail(NK_E_INVALID, "null counter");
  if (!path) return fail(NK_E_INVALID, "null path");
  bool fallback = c->pool == 0;  // pool 0: the host path checks for k-mers (% 0)
  int rc = whole_pool(c);
  if (rc) return rc;
  if (!fallback) {
    rc = ingest_file(c, path, &fallback);
    if (rc) return rc;
  }
  if (fallback) {  // the host reader (nk_fastx.cpp): blank lines between FASTQ records
    std::vector<uint8_t> bases;
    std::vector<uint64_t> offs;
    std::string err;
    rc = read_fastx_all(path, bases, offs, err);
    if (rc) return fail(rc, "%s", err.c_str());
    return process_host(c, bases.data(), offs.data(), offs.size() - 1, streaming);
  }
  hipStream_t s = pick_stream(c, nullptr);
  HIPCHK(mark(c, 0, s));
  HIPCHK(mark(c, 1, s));
  HIPCHK(mark(c, 2, s));
  if ((rc = lif_top_uniques(c, streaming, c->opts.exact_counts && c->exact_built, s))) return rc;
  c->top_valid = true;
  collect_timings(c, true);
  return NK_OK;
}

int nk_process_file_streaming(nk_counter *c, const char *path) {
  return process_file(c, path, 1);
}

int nk_process_file_parallel(nk_counter *c, const char *path) {
  return process_file(c, path, 0);
}

int nk_top_kmers(nk_counter *c, const uint64_t **d_keys, size_t *n_keys) {
  if (!c || !d_keys || !n_keys) return fail(NK_E_INVALID, "null argument");
  (void)hipSetDevice(c->device);
  hipStream_t s = pick_stream(c, nullptr);
  const uint32_t m = (uint32_t)c->top.size();
  if (!m || !c->set_cap) {
    *d_keys = nullptr;
    *n_keys = 0;
    return NK_OK;
  }
  int rc;
  if (!c->top_keys_ready) {  // else: the padded export already compacted this shard's list
    if ((rc = c->top_keys.ensure(c->w128 ? 2 * c->set_cap : c->set_cap + 1))) return rc;
    HIPCHK(hipMemsetAsync(c->top_keys_n.p, 0, 8, s));
    if (c->w128)  // (lo, hi) pairs
      HIPCHK(launch_set_compact128(c->set_keys.p, c->set_cap, c->top_keys.p, c->top_keys_n.p, s));
    else
      HIPCHK(launch_set_compact(c->set_keys.p, c->set_cap, c->special.p, m, c->cand.p, c->pool,
                                c->top_keys.p, c->top_keys_n.p, s));
  }
  unsigned long long n = 0;
  HIPCHK(hipMemcpyAsync(&n, c->top_keys_n.p, 8, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  *d_keys = c->top_keys.p;
  *n_keys = (size_t)n;
  return NK_OK;
}

// uniques column of the top rows from a union of key lists (flat or the
// fixed-stride all-gather form); *complete = 0 if a segment was truncated
// (the top rows are then left as they were)
static int enqueue_merge(nk_counter *c, const MergeSrc &src, uint64_t max_keys, uint32_t m,
                         hipStream_t s, bool sep = false);

static int merge_keys(nk_counter *c, const MergeSrc &src, uint64_t max_keys, int *complete,
                      hipStream_t s) {
  const uint32_t m = (uint32_t)c->top.size();
  if (complete) *complete = 1;
  if (!m) return NK_OK;
  int rc = enqueue_merge(c, src, max_keys, m, s);
  if (rc) return rc;
  uint32_t *hu = reinterpret_cast<uint32_t *>(c->res_h);
  HIPCHK(hipMemcpyAsync(hu, c->uniq.p, m * 4, hipMemcpyDeviceToHost, s));
  HIPCHK(hipMemcpyAsync(hu + m, c->trunc_d.p, 4, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  if (hu[m]) {
    if (complete) *complete = 0;
    return NK_OK;
  }
  for (uint32_t i = 0; i < m; ++i) c->top[i].uniques = hu[i];
  return NK_OK;
}

// the set emptied at the capacity max_keys needs, the uniques column zeroed,
// the merge kernel enqueued (c->trunc_d: bit 0 a truncated segment, bits 1..3
// the segment header flags).  sep: into the merge set (mset_*, muniq,
// mspecial), leaving this shard's own set and uniques as they are (a redo
// still exports them)
static uint64_t merge_cap(uint64_t max_keys) {
  uint64_t cap = 64;
  while (cap < 2 * max_keys + 2) cap <<= 1;
  return cap;
}

static int enqueue_merge(nk_counter *c, const MergeSrc &src, uint64_t max_keys, uint32_t m,
                         hipStream_t s, bool sep) {
  const uint64_t cap = merge_cap(max_keys);
  int rc;
  uint64_t &alloc = sep ? c->mset_alloc : c->set_alloc;
  DevBuf<unsigned long long> &keys = sep ? c->mset_keys : c->set_keys;
  if (cap > alloc) {
    if ((rc = keys.ensure(c->w128 ? 3 * cap : cap))) return rc;
    alloc = cap;
  }
  if (!sep) {  // the merge fills the shard's own set below cap
    c->set_clean = false;
    c->set_dirty = std::max(c->set_dirty, cap);
  }
  if ((rc = c->trunc_d.ensure(1)) || (rc = c->mset_mask_d.ensure(1)) ||
      (rc = c->muniq.ensure(kMaxTopN)) || (rc = c->mspecial.ensure(kMaxTopN)))
    return rc;
  uint64_t *mask = sep ? c->mset_mask_d.p : c->set_mask_d.p;
  uint32_t *uq = sep ? c->muniq.p : c->uniq.p, *sp = sep ? c->mspecial.p : c->special.p;
  if (!sep) c->set_cap = cap;
  // (the export's header kernel already emptied the merge set at this capacity)
  const bool prepped = sep && c->merge_prepped == cap && c->mset_alloc >= cap;
  c->merge_prepped = 0;
  if (!prepped)
    HIPCHK(launch_merge_prep(keys.p, mask, cap, c->w128 ? 1 : 0, uq, sp, m, c->trunc_d.p, s));
  UniqArgs u{};
  u.top = c->cand.p;
  u.n_top = m;
  u.tbl_size = (uint32_t)top_tbl_size(m);
  u.set_keys = keys.p;
  u.set_mask = mask;
  u.uniq = uq;
  u.special = sp;
  MergeSrc ms = src;
  ms.trunc = c->trunc_d.p;
  if (c->w128) {
    HIPCHK(launch_set_merge128(ms, c->pool, u, s));
  } else {
    HIPCHK(launch_set_merge(ms, c->pool, u, s));
  }
  return NK_OK;
}

int nk_merge_top_kmers(nk_counter *c, const uint64_t *d_keys, size_t n_keys, void *stream) {
  if (!c) return fail(NK_E_INVALID, "null counter");
  (void)hipSetDevice(c->device);
  MergeSrc src{};
  src.keys = d_keys;
  src.n = n_keys;
  return merge_keys(c, src, n_keys, nullptr, pick_stream(c, stream));
}

int nk_top_kmers_padded(nk_counter *c, uint64_t *d_out, size_t cap, void *stream) {
  if (!c || !d_out) return fail(NK_E_INVALID, "null argument");
  (void)hipSetDevice(c->device);
  hipStream_t s = pick_stream(c, stream);
  const uint32_t m = (uint32_t)c->top.size();
  if (!m || !c->set_cap) {
    HIPCHK(hipMemsetAsync(d_out, 0, 8, s));
    return NK_OK;
  }
  // Compact this shard's keys once per finish: a later exchange (the second,
  // exact-size pass of the union) must re-pad the SAME list -- the merge of a
  // truncated first pass has by then refilled the set with the union
  // (nk_merge_top_kmers_padded merges into it), so a second compaction would
  // export the truncated union instead of this shard's keys (found by the
  // world-4 loopback run, tests/test_gpu_loopback.py).
  if (!c->top_keys_ready) {
    int rc;
    if ((rc = c->top_keys.ensure(c->w128 ? 2 * c->set_cap : c->set_cap + 1))) return rc;
    HIPCHK(hipMemsetAsync(c->top_keys_n.p, 0, 8, s));
    if (c->w128)
      HIPCHK(launch_set_compact128(c->set_keys.p, c->set_cap, c->top_keys.p, c->top_keys_n.p, s));
    else
      HIPCHK(launch_set_compact(c->set_keys.p, c->set_cap, c->special.p, m, c->cand.p, c->pool,
                                c->top_keys.p, c->top_keys_n.p, s));
    c->top_keys_ready = true;  // kept for the variable-length fallback (nk_top_kmers)
  }
  HIPCHK(launch_pad_keys(c->top_keys.p, c->top_keys_n.p, cap, c->w128 ? 2 : 1, d_out, s));
  return NK_OK;
}

int nk_merge_top_kmers_padded(nk_counter *c, const uint64_t *d_buf, size_t world, size_t stride,
                              size_t cap, int *complete, void *stream) {
  if (!c || !d_buf || !complete) return fail(NK_E_INVALID, "null argument");
  if (!world || world > (1u << 20) || stride < 1 + (c->w128 ? 2 : 1) * cap)
    return fail(NK_E_INVALID, "bad all-gather layout (world %zu, stride %zu, cap %zu)", world,
                stride, cap);
  (void)hipSetDevice(c->device);
  MergeSrc src{};
  src.keys = d_buf;
  src.world = (uint32_t)world;
  src.stride = stride;
  src.cap = cap;
  return merge_keys(c, src, (uint64_t)world * cap, complete, pick_stream(c, stream));
}

// ---------------------------------------------------------------------------
// Multi-GPU step with one host synchronisation (neurokmer_amd/dist.py::
// finalize_step):  nk_accumulate_device -> nk_wire32 -> allreduce(wire, u32)
// -> nk_finalize_export -> allgather(segments) -> nk_merge_export
// [-> redo: nk_finalize_redo + the blocking key exchange]
// ---------------------------------------------------------------------------
int nk_wire32(nk_counter *c, uint32_t *d_wire, void *stream) {
  if (!c || (!d_wire && c->pool)) return fail(NK_E_INVALID, "null argument");
  if (c->cur_in_wire) return fail(NK_E_INVALID, "nk_wire32 twice without nk_finalize_export");
  (void)hipSetDevice(c->device);
  c->k1b_lif = false;  // the LIF reads the (all-reduced) wire
  hipStream_t s = pick_stream(c, stream);
  int rc = settle_state(c, s);
  if (rc || (rc = materialize(c, true, s))) return rc;
  // partitioned count with its partials pending: only overflowed buckets added into cur
  const uint32_t *over = (c->pend_slices && c->part_used) ? c->p_over.p : nullptr;
  HIPCHK(launch_wire32(c->cur.p, c->partials.p, c->pend_slices, over, (int)c->last_pa.bin_bits,
                       c->pool, d_wire, s));
  c->pend_slices = 0;
  c->cur_in_wire = true;
  return NK_OK;
}

int nk_finalize_export(nk_counter *c, int streaming, const uint32_t *d_wire, uint64_t *d_seg,
                       size_t cap, void *stream) {
  if (!c || !d_seg) return fail(NK_E_INVALID, "null argument");
  if (c->cur_in_wire != (d_wire != nullptr))
    return fail(NK_E_INVALID, d_wire ? "d_wire without nk_wire32" : "the currents are in the wire vector: pass it");
  if (cap > (1ull << 40)) return fail(NK_E_INVALID, "cap too large");
  if (int rc0 = whole_pool(c)) return rc0;
  const bool use_kpn = c->opts.exact_counts && c->exact_built && c->kpn_global;
  if (use_kpn)
    return fail(NK_E_UNSUPPORTED, "exact table: the uniques come from kmer_per_neuron (nk_finalize)");
  (void)hipSetDevice(c->device);
  hipStream_t s = pick_stream(c, stream);
  HIPCHK(mark(c, 7, s));
  c->top_keys_ready = false;
  c->top_valid = false;
  c->redo_ready = false;
  const uint64_t want = std::min<uint64_t>(c->opts.top_n, c->pool);
  const bool uniq = want && c->have_input && c->last_in.n_tiles;
  int rc;
  if ((rc = c->export_n.ensure(1))) return rc;
  if (!c->export_n_zeroed) {
    HIPCHK(hipMemsetAsync(c->export_n.p, 0, 8, s));
    c->export_n_zeroed = true;
  }
  const bool fused = top_fused(c, want);
  if (fused) {  // enqueue only: the host waits once, in nk_merge_export
    if ((rc = enqueue_lif(c, streaming, (uint32_t)want, uniq && (c->part_used || c->gen_keep), s,
                          d_wire)))
      return rc;
    HIPCHK(mark(c, 4, s));
    HIPCHK(mark(c, 5, s));
    c->xport_dst = d_seg;  // the pass appends each new key to the segment
    c->xport_cap = cap;
    rc = uniq ? enqueue_uniques(c, (uint32_t)want, false, true, s) : NK_OK;
    c->xport_dst = nullptr;
    if (rc) return rc;
  } else if ((rc = lif_top_uniques(c, streaming, false, s, d_wire))) {  // blocking, corrected
    return rc;
  }
  // the merge that follows (nk_finalize_dist knows its world size): its set
  // emptied by the header kernel
  MergePrep mp{};
  c->merge_prepped = 0;
  if (c->merge_world_hint && want && !getenv("NK_NO_MERGE_PREP_FUSE")) {
    const uint64_t mcap = merge_cap((uint64_t)c->merge_world_hint * cap);
    if (mcap > c->mset_alloc) {
      if ((rc = c->mset_keys.ensure(c->w128 ? 3 * mcap : mcap))) return rc;
      c->mset_alloc = mcap;
    }
    if ((rc = c->trunc_d.ensure(1)) || (rc = c->mset_mask_d.ensure(1)) ||
        (rc = c->muniq.ensure(kMaxTopN)) || (rc = c->mspecial.ensure(kMaxTopN)))
      return rc;
    mp = MergePrep{c->mset_keys.p, c->mset_mask_d.p, mcap, c->muniq.p, c->mspecial.p, (uint32_t)want,
                   c->trunc_d.p};
    c->merge_prepped = mcap;
  }
  c->merge_world_hint = 0;
  HIPCHK(launch_export(c->set_keys.p, c->set_mask_d.p, c->set_alloc, c->w128 ? 1 : 0, uniq,
                       fused, c->special.p, (uint32_t)want, want ? c->topst.p : nullptr,
                       c->post_flags.p, cap, d_seg, c->export_n.p, s, mp));
  c->export_pending = true;
  c->export_blocking = !fused;
  c->export_want = (uint32_t)want;
  c->export_uniq = uniq;
  return NK_OK;
}

int nk_merge_export(nk_counter *c, const uint64_t *d_buf, size_t world, size_t stride, size_t cap,
                    int *redo, void *stream) {
  if (!c || !d_buf || !redo) return fail(NK_E_INVALID, "null argument");
  if (!c->export_pending) return fail(NK_E_INVALID, "nk_finalize_export first");
  if (!world || world > (1u << 20) || stride < 1 + (c->w128 ? 2 : 1) * cap)
    return fail(NK_E_INVALID, "bad all-gather layout (world %zu, stride %zu, cap %zu)", world,
                stride, cap);
  (void)hipSetDevice(c->device);
  hipStream_t s = pick_stream(c, stream);
  c->export_pending = false;
  const uint32_t want = c->export_want;
  int rc;
  if ((rc = c->trunc_d.ensure(1))) return rc;
  if (want) {
    MergeSrc src{};
    src.keys = d_buf;
    src.world = (uint32_t)world;
    src.stride = stride;
    src.cap = cap;
    if ((rc = enqueue_merge(c, src, (uint64_t)world * cap, want, s, true))) return rc;
  }
  if ((rc = enqueue_readback(c, want, want != 0, s, want ? c->trunc_d.p : nullptr,
                             want ? c->muniq.p : nullptr)))
    return rc;
  HIPCHK(mark(c, 6, s));
  if ((rc = wait_readback(c, s))) return rc;
  const ResultHdr *h = reinterpret_cast<const ResultHdr *>(c->res_h);
  const TopCand *hc = reinterpret_cast<const TopCand *>(c->res_h + sizeof(ResultHdr));
  const uint32_t *hu =
      reinterpret_cast<const uint32_t *>(c->res_h + sizeof(ResultHdr) + want * sizeof(TopCand));
  if (!c->export_blocking) {  // the blocking export already counted its spikes
    c->total_spikes += h->stats[0];
    c->total_energy += h->stats[0] * cost_fixed(c->cost);
    c->max_sc = h->stats[1];
  }
  c->top.resize(want);
  for (uint32_t i = 0; i < want; ++i) {
    c->top[i].idx = hc[i].idx;
    c->top[i].spikes = hc[i].sc;
    c->top[i].uniques = hu[i];
    c->top[i]._pad = 0;
  }
  c->set_cap = c->export_uniq ? h->mask + 1 : 0;  // this shard's set (the merge used its own)
  if (c->export_uniq) c->set_dirty = std::max(c->dirty_before, c->set_cap);
  *redo = (want && h->flags[3]) ? 1 : 0;
  c->redo_ready = *redo != 0;
  c->top_valid = !*redo;
  collect_timings(c, c->have_input);
  return NK_OK;
}

int nk_finalize_redo(nk_counter *c, void *stream) {
  if (!c) return fail(NK_E_INVALID, "null counter");
  if (!c->redo_ready) return fail(NK_E_INVALID, "no nk_merge_export asked for a redo");
  (void)hipSetDevice(c->device);
  hipStream_t s = pick_stream(c, stream);
  c->redo_ready = false;
  // c->res_h holds the merge readback: this rank's TopState and flags[0..2]
  int rc = settle_top(c, c->export_want, c->export_uniq, false, false, s);
  if (rc) return rc;
  HIPCHK(hipStreamSynchronize(s));
  c->top_keys_ready = false;
  c->top_valid = true;
  return NK_OK;
}

// ---------------------------------------------------------------------------
// Pool-sliced multi-GPU finish (P up to 2^31):
//   reduce-scatter(currents) -> nk_finalize_slice: LIF + top rows of this
//   rank's neurons [lo, hi) only -> all-gather the slices' candidate rows ->
//   nk_adopt_slices: the global top rows, total spikes, this shard's uniques
//   pass for them -> (dist.union_top_kmers: the union of the shards' keys).
// The neuron state is sharded: after it, a rank's v / refractory / spike
// counts / currents are authoritative on [lo, hi) only.
// ---------------------------------------------------------------------------
static constexpr size_t kSliceHdr = 3;  // [rows, new spikes, max spike count]

// run_lif = false: the slice's LIF already ran (nk_slice_export); only the
// selection is redone, blocking, exact (a redo of the device-side finish)
static int finalize_slice_impl(nk_counter *c, int streaming, const void *d_slice, int slice_bits,
                               size_t lo, size_t hi, uint64_t *d_seg, size_t seg_rows,
                               hipStream_t s, bool run_lif) {
  if (lo > hi || hi > c->pool) return fail(NK_E_INVALID, "slice [%zu, %zu) outside the pool", lo, hi);
  if (run_lif && slice_bits != 32 && slice_bits != 64)
    return fail(NK_E_INVALID, "slice_bits must be 32 or 64");
  if (run_lif && hi > lo && !d_slice) return fail(NK_E_INVALID, "null slice");
  const uint64_t want = std::min<uint64_t>(c->opts.top_n, c->pool);
  if (seg_rows < want) return fail(NK_E_INVALID, "seg_rows (%zu) < top_n rows (%llu)", seg_rows,
                                   (unsigned long long)want);
  HIPCHK(mark(c, 7, s));
  const uint64_t n = hi - lo;
  const uint64_t m = std::min<uint64_t>(want, n);
  int rc;
  if (run_lif) {
    c->k1b_lif = false;  // the slice's LIF runs on the reduced slice
    LifParams lp;
    rc = settle_state(c, s);
    if (rc || (rc = lif_prepare(c, streaming, lp, s))) return rc;
    // the reduced slice replaces this shard's currents and pending partials
    c->pend_slices = 0;
    c->cur_in_wire = false;
    c->cur_fresh = false;
    if ((rc = c->sc8.ensure(c->pool))) return rc;
    if (n) {
      if (slice_bits == 64)
        HIPCHK(hipMemcpyAsync(c->cur.p + lo, d_slice, n * 8, hipMemcpyDeviceToDevice, s));
      const bool w32 = slice_bits == 32;
      HIPCHK(launch_lif_apply(c->cur.p + lo, w32 ? (const uint32_t *)d_slice : nullptr, w32 ? 1u : 0u,
                              w32 ? 1 : 0, nullptr, (int)c->last_pa.bin_bits, c->state_fresh ? 1 : 0,
                              /*derive=*/1, c->v.p + lo, c->r.p + lo, c->sc.p + lo, n, lp, c->lif_tbl.p,
                              kLifTable, c->hist.p, c->stats.p, TopFuse{}, s, c->sc8.p + lo));
    }
    c->sc8_ok = true;  // on [lo, hi), the only range this rank's passes read
    if (c->state_fresh) {  // derived on [lo, hi) (the rest of the pool is not this rank's)
      c->state_derived = true;
      c->derived_lp = lp;
    }
    c->state_fresh = false;
    c->sliced = true;  // only [lo, hi) of v / r / spike counts / currents is this rank's now
  }
  c->top_valid = false;
  c->top_keys_ready = false;
  if (m && run_lif) {
    HIPCHK(launch_topn_threshold(c->hist.p, m, n, c->topst.p, s));
    if ((rc = enqueue_select(c, m, s, lo, n))) return rc;
  }
  if ((rc = enqueue_readback(c, (uint32_t)m, false, s))) return rc;
  if ((rc = wait_readback(c, s))) return rc;
  const ResultHdr *h = reinterpret_cast<const ResultHdr *>(c->res_h);
  // a redo counts no spikes: the LIF that produced them was accounted already
  const uint64_t new_spikes = run_lif ? h->stats[0] : 0, max_sc = h->stats[1];
  // a redo selects by the exact radix passes: nk_slice_export's fused LIF
  // wrote no spike histogram (max_sc: the largest count of any slice, an
  // upper bound of this one's)
  TopState sel = h->st;
  if (m && (h->st.refine || !run_lif)) {  // spike counts >= 4095: exact radix refine over the slice
    if ((rc = refine_threshold(c, m, max_sc, sel, s, lo, n))) return rc;
    HIPCHK(hipMemcpyAsync(c->topst.p, &sel, sizeof sel, hipMemcpyHostToDevice, s));
    if ((rc = enqueue_select(c, m, s, lo, n))) return rc;
  }
  std::vector<TopCand> rows(m);
  std::vector<uint64_t> rcur(m);
  if (m) {
    HIPCHK(hipMemcpyAsync(rows.data(), c->cand.p, m * sizeof(TopCand), hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(rcur.data(), c->top_cur.p, m * 8, hipMemcpyDeviceToHost, s));
  }
  HIPCHK(hipStreamSynchronize(s));
  if (getenv("NK_DEBUG_SELECT")) {  // (tests: the selection state of a slice)
    uint64_t bad = 0;
    for (uint64_t i = 0; i < m; ++i) bad += rows[i].idx >= n;
    fprintf(stderr, "[nk select] slice [%zu, %zu) m %llu T %llu above %llu need %llu max_sc %llu "
                    "redo %d refine %u unfilled %llu\n", lo, hi, (unsigned long long)m,
            (unsigned long long)sel.T, (unsigned long long)sel.n_above,
            (unsigned long long)sel.need, (unsigned long long)max_sc, run_lif ? 0 : 1,
            (unsigned)h->st.refine, (unsigned long long)bad);
  }
  for (uint64_t i = 0; i < m; ++i)
    if (rows[i].idx >= n)
      return fail(NK_E_DEVICE,
                  "slice [%zu, %zu) selection left row %llu unfilled (T %llu, rows above %llu, "
                  "ties %llu, largest count %llu, redo %d)",
                  lo, hi, (unsigned long long)i, (unsigned long long)sel.T,
                  (unsigned long long)sel.n_above, (unsigned long long)sel.need,
                  (unsigned long long)max_sc, run_lif ? 0 : 1);
  std::vector<uint64_t> seg(kSliceHdr + 3 * m);
  seg[0] = m;
  seg[1] = new_spikes;
  seg[2] = max_sc;
  for (uint64_t i = 0; i < m; ++i) {
    seg[kSliceHdr + 3 * i] = rows[i].idx + lo;  // global neuron index
    seg[kSliceHdr + 3 * i + 1] = rows[i].sc;
    seg[kSliceHdr + 3 * i + 2] = rcur[i];
  }
  HIPCHK(hipMemcpyAsync(d_seg, seg.data(), seg.size() * 8, hipMemcpyHostToDevice, s));
  HIPCHK(hipStreamSynchronize(s));  // seg is host memory the copy reads
  c->slice_ready = true;
  return NK_OK;
}

int nk_finalize_slice(nk_counter *c, int streaming, const void *d_slice, int slice_bits,
                      size_t lo, size_t hi, uint64_t *d_seg, size_t seg_rows, void *stream) {
  if (!c || !d_seg) return fail(NK_E_INVALID, "null argument");
  (void)hipSetDevice(c->device);
  return finalize_slice_impl(c, streaming, d_slice, slice_bits, lo, hi, d_seg, seg_rows,
                             pick_stream(c, stream), true);
}

extern "C++" namespace nk {
// the blocking selection of this rank's slice after nk_slice_export (its LIF
// done): a redo of the device-side sliced finish (nk_dist.cpp)
int slice_reselect(nk_counter *c, size_t lo, size_t hi, uint64_t *d_seg, size_t seg_rows,
                   hipStream_t s) {
  (void)hipSetDevice(c->device);
  return finalize_slice_impl(c, 0, nullptr, 32, lo, hi, d_seg, seg_rows, pick_stream(c, s), false);
}
}  // namespace nk

// The pool-sliced finish with no host wait before nk_merge_export:
//   nk_slice_export  LIF of [lo, hi) from the reduce-scattered u32 slice, the
//                    slice's top rows (exact unless a spike count passed
//                    4095: flagged) into d_seg by a kernel;
//   <all-gather of the slice segments>
//   nk_adopt_export  the global rows picked on the device, this shard's
//                    uniques pass for them with its new keys appended to the
//                    key segment (nk_finalize_export's tail);
//   <all-gather of the key segments>
//   nk_merge_export  union -> uniques column, one readback; a redo (refine,
//                    set, bucket, truncation) takes the blocking path.
int nk_slice_export(nk_counter *c, int streaming, const uint32_t *d_slice, size_t lo, size_t hi,
                    uint64_t *d_seg, size_t seg_rows, void *stream) {
  if (!c || !d_seg) return fail(NK_E_INVALID, "null argument");
  if (lo > hi || hi > c->pool) return fail(NK_E_INVALID, "slice [%zu, %zu) outside the pool", lo, hi);
  if (hi > lo && !d_slice) return fail(NK_E_INVALID, "null slice");
  const uint64_t want = std::min<uint64_t>(c->opts.top_n, c->pool);
  if (seg_rows < want) return fail(NK_E_INVALID, "seg_rows (%zu) < top_n rows (%llu)", seg_rows,
                                   (unsigned long long)want);
  (void)hipSetDevice(c->device);
  hipStream_t s = pick_stream(c, stream);
  HIPCHK(mark(c, 7, s));
  c->k1b_lif = false;
  const uint64_t n = hi - lo;
  const uint64_t m = std::min<uint64_t>(want, n);
  LifParams lp;
  int rc = settle_state(c, s);
  if (rc || (rc = lif_prepare(c, streaming, lp, s))) return rc;
  c->pend_slices = 0;
  c->cur_in_wire = false;
  c->cur_fresh = false;
  c->top_valid = false;
  c->top_keys_ready = false;
  c->redo_ready = false;
  if ((rc = c->sc8.ensure(c->pool))) return rc;
  // the slice's top rows selected inside its LIF kernel (+ k_top_final), as the
  // plain finish does, when they fit: 2 kernels instead of the LIF, the
  // threshold and three select passes (a 1-rank rehearsal measured the
  // unfused form +0.04 ms per step, profiles/r04_s2)
  const bool fuse = m && m <= kFuseMaxTopN && lif_blocks(n) <= kFuseMaxBlocks && n <= (1ull << 24);
  TopFuse tf{};
  if (fuse) {
    const uint32_t nbk = lif_blocks(n);
    if ((rc = c->bcand.ensure((uint64_t)nbk * m)) || (rc = c->bcnt.ensure(nbk)) ||
        (rc = c->tbuckets.ensure(m)))
      return rc;
    tf.want = (uint32_t)m;
    tf.bcand = c->bcand.p;
    tf.bcnt = c->bcnt.p;
    tf.st = c->topst.p;
    tf.cand = c->cand.p;
    tf.top_cur = c->top_cur.p;
    // (its uniques bookkeeping is redone for the global rows by nk_adopt_export)
    tf.post = PostArgs{c->set_alloc, nullptr, 0, c->set_mask_d.p, c->tbuckets.p, c->post_flags.p,
                       c->uniq.p, c->special.p, c->n_hits.p, c->last_pa.bin_bits};
  }
  if (n)
    HIPCHK(launch_lif_apply(c->cur.p + lo, d_slice, 1u, 1, nullptr, (int)c->last_pa.bin_bits,
                            c->state_fresh ? 1 : 0, /*derive=*/1, c->v.p + lo, c->r.p + lo,
                            c->sc.p + lo, n, lp, c->lif_tbl.p, kLifTable, c->hist.p, c->stats.p,
                            tf, s, fuse ? nullptr : c->sc8.p + lo));
  c->sc8_ok = !fuse;
  if (c->state_fresh) {
    c->state_derived = true;
    c->derived_lp = lp;
  }
  c->state_fresh = false;
  c->sliced = true;
  if (m && !fuse) {
    HIPCHK(launch_topn_threshold(c->hist.p, m, n, c->topst.p, s));
    if ((rc = enqueue_select(c, m, s, lo, n))) return rc;
  }
  HIPCHK(launch_slice_seg(c->cand.p, c->top_cur.p, c->topst.p, c->stats.p, (uint32_t)m, lo, n, d_seg, s));
  c->slice_ready = true;
  return NK_OK;
}

int nk_adopt_export(nk_counter *c, const uint64_t *d_all, size_t world, size_t stride,
                    uint64_t *d_keyseg, size_t cap, void *stream) {
  if (!c || !d_all || !d_keyseg) return fail(NK_E_INVALID, "null argument");
  if (!c->slice_ready) return fail(NK_E_INVALID, "nk_slice_export first");
  if (cap > (1ull << 40)) return fail(NK_E_INVALID, "cap too large");
  const uint64_t want = std::min<uint64_t>(c->opts.top_n, c->pool);
  if (!world || stride < kSliceHdr + 3 * want)
    return fail(NK_E_INVALID, "bad all-gather layout (world %zu, stride %zu)", world, stride);
  if ((uint64_t)world * want > (uint64_t)kAdoptMax)
    return fail(NK_E_UNSUPPORTED, "world * top_n > %d: nk_adopt_slices", kAdoptMax);
  (void)hipSetDevice(c->device);
  hipStream_t s = pick_stream(c, stream);
  c->slice_ready = false;
  int rc;
  // every rank's slice yields min(top_n, its size) rows: together >= min(top_n, pool) = want
  HIPCHK(launch_slice_adopt(d_all, (uint32_t)world, stride, (uint32_t)want, c->pool, c->cand.p,
                            c->top_cur.p, c->topst.p, c->stats.p, s));
  const bool uniq = want && c->have_input && c->last_in.n_tiles;
  if ((rc = c->export_n.ensure(1))) return rc;
  if (!c->export_n_zeroed) {
    HIPCHK(hipMemsetAsync(c->export_n.p, 0, 8, s));
    c->export_n_zeroed = true;
  }
  c->xport_dst = d_keyseg;  // the uniques pass appends each new key to the segment
  c->xport_cap = cap;
  rc = uniq ? enqueue_uniques(c, (uint32_t)want, false, false, s) : NK_OK;
  c->xport_dst = nullptr;
  if (rc) return rc;
  MergePrep mp{};
  c->merge_prepped = 0;
  if (want && !getenv("NK_NO_MERGE_PREP_FUSE")) {
    const uint64_t mcap = merge_cap((uint64_t)world * cap);
    if (mcap > c->mset_alloc) {
      if ((rc = c->mset_keys.ensure(c->w128 ? 3 * mcap : mcap))) return rc;
      c->mset_alloc = mcap;
    }
    if ((rc = c->trunc_d.ensure(1)) || (rc = c->mset_mask_d.ensure(1)) ||
        (rc = c->muniq.ensure(kMaxTopN)) || (rc = c->mspecial.ensure(kMaxTopN)))
      return rc;
    mp = MergePrep{c->mset_keys.p, c->mset_mask_d.p, mcap, c->muniq.p, c->mspecial.p, (uint32_t)want,
                   c->trunc_d.p};
    c->merge_prepped = mcap;
  }
  HIPCHK(launch_export(c->set_keys.p, c->set_mask_d.p, c->set_alloc, c->w128 ? 1 : 0, uniq,
                       /*appended=*/true, c->special.p, (uint32_t)want, want ? c->topst.p : nullptr,
                       c->post_flags.p, cap, d_keyseg, c->export_n.p, s, mp));
  c->export_pending = true;
  c->export_blocking = false;
  c->export_want = (uint32_t)want;
  c->export_uniq = uniq;
  return NK_OK;
}

int nk_adopt_slices(nk_counter *c, const uint64_t *d_all, size_t world, size_t stride,
                    void *stream) {
  if (!c || !d_all) return fail(NK_E_INVALID, "null argument");
  if (!c->slice_ready) return fail(NK_E_INVALID, "nk_finalize_slice first");
  const uint64_t want = std::min<uint64_t>(c->opts.top_n, c->pool);
  if (!world || world > (1u << 20) || stride < kSliceHdr + 3 * want)
    return fail(NK_E_INVALID, "bad all-gather layout (world %zu, stride %zu)", world, stride);
  (void)hipSetDevice(c->device);
  hipStream_t s = pick_stream(c, stream);
  c->slice_ready = false;
  std::vector<uint64_t> all(world * stride);
  HIPCHK(hipMemcpyAsync(all.data(), d_all, all.size() * 8, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  // every global top row is among its slice's top rows: rank the union by
  // (spikes desc, index asc) — src/spiking_hash.rs:661-673's stable order
  struct Row { uint64_t idx, sc, cur; };
  std::vector<Row> cand;
  uint64_t new_spikes = 0;
  for (size_t r = 0; r < world; ++r) {
    const uint64_t *g = all.data() + r * stride;
    if (g[0] > want || kSliceHdr + 3 * g[0] > stride)
      return fail(NK_E_INVALID, "segment %zu holds %llu rows", r, (unsigned long long)g[0]);
    new_spikes += g[1];
    for (uint64_t i = 0; i < g[0]; ++i) {
      if (g[kSliceHdr + 3 * i] >= c->pool)
        return fail(NK_E_DEVICE, "segment %zu row %llu: neuron %llu outside the pool", r,
                    (unsigned long long)i, (unsigned long long)g[kSliceHdr + 3 * i]);
      cand.push_back(Row{g[kSliceHdr + 3 * i], g[kSliceHdr + 3 * i + 1], g[kSliceHdr + 3 * i + 2]});
    }
  }
  const uint64_t m = std::min<uint64_t>(want, cand.size());
  std::partial_sort(cand.begin(), cand.begin() + m, cand.end(), [](const Row &a, const Row &b) {
    return a.sc != b.sc ? a.sc > b.sc : a.idx < b.idx;
  });
  std::vector<TopCand> tc(m);
  std::vector<uint64_t> tcur(m);
  for (uint64_t i = 0; i < m; ++i) {
    tc[i] = TopCand{cand[i].idx, cand[i].sc};
    tcur[i] = cand[i].cur;
  }
  TopState st{};
  if (m) {
    HIPCHK(hipMemcpyAsync(c->cand.p, tc.data(), m * sizeof(TopCand), hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(c->top_cur.p, tcur.data(), m * 8, hipMemcpyHostToDevice, s));
  }
  HIPCHK(hipMemcpyAsync(c->topst.p, &st, sizeof st, hipMemcpyHostToDevice, s));
  c->total_spikes += new_spikes;
  c->total_energy += new_spikes * cost_fixed(c->cost);
  // this shard's distinct keys of the global rows (the caller unions them)
  const bool uniq = m && c->have_input && c->last_in.n_tiles;
  int rc;
  if (uniq && (rc = enqueue_uniques(c, (uint32_t)m, false, false, s))) return rc;
  if ((rc = enqueue_readback(c, (uint32_t)m, uniq, s))) return rc;
  if ((rc = wait_readback(c, s))) return rc;
  if ((rc = settle_top(c, m, uniq, false, false, s))) return rc;
  HIPCHK(hipStreamSynchronize(s));  // tc / tcur are host memory the copies read
  c->top_valid = true;
  collect_timings(c, c->have_input);
  return NK_OK;
}

static int table_ready(nk_counter *c, hipStream_t *s);

// Rows past the ones the last call selected (src/spiking_hash.rs:661-673: the
// stable sort, ties by index), the uniques column from kmer_per_neuron (built
// on demand from the last input without opts.exact_counts).
//   m <= kMaxTopN: the exact threshold by radix passes over the spike counts
//     (as many 8-bit digits as the known largest count has) and the select
//     kernels of the top-N path: O(P / 2048) scratch, no pool-sized sort.
//   more rows: the whole pool ranked by a stable radix sort over the bits of
//     the largest count (24 B of scratch per neuron).
static long extended_top(nk_counter *c, size_t m, nk_top_row *out) {
  hipStream_t s;
  int rc = table_ready(c, &s);
  if (rc) return rc;
  if ((rc = whole_pool(c))) return rc;
  const uint64_t P = c->pool;
  if ((rc = materialize(c, false, s))) return rc;
  if ((rc = c->rk_cand.ensure(m)) || (rc = c->rk_uniq.ensure(m))) return rc;
  std::vector<TopCand> tc(m);
  if (m <= (size_t)kMaxTopN) {
    // the rows land in c->cand / c->top_cur: their first top_n rows are the
    // call's own rows (same exact order), which the multi-GPU helpers read
    TopState st{};
    if ((rc = refine_threshold(c, m, c->max_sc, st, s))) return rc;
    HIPCHK(hipMemcpyAsync(c->topst.p, &st, sizeof st, hipMemcpyHostToDevice, s));
    if ((rc = enqueue_select(c, m, s))) return rc;
    HIPCHK(hipMemcpyAsync(tc.data(), c->cand.p, m * sizeof(TopCand), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));  // st is host memory the copy reads
  } else {
    if (P > 0xFFFFFFFFull)
      return fail(NK_E_UNSUPPORTED, "more than %d rows past top_n need pool_size < 2^32", kMaxTopN);
    if ((rc = c->rk_keys.ensure(2 * P)) || (rc = c->rk_idx.ensure(2 * P)) ||
        (rc = c->rk_tmp.ensure(rank_rows_temp_bytes(P))) || (rc = settle_state(c, s)))
      return rc;
    HIPCHK(rank_rows(c->sc.p, P, c->max_sc, c->rk_keys.p, c->rk_keys.p + P, c->rk_idx.p,
                     c->rk_idx.p + P, c->rk_tmp.p, c->rk_tmp.n, s));
    std::vector<uint64_t> key(m);
    std::vector<uint32_t> idx(m);
    HIPCHK(hipMemcpyAsync(key.data(), c->rk_keys.p + P, m * 8, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(idx.data(), c->rk_idx.p + P, m * 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    for (size_t i = 0; i < m; ++i) tc[i] = TopCand{idx[i], c->max_sc - key[i]};
  }
  std::vector<uint32_t> uq(m, 0);
  if (c->kpn_valid) {
    HIPCHK(hipMemcpyAsync(c->rk_cand.p, tc.data(), m * sizeof(TopCand), hipMemcpyHostToDevice, s));
    HIPCHK(exact_top_uniques(c->rk_cand.p, (uint32_t)m, c->kpn.p, c->rk_uniq.p, s));
    HIPCHK(hipMemcpyAsync(uq.data(), c->rk_uniq.p, m * 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
  }
  for (size_t i = 0; i < m; ++i) out[i] = nk_top_row{tc[i].idx, tc[i].sc, uq[i], 0};
  return (long)m;
}

long nk_top_abundant_neurons(nk_counter *c, size_t n, nk_top_row *out) {
  if (!c) return fail(NK_E_INVALID, "null counter");
  size_t m = std::min(n, c->pool);
  if (m && !out) return fail(NK_E_INVALID, "null output");
  if (!c->top_valid) {
    // fresh (or reset) neurons: all spike counts 0 -> indices in order, no k-mers
    for (size_t i = 0; i < m; ++i) out[i] = nk_top_row{i, 0, 0, 0};
    return (long)m;
  }
  if (m > c->top.size()) return extended_top(c, m, out);
  for (size_t i = 0; i < m; ++i) out[i] = c->top[i];
  return (long)m;
}

static DeltaArgs delta_args(nk_counter *c) {
  DeltaArgs d{};
  if (c->d_dirty || !c->d_cap) return d;  // keys == null: no delta
  d.keys = c->d_keys.p;
  d.vals = c->d_vals.p;
  d.mask = c->d_cap - 1;
  d.meta = c->d_meta.p;
  return d;
}

// room in the delta for `add` more distinct keys (load <= 1/2)
static int delta_reserve(nk_counter *c, uint64_t add, hipStream_t s) {
  int rc;
  if ((rc = c->d_meta.ensure(2))) return rc;
  uint64_t cap = c->d_cap ? c->d_cap : 1024;
  while (2 * (c->d_bound + add) > cap) cap <<= 1;
  if (c->d_dirty) {
    if (cap > c->d_cap) {
      if ((rc = c->d_keys.ensure(cap)) || (rc = c->d_vals.ensure(cap))) return rc;
      c->d_cap = cap;
    }
    DeltaArgs d{c->d_keys.p, c->d_vals.p, c->d_cap - 1, c->d_meta.p};
    HIPCHK(delta_clear(d, s));
    c->d_dirty = false;
    c->d_bound = 0;
  } else if (cap > c->d_cap) {  // grow: rehash into a new table
    DevBuf<unsigned long long> nk;
    DevBuf<uint32_t> nv;
    if ((rc = nk.ensure(cap)) || (rc = nv.ensure(cap))) return rc;
    DeltaArgs from = delta_args(c);
    DevBuf<unsigned long long> nm;
    if ((rc = nm.ensure(2))) return rc;
    DeltaArgs to{nk.p, nv.p, cap - 1, nm.p};
    HIPCHK(delta_clear(to, s));
    HIPCHK(delta_rehash(from, to, s));
    HIPCHK(hipMemcpyAsync(c->d_meta.p, nm.p, 16, hipMemcpyDeviceToDevice, s));
    HIPCHK(hipStreamSynchronize(s));
    std::swap(c->d_keys.p, nk.p);
    std::swap(c->d_keys.n, nk.n);
    std::swap(c->d_vals.p, nv.p);
    std::swap(c->d_vals.n, nv.n);
    c->d_cap = cap;
    nm.release();
    nk.release();
    nv.release();
  }
  return NK_OK;
}

static int need_exact(nk_counter *c) {
  if (!c) return fail(NK_E_INVALID, "null counter");
  if (!c->opts.exact_counts)
    return fail(NK_E_UNSUPPORTED, "the exact k-mer table needs nk_opts.exact_counts = 1");
  return NK_OK;
}

// ---------------------------------------------------------------------------
// Chunked accumulate over a growing resident input (GPU FASTX ingest)
// ---------------------------------------------------------------------------
struct StreamAcc {
  CountPlan cp;
  bool keep = false;  // Part keeps every record until acc_end (the uniques scan reads them)
};

// zero the accumulators and size the partition arena: Part keeps every
// record until acc_end (~est_bases bases, up to count_chunk()); Gen/Wide, and
// Part past count_chunk(), histogram each batch (<= batch_bases bases) as it
// is counted and drop its records (the uniques pass then rescans the input)
static int acc_begin(nk_counter *c, uint64_t est_bases, uint64_t batch_bases, StreamAcc &sa,
                     hipStream_t s) {
  int rc;
  ZeroList z{};
  z.ptr[z.n] = c->cur.p; z.bytes[z.n++] = c->pool * 8;
  const uint64_t B = (c->pool + kBinsPerBucket - 1) >> kBinBits;
  bool part_like = !c->w128 && c->k <= 32 && B <= (uint64_t)kMaxBuckets &&
                   !wide_bits_forced() && est_bases <= count_chunk(est_bases, c->pool, c->w128 || c->k > 32, arena_bytes(c));
  uint64_t est = part_like ? est_bases : std::min(est_bases, batch_bases);
  // segments per bucket: one per tile per launch; chunk-straddling tiles add a few
  uint64_t max_segs = n_tiles_for(std::max<uint64_t>(est, 1), kPartTile) + 4096;
  rc = plan_count(c, est, 4 * kPartTile, max_segs, sa.cp, z);
  if (rc == NK_E_OOM && part_like && est > batch_bases) {
    // the one-launch arena (sized from an estimate of the file's bases) did
    // not fit after all -- other handles took the memory since the check:
    // histogram batch by batch instead, as accumulate() does
    z = ZeroList{};
    z.ptr[z.n] = c->cur.p; z.bytes[z.n++] = c->pool * 8;
    part_like = false;
    est = std::min(est_bases, batch_bases);
    max_segs = n_tiles_for(std::max<uint64_t>(est, 1), kPartTile) + 4096;
    rc = plan_count(c, est, 4 * kPartTile, max_segs, sa.cp, z);
  }
  if (rc) return rc;
  z.ptr[z.n] = c->hist.p;  z.bytes[z.n++] = kHistBins * kHistCopies * 4;
  z.ptr[z.n] = c->stats.p; z.bytes[z.n++] = 16;
  c->lif_zeroed = true;
  c->k1b_lif = false;
  if (c->pool) HIPCHK(launch_zero(z, s));
  c->cur_fresh = false;
  sa.keep = sa.cp.path == CountPath::Part && part_like;
  c->part_used = sa.keep;
  c->gen_keep = false;
  c->gen_km = (sa.cp.path == CountPath::Gen || sa.cp.path == CountPath::Wide) ? sa.cp.km : -1;
  return NK_OK;
}

// count the windows that start in [pos_lo, pos_hi) of the resident input
static int acc_batch(nk_counter *c, StreamAcc &sa, const KmerInput &whole, uint64_t pos_lo,
                     uint64_t pos_hi, hipStream_t s) {
  if (pos_hi <= pos_lo || !c->pool) return NK_OK;
  const CountPlan &cp = sa.cp;
  KmerInput in = whole;
  in.tile_base = pos_lo / cp.tile;
  in.n_tiles = (pos_hi + cp.tile - 1) / cp.tile - in.tile_base;
  in.pos_lo = pos_lo;
  in.pos_hi = pos_hi;
  int rc = c->tile_rec.ensure(in.n_tiles);
  if (rc) return rc;
  in.tile_rec = c->tile_rec.p;
  HIPCHK(launch_tile_rec(in, cp.tile, c->tile_rec.p, s));
  switch (cp.path) {
    case CountPath::Part:
      if (sa.keep) {
        HIPCHK(launch_part(in, (int)c->k, c->canonical, c->pool, cp.pa, s));
        break;
      }
      [[fallthrough]];
    case CountPath::Gen:
    case CountPath::Wide:
      HIPCHK(batch_count(c, cp, in, s));
      break;
    case CountPath::Atomic:
      if (c->w128)
        HIPCHK(launch_count128(in, (int)c->k, c->canonical, c->pool, c->cur.p, s));
      else
        HIPCHK(launch_count(in, (int)c->k, c->canonical, c->pool, c->cur.p, s));
      break;
  }
  return NK_OK;
}

// bucket histograms (folded into the LIF kernel of the process call) and the
// bookkeeping of a finished input
static int acc_end(nk_counter *c, StreamAcc &sa, const KmerInput &whole, hipStream_t s) {
  int rc;
  if (sa.keep) {
    HIPCHK(launch_bucket_hist(sa.cp.pa, c->pool, sa.cp.slices, c->partials.p, s));
    c->pend_slices = sa.cp.slices;
    c->last_pa = sa.cp.pa;
  }
  c->last_in = whole;
  c->last_in.n_tiles = n_tiles_for(whole.n_bases, sa.cp.tile);
  c->have_input = true;
  c->top_valid = false;
  c->input_owned = whole.bases == c->in_bases.p;
  if ((rc = table_for_input(c, whole, s))) return rc;
  return NK_OK;
}

static size_t ingest_chunk_bytes() {
  const char *e = getenv("NK_INGEST_CHUNK");  // tests: small chunks exercise the carries
  size_t v = e ? (size_t)strtoull(e, nullptr, 10) : 0;
  if (v < 64) v = (size_t)64 << 20;
  return v;
}

// Parse a FASTA/FASTQ file on the device in chunks and count it as it arrives
// (src/spiking_hash.rs:277-486 semantics for the records; the caller runs the
// LIF rule).  *fallback: the file needs the host reader (a blank line between
// FASTQ records).
static int ingest_file(nk_counter *c, const char *path, bool *fallback) {
  *fallback = false;
  ChunkSource src;
  std::string err;
  int rc = src.open(path, err);
  if (rc) return fail(rc, "%s", err.c_str());
  (void)hipSetDevice(c->device);
  hipStream_t s = pick_stream(c, nullptr);
  // Three stages overlap: the reader thread fills pinned host buffer (c+2) % 3
  // with chunk c+2 while the copy stream moves chunk c+1 up and the count
  // stream parses and counts chunk c.  A FASTQ chunk's unfinished last record
  // (the carry) is copied on the device in front of the next chunk's bytes.
  size_t chunk = ingest_chunk_bytes();
  size_t room = std::max<size_t>(chunk / 8, 1 << 16);
  // (kept by the handle: pinning ~200 MB of host memory per call cost more
  // than reading a 100 MB file from the page cache)
  PinnedBuf *hb = c->ing_hb;
  for (int i = 0; i < 3; ++i)
    if ((rc = hb[i].ensure(chunk))) return rc;
  size_t have = src.read(hb[0].p, chunk);
  bool eof = have < chunk;
  if (!have) return fail(NK_E_PARSE, "empty file");
  const bool fastq = hb[0].p[0] == '@';
  if (hb[0].p[0] != '>' && !fastq)
    return fail(NK_E_PARSE, "unknown format: first byte is neither '>' nor '@'");
  std::future<size_t> next;
  auto prefetch = [&](int b) {
    next = std::async(std::launch::async, [&src, hb, b, chunk] { return src.read(hb[b].p, chunk); });
  };
  if (!eof) prefetch(1);
  // resident input: the file size bounds the bases of a plain file
  const uint64_t fsize = src.file_size();
  uint64_t cap_bases = (src.gz() ? 4 * fsize : fsize) + 64;
  if ((rc = c->in_bases.ensure(cap_bases + 16)) || (rc = c->in_offs.ensure(1025))) return rc;
  // device chunk buffers: [room for the carry | chunk | 16 B the parse's
  // aligned 16-B groups may read past the end]
  DevBuf<uint8_t> *draws[2] = {&c->ing_draw, &c->ing_draw2};
  DevBuf<uint8_t> &scratch = c->ing_scratch;
  DevBuf<IngestState> &dst = c->ing_dst;
  if ((rc = draws[0]->ensure(room + chunk + 16)) || (rc = draws[1]->ensure(room + chunk + 16)) ||
      (rc = scratch.ensure(ingest_scratch_bytes(room + chunk))) || (rc = dst.ensure(1)))
    return rc;
  if (!c->ing_cs) {
    HIPCHK(hipStreamCreateWithFlags(&c->ing_cs, hipStreamNonBlocking));
    for (hipEvent_t &e : c->ing_ev) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  }
  hipStream_t cs = c->ing_cs;
  hipEvent_t *ev_copied = c->ing_ev, *ev_free = c->ing_ev + 2;
  // every exit leaves no copy in flight into the handle's buffers
  struct CsDrain {
    hipStream_t cs;
    std::future<size_t> *next;
    ~CsDrain() {
      (void)hipStreamSynchronize(cs);
      if (next->valid()) next->wait();
    }
  } drain{cs, &next};
  bool used[2] = {false, false};
  // chunk bytes -> draws[b] + room on the copy stream, once the carry out of
  // that buffer and its parse are done
  auto upload = [&](int b, const uint8_t *h, size_t n) -> int {
    if (used[b]) HIPCHK(hipStreamWaitEvent(cs, ev_free[b], 0));
    HIPCHK(hipMemcpyAsync(draws[b]->p + room, h, n, hipMemcpyHostToDevice, cs));
    HIPCHK(hipEventRecord(ev_copied[b], cs));
    return NK_OK;
  };
  if ((rc = upload(0, hb[0].p, have))) return rc;
  int db = 0;        // the device buffer of this chunk
  uint64_t ci = 0;   // this chunk's number (host buffer ci % 3)
  size_t carry = 0;  // bytes of the previous chunk in front of this one
  IngestState st{};
  st.at_line_start = 1;
  HIPCHK(hipMemcpyAsync(dst.p, &st, sizeof st, hipMemcpyHostToDevice, s));
  StreamAcc sa;
  if ((rc = acc_begin(c, fastq ? cap_bases / 2 : cap_bases, chunk + room + 64, sa, s))) return rc;
  uint64_t counted = 0;  // windows below this start were counted
  // NK_INGEST_PROFILE=1: host time per phase, printed to stderr at the end
  // (parse = the device parse, waited for; count = the count enqueue; read =
  // waiting for the reader thread; carry = the carry copy's enqueue)
  static const bool prof = getenv("NK_INGEST_PROFILE") != nullptr;
  using clk = std::chrono::steady_clock;
  double t_parse = 0, t_count = 0, t_read = 0, t_carry = 0;
  uint64_t n_chunks = 0;
  auto since = [](clk::time_point a) {
    return std::chrono::duration<double, std::milli>(clk::now() - a).count();
  };
  struct ProfOut {
    bool on;
    double *p, *c, *r, *y;
    uint64_t *n;
    ~ProfOut() {
      if (on)
        fprintf(stderr, "[nk ingest] chunks %llu  parse %.1f ms  count enqueue %.1f ms  "
                        "read wait %.1f ms  carry %.1f ms\n",
                (unsigned long long)*n, *p, *c, *r, *y);
    }
  } prof_out{prof, &t_parse, &t_count, &t_read, &t_carry, &n_chunks};
  for (;;) {
    ++n_chunks;
    // the next chunk: wait for its bytes, send them up, start reading the one after
    size_t got = 0;
    if (!eof) {
      const clk::time_point t2 = clk::now();
      got = next.get();
      if (prof) t_read += since(t2);
      if ((rc = upload(db ^ 1, hb[(ci + 1) % 3].p, got))) return rc;
      if (got == chunk) prefetch((int)((ci + 2) % 3));  // chunk ci - 1's buffer: its H2D is done
    }
    const clk::time_point t0 = clk::now();
    const size_t len = carry + have;
    // capacity of the resident buffers for this chunk (grow: wait, copy, free)
    const uint64_t need_b = st.data_end + len + 64, need_r = st.n_rec + len / 2 + 4;
    if (need_b > c->in_bases.n || need_r + 1 > c->in_offs.n) {
      HIPCHK(hipStreamSynchronize(s));
      if (need_b > c->in_bases.n) {
        DevBuf<uint8_t> nb;
        if ((rc = nb.ensure(std::max<uint64_t>(need_b, 2 * c->in_bases.n)))) return rc;
        HIPCHK(hipMemcpy(nb.p, c->in_bases.p, st.data_end, hipMemcpyDeviceToDevice));
        std::swap(nb.p, c->in_bases.p);
        std::swap(nb.n, c->in_bases.n);
        nb.release();
      }
      if (need_r + 1 > c->in_offs.n) {
        DevBuf<uint64_t> no;
        if ((rc = no.ensure(std::max<uint64_t>(need_r + 1, 2 * c->in_offs.n)))) return rc;
        HIPCHK(hipMemcpy(no.p, c->in_offs.p, (st.n_rec + 1) * 8, hipMemcpyDeviceToDevice));
        std::swap(no.p, c->in_offs.p);
        std::swap(no.n, c->in_offs.n);
        no.release();
      }
    }
    const uint8_t *raw = draws[db]->p + room - carry;
    HIPCHK(hipStreamWaitEvent(s, ev_copied[db], 0));
    IngestBufs ib{c->in_bases.p, c->in_offs.p, c->in_bases.n, c->in_offs.n - 1, scratch.p};
    HIPCHK(fastq ? ingest_fastq(raw, len, eof, ib, dst.p, s) : ingest_fasta(raw, len, eof, ib, dst.p, s));
    HIPCHK(hipMemcpyAsync(&st, dst.p, sizeof st, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    if (prof) t_parse += since(t0);
    if (fastq && st.blank) {
      *fallback = true;
      return NK_OK;
    }
    // the carry goes in front of the next chunk's bytes (they sit at + room);
    // enqueued before this chunk's count so the next H2D into this buffer can start
    const bool last = eof || st.stop;
    size_t nc = 0;
    if (!last) {
      const clk::time_point t3 = clk::now();
      nc = fastq ? len - (size_t)st.consumed : 0;
      const uint8_t *from = raw + st.consumed;
      if (nc > room) {  // a record longer than the carry room: regrow both buffers
        HIPCHK(hipStreamSynchronize(cs));
        HIPCHK(hipStreamSynchronize(s));
        const size_t nroom = 2 * nc;
        DevBuf<uint8_t> nb[2];
        if ((rc = nb[0].ensure(nroom + chunk + 16)) || (rc = nb[1].ensure(nroom + chunk + 16)) ||
            (rc = scratch.ensure(ingest_scratch_bytes(nroom + chunk))))
          return rc;
        HIPCHK(hipMemcpy(nb[db ^ 1].p + nroom, draws[db ^ 1]->p + room, got, hipMemcpyDeviceToDevice));
        HIPCHK(hipMemcpy(nb[db ^ 1].p + nroom - nc, from, nc, hipMemcpyDeviceToDevice));
        for (int i = 0; i < 2; ++i) {
          std::swap(nb[i].p, draws[i]->p);
          std::swap(nb[i].n, draws[i]->n);
          nb[i].release();
        }
        room = nroom;
        used[0] = used[1] = false;
        HIPCHK(hipEventRecord(ev_copied[db ^ 1], s));
      } else {
        if (nc)
          HIPCHK(hipMemcpyAsync(draws[db ^ 1]->p + room - nc, from, nc, hipMemcpyDeviceToDevice, s));
        HIPCHK(hipEventRecord(ev_free[db], s));  // this buffer's parse and carry are done
        used[db] = true;
      }
      if (prof) t_carry += since(t3);
    }
    // count what is complete: every window of a FASTQ chunk's records (they
    // are whole); FASTA: windows that end inside the bases parsed so far
    const clk::time_point t1 = clk::now();
    KmerInput whole{};
    whole.bases = c->in_bases.p;
    whole.offsets = c->in_offs.p;
    whole.n_recs = st.n_rec;
    whole.n_bases = st.data_end;
    uint64_t hi = st.data_end;
    if (!fastq && !last) hi = st.data_end >= c->k - 1 ? st.data_end - (c->k - 1) : 0;
    if (st.n_rec && hi > counted) {
      if ((rc = acc_batch(c, sa, whole, counted, hi, s))) return rc;
      counted = hi;
    }
    if (prof) t_count += since(t1);
    if (last) {
      if ((rc = acc_end(c, sa, whole, s))) return rc;
      break;
    }
    db ^= 1;
    ++ci;
    carry = nc;
    have = got;
    eof = got < chunk;
  }
  return NK_OK;
}

// SpikingKmerCounter::process_sequence (src/spiking_hash.rs:203-273)
int nk_process_sequence(nk_counter *c, const uint8_t *seq, size_t len) {
  if (!c) return fail(NK_E_INVALID, "null counter");
  if (c->w128)
    return fail(NK_E_UNSUPPORTED, "process_sequence takes the reference's u64 keys (NK_KMER_COMPAT)");
  if (len && !seq) return fail(NK_E_INVALID, "null sequence");
  if (int rc0 = whole_pool(c)) return rc0;
  if (len < c->k) return NK_OK;  // :205-207: no k-mers, no LIF step
  c->k1b_lif = false;
  if (c->pool == 0)
    return fail(NK_E_INVALID, "pool_size 0 with k-mers present (the reference panics on % 0)");
  hipStream_t s;
  // counts / kmer_per_neuron of the last process call first (its input is
  // about to be replaced by this sequence in the handle's input buffer)
  int rc = table_ready(c, &s);
  if (rc) return rc;
  if (c->cur_in_wire)
    return fail(NK_E_INVALID, "the currents are in the wire vector until nk_finalize_export");
  if ((rc = settle_state(c, s)) || (rc = materialize(c, true, s)) || (rc = fold_pending(c, s)))
    return rc;
  if ((rc = c->in_bases.ensure(len + 16)) || (rc = c->in_offs.ensure(2)) ||
      (rc = c->x_n.ensure(8)) || (rc = c->kpn.ensure(c->pool)))
    return rc;
  const uint64_t offs[2] = {0, (uint64_t)len};
  HIPCHK(hipMemcpyAsync(c->in_bases.p, seq, len, hipMemcpyHostToDevice, s));
  HIPCHK(hipMemcpyAsync(c->in_offs.p, offs, 16, hipMemcpyHostToDevice, s));
  KmerInput in{};
  in.bases = c->in_bases.p;
  in.offsets = c->in_offs.p;
  in.n_recs = 1;
  in.n_bases = len;
  in.n_tiles = n_tiles_for(len, kTile);
  if ((rc = c->x_tile_rec.ensure(in.n_tiles)) || (rc = c->x_keys.ensure(len))) return rc;
  in.tile_rec = c->x_tile_rec.p;
  // this step reads the state: materialise lazily-zero buffers
  if ((rc = materialize(c, true, s)) || (rc = materialize(c, false, s))) return rc;
  if (!c->kpn_valid) {
    HIPCHK(hipMemsetAsync(c->kpn.p, 0, c->pool * 4, s));
    c->kpn_valid = true;
  }
  if (!c->touched.n) {
    if ((rc = c->touched.ensure(c->pool))) return rc;
    HIPCHK(hipMemsetAsync(c->touched.p, 0, c->pool, s));  // seq_lif keeps it zero
  }
  const uint64_t add = len - c->k + 1;
  if ((rc = delta_reserve(c, add, s))) return rc;
  c->d_bound += add;
  HIPCHK(hipMemsetAsync(c->x_n.p, 0, 8, s));  // [0] only: [1] is the sorted table's size
  HIPCHK(launch_tile_rec(in, kTile, c->x_tile_rec.p, s));
  HIPCHK(exact_keys(in, (int)c->k, c->canonical, c->x_keys.p, c->x_n.p, s));
  HIPCHK(seq_accumulate(c->x_keys.p, c->x_n.p, add, c->pool, (unsigned long long *)c->cur.p,
                        c->touched.p, delta_args(c), table_view(c), s));
  ZeroList z{};
  z.ptr[0] = c->hist.p;  z.bytes[0] = kHistBins * kHistCopies * 4;
  z.ptr[1] = c->stats.p; z.bytes[1] = 16;
  z.n = 2;
  HIPCHK(launch_zero(z, s));
  c->sc8_ok = false;
  HIPCHK(seq_lif(c->pool, (unsigned long long *)c->cur.p, c->touched.p, c->kpn.p, c->v.p, c->r.p,
                 c->sc.p, c->thr, c->leak, c->refr, c->hist.p, c->stats.p, s));
  c->have_input = false;  // no uniques pass: the column comes from kmer_per_neuron
  const uint64_t want = std::min<uint64_t>(c->opts.top_n, c->pool);
  if ((rc = finish_top(c, want, false, want != 0, true, s))) return rc;
  c->top_valid = true;
  return NK_OK;
}

// the table for a query: built now from the last input when it is lazy
static int table_ready(nk_counter *c, hipStream_t *s) {
  if (!c) return fail(NK_E_INVALID, "null counter");
  (void)hipSetDevice(c->device);
  *s = pick_stream(c, nullptr);
  return ensure_table(c, *s);
}

int nk_get_counts(nk_counter *c, const uint64_t *kmers, size_t n, uint32_t *out,
                  uint8_t *present) {
  hipStream_t s;
  int rc = table_ready(c, &s);
  if (rc) return rc;
  if (c->w128) return fail(NK_E_INVALID, "128-bit keys: use nk_get_counts128");
  if (n && (!kmers || !out || !present)) return fail(NK_E_INVALID, "null argument");
  if (!n) return NK_OK;
  if (!c->exact_built && c->d_dirty) {  // empty table (fresh or reset counter)
    memset(out, 0, n * 4);
    memset(present, 0, n);
    return NK_OK;
  }
  if ((rc = c->x_q.ensure(n)) || (rc = c->x_out.ensure(n)) || (rc = c->x_pres.ensure(n)))
    return rc;
  HIPCHK(hipMemcpyAsync(c->x_q.p, kmers, n * 8, hipMemcpyHostToDevice, s));
  HIPCHK(exact_lookup2(table_view(c), delta_args(c), c->x_q.p, n, c->x_out.p, c->x_pres.p, s));
  std::vector<uint32_t> pres(n);
  HIPCHK(hipMemcpyAsync(out, c->x_out.p, n * 4, hipMemcpyDeviceToHost, s));
  HIPCHK(hipMemcpyAsync(pres.data(), c->x_pres.p, n * 4, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  for (size_t i = 0; i < n; ++i) present[i] = pres[i] ? 1 : 0;
  return NK_OK;
}

int nk_get_count(nk_counter *c, uint64_t kmer, uint32_t *out, int *present) {
  if (!out || !present) return fail(NK_E_INVALID, "null argument");
  uint8_t p = 0;
  int rc = nk_get_counts(c, &kmer, 1, out, &p);
  *present = p;
  return rc;
}

int nk_get_counts128(nk_counter *c, const uint64_t *kmers2, size_t n, uint32_t *out,
                     uint8_t *present) {
  hipStream_t s;
  int rc = table_ready(c, &s);
  if (rc) return rc;
  if (!c->w128) return fail(NK_E_INVALID, "64-bit keys: use nk_get_counts");
  if (n && (!kmers2 || !out || !present)) return fail(NK_E_INVALID, "null argument");
  if (!n) return NK_OK;
  if (!c->exact_built) {  // empty table (fresh or reset counter)
    memset(out, 0, n * 4);
    memset(present, 0, n);
    return NK_OK;
  }
  if ((rc = c->x_q.ensure(2 * n)) || (rc = c->x_out.ensure(n)) || (rc = c->x_pres.ensure(n)))
    return rc;
  HIPCHK(hipMemcpyAsync(c->x_q.p, kmers2, n * 16, hipMemcpyHostToDevice, s));
  HIPCHK(exact_lookup128(c->x_uniq.p, c->x_cnt.p, c->x_n.p + 1, c->x_q.p, n, c->x_out.p,
                         c->x_pres.p, s));
  std::vector<uint32_t> pres(n);
  HIPCHK(hipMemcpyAsync(out, c->x_out.p, n * 4, hipMemcpyDeviceToHost, s));
  HIPCHK(hipMemcpyAsync(pres.data(), c->x_pres.p, n * 4, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  for (size_t i = 0; i < n; ++i) present[i] = pres[i] ? 1 : 0;
  return NK_OK;
}

long nk_distinct_kmers(nk_counter *c) {
  hipStream_t s;
  int rc = table_ready(c, &s);
  if (rc) return rc;
  HIPCHK(hipStreamSynchronize(s));
  unsigned long long n = 0, m[2] = {0, 0};
  // grouped: [6] (the span [1] holds the zero-count tails of the buckets)
  if (c->exact_built) HIPCHK(hipMemcpy(&n, c->x_n.p + (c->x_grouped ? 6 : 1), 8, hipMemcpyDeviceToHost));
  if (!c->d_dirty) HIPCHK(hipMemcpy(m, c->d_meta.p, 16, hipMemcpyDeviceToHost));
  // meta[1]: keys process_sequence added that the sorted table did not hold
  // (k_seq_accumulate; the ~0 key included)
  return (long)(n + m[1]);
}

uint32_t nk_exact_owner(uint64_t kmer, uint32_t world) { return world ? exact_owner(kmer, world) : 0; }

int nk_exact_partition(nk_counter *c, uint32_t world, uint64_t *send_counts,
                       const uint64_t **d_keys, const uint32_t **d_counts, void *stream) {
  int rc = need_exact(c);
  if (rc) return rc;
  if (c->w128) return fail(NK_E_UNSUPPORTED, "the multi-GPU exact table takes NK_KMER_COMPAT keys");
  if (!world || world > 4096) return fail(NK_E_INVALID, "world must be in 1..4096");
  if (!send_counts || !d_keys || !d_counts) return fail(NK_E_INVALID, "null argument");
  if (!c->exact_built) return fail(NK_E_INVALID, "no exact table: run a process/accumulate call first");
  if (c->d_bound)
    return fail(NK_E_UNSUPPORTED, "process_sequence additions are not partitioned across ranks");
  (void)hipSetDevice(c->device);
  hipStream_t s = pick_stream(c, stream);
  unsigned long long n = 0;
  HIPCHK(hipMemcpyAsync(&n, c->x_n.p + 1, 8, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  if ((rc = c->xp_keys.ensure(std::max<uint64_t>(n, 1))) || (rc = c->xp_cnt.ensure(std::max<uint64_t>(n, 1))) ||
      (rc = c->xp_ctr.ensure(world)))
    return rc;
  std::vector<unsigned long long> cnt(world, 0);
  if (n) {
    HIPCHK(hipMemsetAsync(c->xp_ctr.p, 0, world * 8, s));
    HIPCHK(exact_owner_hist(c->x_uniq.p, c->x_n.p + 1, n, world, c->xp_ctr.p, s,
                            c->x_grouped ? c->x_cnt.p : nullptr));
    HIPCHK(hipMemcpyAsync(cnt.data(), c->xp_ctr.p, world * 8, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    std::vector<unsigned long long> cur(world);
    unsigned long long run = 0;
    for (uint32_t r = 0; r < world; ++r) {
      cur[r] = run;
      run += cnt[r];
    }
    HIPCHK(hipMemcpyAsync(c->xp_ctr.p, cur.data(), world * 8, hipMemcpyHostToDevice, s));
    HIPCHK(exact_owner_scatter(c->x_uniq.p, c->x_cnt.p, c->x_n.p + 1, n, world, c->xp_ctr.p,
                               c->xp_keys.p, c->xp_cnt.p, s, c->x_grouped));
    HIPCHK(hipStreamSynchronize(s));  // cur[] is host memory the copy reads
  }
  for (uint32_t r = 0; r < world; ++r) send_counts[r] = cnt[r];
  *d_keys = c->xp_keys.p;
  *d_counts = c->xp_cnt.p;
  return NK_OK;
}

int nk_exact_adopt(nk_counter *c, const uint64_t *d_keys, const uint32_t *d_counts, size_t n,
                   void *stream) {
  int rc = need_exact(c);
  if (rc) return rc;
  if (c->w128) return fail(NK_E_UNSUPPORTED, "the multi-GPU exact table takes NK_KMER_COMPAT keys");
  if (n && (!d_keys || !d_counts)) return fail(NK_E_INVALID, "null argument");
  (void)hipSetDevice(c->device);
  hipStream_t s = pick_stream(c, stream);
  const int end_bit = c->k <= 32 ? (int)(2 * c->k) : 64;
  const uint64_t nn = std::max<uint64_t>(n, 1);
  if ((rc = c->x_n.ensure(8)) || (rc = c->x_sorted.ensure(nn)) || (rc = c->x_cs.ensure(nn)) ||
      (rc = c->x_uniq.ensure(nn)) || (rc = c->x_cnt.ensure(nn)) || (rc = c->kpn.ensure(c->pool)) ||
      (rc = c->x_tmp.ensure(exact_merge_temp_bytes(nn, end_bit))))
    return rc;
  HIPCHK(exact_merge_pairs(d_keys, d_counts, n, end_bit, c->x_sorted.p, c->x_cs.p, c->x_uniq.p,
                           c->x_cnt.p, c->x_n.p + 1, c->x_tmp.p, c->x_tmp.n, s));
  if ((rc = table_kpn(c, c->x_uniq.p, c->x_n.p + 1, n, 1, s))) return rc;
  HIPCHK(hipStreamSynchronize(s));  // the caller may free the received buffers
  c->x_grouped = false;
  c->exact_built = true;
  c->kpn_valid = true;
  c->kpn_global = true;
  c->d_dirty = true;
  c->d_bound = 0;
  return NK_OK;
}

uint32_t *nk_device_kmer_per_neuron(nk_counter *c) {
  if (!c || !c->pool) return nullptr;
  hipStream_t s;
  if (table_ready(c, &s)) return nullptr;
  if (!c->kpn_valid) {
    (void)hipSetDevice(c->device);
    if (c->kpn.ensure(c->pool) || hipMemset(c->kpn.p, 0, c->pool * 4) != hipSuccess) return nullptr;
    c->kpn_valid = true;
  }
  return c->kpn.p;
}

int nk_copy_kmer_per_neuron(nk_counter *c, uint32_t *out, size_t n) {
  hipStream_t s;
  int rc = table_ready(c, &s);
  if (rc) return rc;
  if (n != c->pool) return fail(NK_E_INVALID, "n (%zu) must equal pool_size (%zu)", n, c->pool);
  if (!n) return NK_OK;
  if (!out) return fail(NK_E_INVALID, "null argument");
  if (!c->kpn_valid) {
    memset(out, 0, n * 4);
    return NK_OK;
  }
  (void)hipSetDevice(c->device);
  HIPCHK(hipStreamSynchronize(pick_stream(c, nullptr)));
  HIPCHK(hipMemcpy(out, c->kpn.p, n * 4, hipMemcpyDeviceToHost));
  return NK_OK;
}

uint64_t nk_total_spikes(const nk_counter *c) { return c ? c->total_spikes : 0; }
double nk_energy_used(const nk_counter *c) {
  return c ? (double)c->total_energy / 1000.0 : 0.0;
}
void nk_set_steps(nk_counter *c, uint64_t steps) {
  if (c) c->steps = steps;
}
uint64_t nk_get_steps(const nk_counter *c) { return c ? c->steps : 0; }
size_t nk_pool_size(const nk_counter *c) { return c ? c->pool : 0; }
size_t nk_k(const nk_counter *c) { return c ? c->k : 0; }
int nk_use_canonical(const nk_counter *c) { return c ? c->canonical : 0; }
int nk_settle(nk_counter *c, void *stream) {
  if (!c) return fail(NK_E_INVALID, "null counter");
  (void)hipSetDevice(c->device);
  hipStream_t s = pick_stream(c, stream);
  return settle_state(c, s);
}

uint64_t *nk_device_currents(nk_counter *c) {
  if (!c) return nullptr;
  if (c->cur_in_wire) {
    fail(NK_E_INVALID, "the currents are in the wire vector until nk_finalize_export");
    return nullptr;
  }
  // lazily-reset currents / K1b partials pending / a derived state (the caller
  // may change the counts it is a function of: written out first)
  c->k1b_lif = false;
  if (c->cur_fresh || c->pend_slices || c->state_derived) {
    (void)hipSetDevice(c->device);
    hipStream_t s = pick_stream(c, nullptr);
    if (settle_state(c, s) || materialize(c, true, s) || fold_pending(c, s) ||
        hipStreamSynchronize(s) != hipSuccess)
      return nullptr;
  } else if (c->last_s && c->last_s == c->own_stream) {
    // the last call ran on the handle's private stream, which the caller
    // cannot order against: wait for it (a caller stream stays the caller's)
    (void)hipSetDevice(c->device);
    if (hipStreamSynchronize(c->own_stream) != hipSuccess) {
      fail(NK_E_DEVICE, "hipStreamSynchronize failed");
      return nullptr;
    }
  }
  return c->cur.p;
}

int nk_copy_currents(nk_counter *c, uint64_t *out, size_t n) { return copy_out(c, c->cur, out, n); }
int nk_copy_spike_counts(nk_counter *c, uint64_t *out, size_t n) {
  return copy_out(c, c->sc, out, n);
}
int nk_copy_voltages(nk_counter *c, float *out, size_t n) { return copy_out(c, c->v, out, n); }
int nk_copy_refractory(nk_counter *c, uint32_t *out, size_t n) {
  return copy_out(c, c->r, out, n);
}

int nk_diag_hash_ms(int device, uint64_t n_keys, uint64_t pool, int reps, float *ms) {
  return nk_diag_hash_ms_w(device, n_keys, pool, 64, reps, ms);
}

int nk_diag_hash_ms_w(int device, uint64_t n_keys, uint64_t pool, int width, int reps, float *ms) {
  if (!ms || !n_keys || !pool || pool >= (1ull << 30) || reps < 1 || (width != 64 && width != 128))
    return fail(NK_E_INVALID, "nk_diag_hash_ms: n_keys, pool in [1, 2^30), width 64|128, reps >= 1, ms");
  if (hipSetDevice(device) != hipSuccess) return fail(NK_E_NO_DEVICE, "hipSetDevice failed");
  uint32_t *out = nullptr;
  hipStream_t s = nullptr;
  hipEvent_t a = nullptr, b = nullptr;
  int rc = NK_OK;
  float best = 1e30f;
  if (hipMalloc(&out, diag_hash_out_words(n_keys) * 4) != hipSuccess) return fail(NK_E_OOM, "hipMalloc");
  if (hipStreamCreate(&s) != hipSuccess || hipEventCreate(&a) != hipSuccess ||
      hipEventCreate(&b) != hipSuccess) {
    rc = fail(NK_E_DEVICE, "stream/event creation failed");
  }
  for (int i = 0; rc == NK_OK && i < reps + 1; ++i) {  // + 1 untimed warm-up
    float t = 0.0f;
    if (hipEventRecord(a, s) != hipSuccess || launch_diag_hash(n_keys, pool, out, s, width) != hipSuccess ||
        hipEventRecord(b, s) != hipSuccess || hipEventSynchronize(b) != hipSuccess ||
        hipEventElapsedTime(&t, a, b) != hipSuccess)
      rc = fail(NK_E_DEVICE, "diag hash kernel failed");
    else if (i > 0 && t < best)
      best = t;
  }
  if (a) (void)hipEventDestroy(a);
  if (b) (void)hipEventDestroy(b);
  if (s) (void)hipStreamDestroy(s);
  (void)hipFree(out);
  if (rc == NK_OK) *ms = best;
  return rc;
}

int nk_set_stage_timing(nk_counter *c, uint32_t level) {
  if (!c) return fail(NK_E_INVALID, "null counter");
  if (level > 3) return fail(NK_E_INVALID, "stage timing level must be 0, 1, 2 or 3");
  c->opts.stage_timing = level;
  return NK_OK;
}

int nk_count_spans(nk_counter *c, float *ms, int cap) {
  if (!c || (!ms && cap > 0) || cap < 0) return fail(NK_E_INVALID, "null argument");
  (void)hipSetDevice(c->device);
  const uint64_t have = std::min<uint64_t>(c->span_calls, nk_counter::kCountRing);
  const int n = (int)std::min<uint64_t>(have, (uint64_t)cap);
  if (!n) return 0;
  std::vector<unsigned long long> h(2 * nk_counter::kCountRing);
  if (c->last_s) HIPCHK(hipStreamSynchronize(c->last_s));
  HIPCHK(hipMemcpy(h.data(), c->span.p, h.size() * 8, hipMemcpyDeviceToHost));
  for (int i = 0; i < n; ++i) {
    const uint64_t call = c->span_calls - (uint64_t)n + (uint64_t)i;
    const unsigned long long *w = &h[2 * (call % nk_counter::kCountRing)];
    ms[i] = w[1] > w[0] ? (float)((double)(w[1] - w[0]) * 1e-5) : -1.0f;  // 10 ns ticks
  }
  return n;
}

int nk_count_history(const nk_counter *c, float *ms, int cap) {
  if (!c || !ms || cap <= 0) return 0;
  (void)hipSetDevice(c->device);
  const uint64_t n = std::min<uint64_t>({(uint64_t)cap, c->cnt_calls, (uint64_t)nk_counter::kCountRing});
  for (uint64_t i = 0; i < n; ++i) {
    const uint64_t call = c->cnt_calls - n + i;
    const auto &pr = c->cnt_ev[call % nk_counter::kCountRing];
    float t = 0.0f;
    if (hipEventSynchronize(pr[1]) != hipSuccess || hipEventElapsedTime(&t, pr[0], pr[1]) != hipSuccess)
      t = -1.0f;
    ms[i] = t;
  }
  return (int)n;
}

int nk_last_timings(const nk_counter *c, const char **names, float *ms, int cap) {
  if (!c) return 0;
  if (c->timing_pending) {  // logically const: fills the cache of the last call's timings
    nk_counter *m = const_cast<nk_counter *>(c);
    (void)hipSetDevice(m->device);
    const bool wc = m->timing_pending == 2;
    m->timing_pending = 0;
    if (hipEventSynchronize(m->ev[6]) == hipSuccess) collect_timings_now(m, wc);
    else std::fill(m->stage_ms, m->stage_ms + kStages, 0.0f);
  }
  int n = std::min(cap, c->n_stage);
  for (int i = 0; i < n; ++i) {
    if (names) names[i] = full_timing(c) ? kStageNames[i] : kStageNamesLight[i];
    if (ms) ms[i] = c->stage_ms[i];
  }
  return n;
}

}  // extern "C"
