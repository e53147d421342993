// nk_handle.h — the counter handle (struct nk_counter) and the host
// functions its translation units share (internal; not ABI).  The host side
// behind the C ABI (include/neurokmer.h) is split by path:
//   nk_counter.cpp      handle lifecycle, lazy state, accessors, timings
//   nk_count.cpp        the count (plan, partition launches, batches)
//   nk_finish.cpp       LIF, top-N selection, uniques, readback, process calls
//   nk_export.cpp       the multi-GPU finish pieces (wire, export, merge, slices)
//   nk_table_host.cpp   the exact k-mer table, process_sequence, extended top rows
//   nk_ingest_host.cpp  file ingest (device FASTA/FASTQ parse, host FASTQ extraction)
// Mirrors SpikingKmerCounter (src/spiking_hash.rs:16-715) with all per-neuron
// state resident in HBM of one MI355X:
//   currents u64[P] | voltage f32[P] | refractory u32[P] | spike_count u64[P]
#pragma once
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
#include "nk_fqhost.h"
#include "nk_ingest.h"
#include "nk_reader.h"
#include "nk_kernels.h"

using namespace nk;

// everything below is internal to libneurokmer.so (not exported)
#pragma GCC visibility push(hidden)

// K1b workgroups per batch (one 128 KiB-LDS workgroup per CU: one round on 256 CUs)
#ifndef NK_K1B_WGS
#define NK_K1B_WGS 256
#endif

extern thread_local std::string g_err;
extern std::atomic<uint64_t> g_next_uid;  // handle ids (nk_counter::uid)
// sets the thread's last error (nk_last_error) and returns code
int fail(int code, const char *fmt, ...);

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
extern const char *kStageNames[7];
// default (opts.stage_timing == 0): events only around the count kernel and at
// both ends; an event between two kernels idles the GPU for ~6 us on MI355X
constexpr int kStagesLight = 4;
extern const char *kStageNamesLight[4];

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
  // host FASTQ extraction (nk_fqhost.h): record ends per pinned buffer, the
  // event of each buffer's last H2D, the parser threads
  PinnedBuf ing_he[3];
  hipEvent_t fq_ev[3] = {};
  FqScratch fq_scratch;
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
  // pipelined split (split_pipelined): w_snap[g][bucket] = the records
  // reserved after k_gen_split launch g
  static constexpr int kSplitMax = 64;
  DevBuf<unsigned long long> w_snap;
  // overflow target of a write-through K1b (PartArgs::out), kept zero
  DevBuf<unsigned long long> ovf;
  size_t ovf_zeroed = 0;  // entries known zero
  uint32_t pend_slices = 0;  // K1b partials not yet folded into cur (fused into LIF)
  // K1b left to the next count's K1a (opts.defer_hist, k_part_fused): 0 none;
  // 1 pending in the device's slot (nk_count.cpp: hist_*); 2 enqueued (taken
  // by another handle's fused count, or run standalone), its end marked by
  // hist_ev; 3 being taken.  Read and written under nk_count.cpp's slot lock.
  int hist_state = 0;
  uint32_t hist_slices = 0;
  hipEvent_t hist_ev = nullptr;
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
  // every operation enqueued so far is known complete (nk_finalize saw its
  // readback, which the finish's last kernel writes after its last access):
  // the next stream switch needs no wait (pick_stream)
  bool quiescent = false;
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

enum class CountPath { Atomic, Part, Gen, Wide };
struct CountPlan {
  CountPath path = CountPath::Atomic;
  int km = 0;               // key mode of k_part_gen
  uint64_t tile = kTile;
  uint32_t slices = 0;      // K1b slices (Part, or > 1: partials; else adds into cur)
  PartArgs pa{};            // the 32768-bin buckets k_bucket_hist reads
  GenPartArgs ga{};         // Gen: same arrays as pa; Wide: the coarse buckets
};

// ---- shared host functions (definitions in the files named above) ----
bool full_timing(const nk_counter *c);
bool count_timing(const nk_counter *c);
hipError_t mark(nk_counter *c, int i, hipStream_t s);
uint64_t cost_fixed(double cost);
hipStream_t pick_stream(nk_counter *c, void *s);
void record_order(nk_counter *c, hipStream_t s);
int zero_state_on(nk_counter *c, hipStream_t);
int settle_state(nk_counter *c, hipStream_t s);
SpikeSrc spike_src(const nk_counter *c, uint64_t lo);
int whole_pool(nk_counter *c);
int materialize(nk_counter *c, bool currents, hipStream_t s);
int fold_pending(nk_counter *c, hipStream_t s);
int zero_state(nk_counter *c);
int table_kpn(nk_counter *c, const uint64_t *uniq, const unsigned long long *n_uniq,
                     uint64_t max_n, int wpk, hipStream_t s);
TableView table_view(const nk_counter *c);
int build_sorted(nk_counter *c, const KmerInput &in0, hipStream_t s);
uint32_t xbin_bits();
bool grouped_ok(const nk_counter *c, uint64_t n_bases);
uint64_t side_cap_for(uint64_t n_bases);
int keyed_args(nk_counter *c, uint64_t n_bases, PartArgs &pa, bool own, hipStream_t s);
int build_grouped(nk_counter *c, const KmerInput &in0, const PartArgs *keyed, hipStream_t s);
int build_exact(nk_counter *c, const KmerInput &in, hipStream_t s,
                       const PartArgs *keyed = nullptr);
int table_for_input(nk_counter *c, const KmerInput &in, hipStream_t s,
                           const PartArgs *keyed = nullptr);
int ensure_table(nk_counter *c, hipStream_t s);
int wide_bits_forced();
bool atomic_forced();
uint64_t count_chunk(uint64_t n_bases = 0, uint64_t pool = 0, bool wide = false,
                            uint64_t held = 0);
uint64_t arena_bytes(const nk_counter *c);
int plan_count(nk_counter *c, uint64_t est_bases, uint64_t slack, uint64_t max_segs,
                      CountPlan &cp, ZeroList &z, bool keep_gen = false, int part_bits = 0);
hipError_t gen_hist(nk_counter *c, const CountPlan &cp, bool defer_partials, hipStream_t s);
// the deferred K1b (opts.defer_hist): hist_ready before anything reads this
// handle's partials (runs it, or waits for the fused count that took it);
// hist_arena before this handle's next count rewrites its records; hist_void
// when a reset voids the partials; hist_forget when the handle is freed
int hist_ready(nk_counter *c, hipStream_t s);
int hist_arena(nk_counter *c, hipStream_t s);
void hist_void(nk_counter *c);
void hist_forget(nk_counter *c);
uint32_t split_launches(uint64_t n_tiles);
hipError_t split_pipelined(nk_counter *c, const CountPlan &cp, const KmerInput &in, uint32_t G,
                                  hipStream_t s);
hipError_t gen_count(nk_counter *c, const CountPlan &cp, const KmerInput &in, hipStream_t s,
                            bool pipeline = false);
hipError_t batch_count(nk_counter *c, const CountPlan &cp, const KmerInput &in, hipStream_t s);
uint32_t env_u32(const char *name, uint32_t dflt);
int accumulate(nk_counter *c, const uint8_t *d_bases, const uint64_t *d_offs,
                      size_t n_recs, size_t n_bases, void *stream, bool defer_partials,
                      uint64_t first_pos = 0);
int refine_threshold(nk_counter *c, uint64_t want, uint64_t max_sc, TopState &st,
                            hipStream_t s, uint64_t lo = 0, uint64_t n = ~0ull);
LifParams lif_params(const nk_counter *c, int streaming);
int lif_table(nk_counter *c, const LifParams &lp, hipStream_t s);
int lif_prepare(nk_counter *c, int streaming, LifParams &lp, hipStream_t s);
bool k1b_lif_holds(const nk_counter *c, const LifParams &lp, uint32_t fuse_want,
                          const uint32_t *wire);
int enqueue_lif(nk_counter *c, int streaming, uint32_t fuse_want, bool part,
                       hipStream_t s, const uint32_t *wire = nullptr);
int enqueue_select(nk_counter *c, uint64_t want, hipStream_t s, uint64_t lo = 0,
                          uint64_t n = ~0ull);
PostArgs post_args(nk_counter *c, bool rescan);
int enqueue_uniques(nk_counter *c, uint32_t m, bool rescan, bool post_done,
                           hipStream_t s);
int enqueue_readback(nk_counter *c, uint32_t m, bool uniq, hipStream_t s,
                            const uint32_t *flag3 = nullptr, const uint32_t *uniq_src = nullptr);
int wait_readback(nk_counter *c, hipStream_t s);
bool top_fused(const nk_counter *c, uint64_t want);
int lif_top_uniques(nk_counter *c, int streaming, bool use_kpn, hipStream_t s,
                           const uint32_t *wire = nullptr);
int finish_top(nk_counter *c, uint64_t want, bool fused, bool uniq, bool use_kpn,
                      hipStream_t s);
int settle_top(nk_counter *c, uint64_t want, bool uniq, bool use_kpn, bool account,
                      hipStream_t s);
void collect_timings(nk_counter *c, bool with_count);
void collect_timings_now(nk_counter *c, bool with_count);
int process_device(nk_counter *c, const uint8_t *d_bases, const uint64_t *d_offs,
                          size_t n_recs, size_t n_bases, void *stream, int streaming);
int check_offsets(const uint64_t *offs, size_t n_recs);
bool any_kmer(const uint64_t *offs, size_t n_recs, size_t k);
int process_host(nk_counter *c, const uint8_t *bases, const uint64_t *offs, size_t n_recs,
                        int streaming);
int process_file(nk_counter *c, const char *path, int streaming);
int merge_keys(nk_counter *c, const MergeSrc &src, uint64_t max_keys, int *complete,
                      hipStream_t s);
uint64_t merge_cap(uint64_t max_keys);
int enqueue_merge(nk_counter *c, const MergeSrc &src, uint64_t max_keys, uint32_t m,
                         hipStream_t s, bool sep = false);
int finalize_slice_impl(nk_counter *c, int streaming, const void *d_slice, int slice_bits,
                               size_t lo, size_t hi, uint64_t *d_seg, size_t seg_rows,
                               hipStream_t s, bool run_lif);
long extended_top(nk_counter *c, size_t m, nk_top_row *out);
DeltaArgs delta_args(nk_counter *c);
int delta_reserve(nk_counter *c, uint64_t add, hipStream_t s);
int need_exact(nk_counter *c);
size_t ingest_chunk_bytes();
int ingest_file(nk_counter *c, const char *path, bool *fallback);
int table_ready(nk_counter *c, hipStream_t *s);

#pragma GCC visibility pop
