// nk_kernels.h — host-side launchers of the gfx950 kernels (internal; not ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace nk {

constexpr int kTile = 4096;      // k-mer start positions per workgroup
constexpr int kBlock = 256;      // threads per workgroup (4 waves)
constexpr int kHistBins = 4096;  // spike-count histogram for top-N selection
constexpr int kHistCopies = 8;   // one per XCD group of LIF blocks
constexpr int kMaxTopN = 1024;
// partitioned count
constexpr int kPartTile = 8192;       // positions per K1a workgroup
constexpr int kPartBlock = 512;       // threads per K1a workgroup
constexpr int kBinBits = 15;
constexpr int kBinsPerBucket = 1 << kBinBits;  // 32768 u32 bins = 128 KiB LDS
constexpr int kMaxBuckets = 512;      // pool <= 16,777,216 takes the partitioned path
constexpr uint32_t kSubShift = 3;       // K1a sub-regions per bucket: one per XCD (PartArgs::sub_shift)
constexpr uint64_t kSubMinBuckets = 128;  // ... when the Part count has more buckets than this
constexpr int kHistBlock = 1024;

struct LifParams {
  uint64_t steps;
  float thr;
  float leak;
  uint32_t refr;
  int32_t skip_zero;
};

struct LifEntry {  // closed-form result for a fresh neuron (v = 0, r = 0)
  uint64_t spikes;
  float v;
  uint32_t r;
};

// Where a top-N pass reads the spike counts: the materialised array, or --
// after a LIF from the reset state, whose outcome is a function of each
// neuron's count alone (the "derived" state: v / refractory / spike counts
// are not written) -- from the counts through the closed form.
struct SpikeSrc {
  const uint8_t *sc8;   // non-null: min(spikes, 255) per neuron, read first
  const uint64_t *sc;   // non-null: materialised spike counts
  const uint64_t *cur;  // derived: the counts
  const LifEntry *tbl;  // closed-form rows of fresh neurons (counts < tbl_n)
  int tbl_n;
  LifParams lp;         // of the LIF that produced the state
};

struct TopState {
  uint64_t T;          // spike count of the N-th row
  uint64_t n_above;    // rows with spikes > T (all selected)
  uint64_t need;       // rows with spikes == T to take, lowest index first
  uint64_t emit_above; // device-side cursor
  uint32_t refine;     // 1: T lies in the overflow bin, exact radix refine needed
  uint32_t pad;
};

struct TopCand {
  uint64_t idx;
  uint64_t sc;
};

// What k_top_post derives from the final top rows (set sizing for uniques).
struct PostArgs {
  uint64_t set_alloc;
  const uint32_t *overflow;  // per bucket (partitioned count) or null
  int part;
  uint64_t *set_mask;
  uint32_t *tbuckets;
  uint32_t *flags;
  uint32_t *uniq;
  uint32_t *special;
  unsigned long long *n_hits;
  uint32_t bin_bits = kBinBits;  // of the partitioned count's buckets
  uint32_t n_over = 0;           // entries of overflow (0: unchecked)
};

// Top-N selection fused into the LIF kernel (want <= kFuseMaxTopN): every LIF
// block keeps its own top `want` rows by (spikes desc, index asc) -- a superset
// of its share of the global top rows -- and one small kernel after it selects,
// sorts and post-processes the global rows.
constexpr uint32_t kFuseMaxTopN = 64;
constexpr uint32_t kFuseMaxBlocks = 1024;
struct TopFuse {
  uint32_t want;      // 0: not fused
  uint64_t *bcand;    // [blocks * want] keys (spikes << 24 | 0xFFFFFF - index)
  uint32_t *bcnt;     // [blocks]
  TopState *st;
  TopCand *cand;      // final rows, sorted
  uint64_t *top_cur;  // currents of the final rows
  PostArgs post;
  // the pool-sliced finish (nk_slice_export): the final step also writes this
  // slice's all-gather segment (k_slice_seg's layout; neurons [seg_lo, ...),
  // new spikes and largest count from seg_stats); a deferred selection exports
  // no rows, only the refine flag
  uint64_t *seg = nullptr;
  uint64_t seg_lo = 0;
  const uint64_t *seg_stats = nullptr;
};
constexpr uint64_t kSegRefine = 1ull << 56;  // slice segment header: this slice needs the exact refine

constexpr int kZeroMax = 8;
struct ZeroList {  // (filled with fill[b] bytes: 0, or 0xFF for the uniques set's kEmpty)
  void *ptr[kZeroMax];
  uint64_t bytes[kZeroMax];
  uint8_t fill[kZeroMax];
  int n;
};

struct ResultHdr {  // header of the packed finalize results (one D2H copy)
  TopState st;
  uint64_t stats[2];
  uint64_t mask;
  uint32_t flags[4];
};

// input description shared by the k-mer kernels
struct KmerInput {
  const uint8_t *bases;
  const uint64_t *offsets;
  uint64_t n_recs;
  uint64_t n_bases;
  const uint32_t *tile_rec;  // first record of each launched tile (index: tile - tile_base)
  uint64_t n_tiles;          // tiles launched
  // chunked input (streaming ingest): the launch covers tiles tile_base ..
  // tile_base + n_tiles - 1 and counts only windows starting in [pos_lo, pos_hi)
  uint64_t tile_base = 0;
  uint64_t pos_lo = 0;
  uint64_t pos_hi = ~0ull;
};

// The LIF from the reset state fused into a write-through K1b (its outcome is
// a function of each neuron's count): the u8 spike mirror, the spike
// histogram (bin 0 not counted) and the totals, as k_lif_apply writes them
struct K1bLif {
  uint8_t *sc8 = nullptr;  // non-null: on
  const LifEntry *tbl = nullptr;
  int tbl_n = 0;
  LifParams lp{};
  uint32_t *hist = nullptr;             // [kHistCopies][kHistBins]
  unsigned long long *stats = nullptr;  // [0] total spikes [1] max spikes
};

struct PartArgs {
  uint32_t n_buckets;
  uint64_t cap;                   // records per bucket region
  uint16_t *off;                  // [bucket][cap] bin offset within the bucket
  uint16_t *pos;                  // [bucket][cap] k-mer position within its tile
  unsigned long long *fill;       // [bucket] records (low 40 bits) | segments << 40
  uint2 *desc;                    // [bucket][max_segs] {tile, first record}
  uint64_t max_segs;
  uint32_t *overflow;             // [bucket] region overflowed (records counted directly)
  unsigned long long *currents;   // overflow target
  uint32_t bin_bits = kBinBits;   // bucket = neuron >> bin_bits (13..15 on the partitioned path)
  // [2] or null: earliest workgroup start and latest workgroup end of the
  // launch (s_memrealtime, 100 MHz), folded with atomicMin / atomicMax by one
  // lane per workgroup: the kernel's duration without an event in the stream
  unsigned long long *span = nullptr;
  // exact table (nk_table.hip): non-null = K1a also writes each record's key
  // ([bucket][cap], beside off; pos is then not written) and appends the keys
  // of records past a full region to spill[*n_spill++] (< spill_cap)
  uint64_t *key = nullptr;
  uint64_t *spill = nullptr;
  unsigned long long *n_spill = nullptr;
  uint64_t spill_cap = 0;
  // K1b write-through (one slice per bucket, one batch): every bin of the
  // bucket is written to out (no zeroed or read-modified currents); the
  // overflow target `currents` is then a separate array kept zero -- a bucket
  // whose region (or, wide, whose coarse bucket's region) overflowed folds
  // its entries in and zeroes them again
  unsigned long long *out = nullptr;
  const uint32_t *over_coarse = nullptr;  // wide: coarse overflow flags
  uint32_t coarse_shift = 0;              // fine bucket -> coarse bucket
  // K1a (Part path, many buckets): 2^sub_shift sub-regions per bucket, one per
  // XCD (tile & 7: workgroup i runs on XCD i mod 8, tools/xccmap.hip), so a
  // bucket's consecutive descriptors are written through one L2.  fill / desc
  // / the region then index the virtual bucket v = b << sub_shift | x, each
  // of `cap` records and `max_segs` descriptors; overflow stays per bucket.
  uint32_t sub_shift = 0;
  K1bLif lif;                             // write-through only
};

// Generic partition (nk_wide.hip): any key mode; narrow (u16 offsets into
// 32768-bin buckets, bin_bits 15) or wide (u32 offsets into <= 256 coarse
// buckets of 2^bin_bits bins, split into fine buckets by k_split).
constexpr int kWideMaxBuckets = 256;
constexpr int kMaxSplitBits = 9;
constexpr int kMaxSplit = 1 << kMaxSplitBits;  // fine buckets per coarse bucket
struct GenPartArgs {
  uint32_t n_buckets;
  int bin_bits;
  uint64_t cap;                   // records per bucket region (multiple of 64)
  void *rec;                      // [bucket][cap] u16 (narrow) or u32 (wide) bin offsets
  unsigned long long *fill;       // [bucket] records reserved
  uint32_t *overflow;             // [bucket] region overflowed (counted directly)
  unsigned long long *currents;   // overflow target
  // kept records (k_part_gen only): per (bucket, segment) {tile, first record},
  // the segment count in fill's bits 40..; the uniques pass finds the tiles
  // that hold a top row's records and rescans only those (k_uniq_tiles)
  uint2 *desc = nullptr;
  uint64_t max_segs = 0;
  // wide + kept, bin_bits <= kLaneTagMaxBits: each record also carries its
  // k_part_gen lane (bits bin_bits .. bin_bits + 8), so the uniques rescan
  // hashes only the lanes that produced a top row's records
  uint32_t lane_tag = 0;
};
constexpr int kLaneTagMaxBits = 22;  // + 9 lane bits < 32: never the pad (all ones)
// K1g<KEYS> (k_part_gen_keys): where each kept record's u64 key goes
struct GenKeyArgs {
  uint64_t *key;                  // [bucket][cap], beside the u16 records
  uint64_t *spill;                // keys of records past a full region
  unsigned long long *n_spill;
  uint64_t spill_cap;
};
constexpr int kLaneWords = 16;       // 512 lanes of a k_part_gen tile, one bit each

// keys handed to the uniques merge: a flat list (world == 0) or the
// fixed-stride segments [n_r, keys...] of an all-gather buffer
struct MergeSrc {
  const uint64_t *keys;
  uint64_t n;          // flat: number of keys
  uint32_t world;      // segments (0: flat)
  uint64_t stride;     // u64 words per segment
  uint64_t cap;        // keys stored per segment
  uint32_t *trunc;     // bit 0: a segment's n_r > cap; bits 1..3: the header flags of any segment
};

struct UniqArgs {
  const TopCand *top;  // top-N rows (sorted)
  uint32_t n_top;
  uint32_t tbl_size;   // LDS probe table size (pow2 >= 2*n_top)
  unsigned long long *set_keys;  // global hash set of k-mer keys
  const uint64_t *set_mask;      // device word: capacity - 1
  uint32_t *uniq;      // per top row: distinct keys
  uint32_t *special;   // per top row: key == ~0 seen
  // multi-GPU export (nk_finalize_export): every key the set takes for the
  // first time is also appended to xdst[1 + w*i] (w u64 words per key, i < xcap
  // kept; *xn counts them all) -- the all-gather segment, without a set scan
  uint64_t *xdst;
  unsigned long long *xn;
  uint64_t xcap;
};

hipError_t launch_tile_rec(const KmerInput &in, uint64_t tile_size, uint32_t *tile_rec,
                           hipStream_t s);
hipError_t launch_count(const KmerInput &in, int k, int canonical, uint64_t pool,
                        uint64_t *currents, hipStream_t s);
hipError_t launch_uniques(const KmerInput &in, int k, int canonical, uint64_t pool,
                          const UniqArgs &u, hipStream_t s);
hipError_t launch_lif_table(LifEntry *tbl, int n, LifParams lp, hipStream_t s);
// diagnostic: SipHash-1-3 + % pool of n_keys register-generated keys
hipError_t launch_diag_hash(uint64_t n_keys, uint64_t pool, uint32_t *out, hipStream_t s,
                            int width = 64);
uint64_t diag_hash_out_words(uint64_t n_keys);
// partials/slices: when slices > 0, currents[i] += sum of the K1b partials
// first (the fused K1c of a single-device process call) and is written back.
// fresh: v/r/sc are taken as 0 (lazy reset) and every neuron is written.
// derive (with fresh): v / r / spike counts are not written (the derived
// state, SpikeSrc); launch_lif_derive materialises them from the counts.
// sc8 (non-fused top-N only): min(spikes, 255) of every neuron, the compact
// copy the top-N passes read (the global histogram's bin 0 is not counted).
hipError_t launch_lif_apply(uint64_t *currents, const uint32_t *partials, uint32_t slices,
                            int cur_zero, const uint32_t *over, int over_bits,
                            int fresh, int derive, float *v, uint32_t *r, uint64_t *sc, uint64_t pool,
                            LifParams lp, const LifEntry *tbl, int tbl_n, uint32_t *hist,
                            uint64_t *stats, const TopFuse &tf, hipStream_t s,
                            uint8_t *sc8 = nullptr);
hipError_t launch_lif_derive(const uint64_t *currents, float *v, uint32_t *r, uint64_t *sc,
                             uint64_t pool, LifParams lp, const LifEntry *tbl, int tbl_n,
                             hipStream_t s);
uint32_t lif_blocks(uint64_t pool);  // grid size of the LIF kernel
hipError_t launch_topn_threshold(const uint32_t *hist, uint64_t n, uint64_t pool, TopState *st,
                                 hipStream_t s);
hipError_t launch_radix_hist(const SpikeSrc &sc, uint64_t pool, int shift, uint64_t prefix,
                             uint32_t *hist256, hipStream_t s);
hipError_t launch_topn_count(const SpikeSrc &sc, uint64_t pool, TopState *st,
                             uint32_t *tie_cnt, TopCand *cand, hipStream_t s);
hipError_t launch_topn_emit(const SpikeSrc &sc, uint64_t pool, TopState *st,
                            const uint32_t *tie_cnt, TopCand *cand, hipStream_t s);
hipError_t launch_topn_sort(TopCand *cand, uint32_t m, uint64_t n, const uint64_t *currents,
                            uint64_t *top_cur, hipStream_t s);
hipError_t launch_set_fill(unsigned long long *keys, const uint64_t *mask, uint64_t max_cap,
                           hipStream_t s);
hipError_t launch_top_post(const TopCand *top, const uint64_t *top_cur, uint32_t m,
                           uint64_t set_alloc, const uint32_t *overflow, int part,
                           uint64_t *set_mask, uint32_t *tbuckets, uint32_t *flags,
                           uint32_t *uniq, uint32_t *special, unsigned long long *n_hits,
                           uint32_t bin_bits, hipStream_t s, uint32_t n_over = 0);
// --kmer-width=128 (k <= 64): the count, the top rows' uniques (set of 3
// words per slot, u.set_keys), and the set helpers; keys outside the set are
// (lo, hi) pairs of u64.
hipError_t launch_count128(const KmerInput &in, int k, int canonical, uint64_t pool,
                           uint64_t *currents, hipStream_t s);
hipError_t launch_uniques128(const KmerInput &in, int k, int canonical, uint64_t pool,
                             const UniqArgs &u, hipStream_t s);
hipError_t launch_set_fill128(unsigned long long *set3, const uint64_t *mask, uint64_t max_cap,
                              hipStream_t s);
hipError_t launch_set_compact128(const unsigned long long *set3, uint64_t cap, uint64_t *out,
                                 unsigned long long *count, hipStream_t s);
hipError_t launch_set_merge128(const MergeSrc &m, uint64_t pool, const UniqArgs &u, hipStream_t s);
hipError_t launch_set_word(uint64_t *w, uint64_t v, hipStream_t s);
// tile -> first record index for the count kernels, fused with a zero list
// span (optional): the count kernel's [start, end] words, set to [~0, 0]
hipError_t launch_prep(const KmerInput &in, uint64_t tile_size, uint32_t *tile_rec,
                       const ZeroList &z, hipStream_t s, unsigned long long *span = nullptr);
hipError_t launch_zero(const ZeroList &z, hipStream_t s);
hipError_t launch_merge_prep(unsigned long long *set_keys, uint64_t *mask, uint64_t cap, int w128,
                             uint32_t *uniq, uint32_t *special, uint32_t m, uint32_t *trunc,
                             hipStream_t s);
hipError_t launch_wire32(const uint64_t *cur, const uint32_t *partials, uint32_t slices,
                         const uint32_t *over, int over_bits, uint64_t pool, uint32_t *wire,
                         hipStream_t s);
// the merge that follows an export, prepared by the export's header kernel
// (k_merge_prep's work: the merge set emptied at capacity cap, its mask, the
// merge's uniques column and kEmpty flags, the truncation word): S == null: none
struct MergePrep {
  unsigned long long *S = nullptr;
  uint64_t *mask = nullptr;
  uint64_t cap = 0;
  uint32_t *uniq = nullptr;
  uint32_t *special = nullptr;
  uint32_t m = 0;
  uint32_t *trunc = nullptr;
};
// the device-side sliced finish (nk_slice.hip): a slice's top rows into its
// all-gather segment, and the global rows picked from the gathered segments
// (world * want <= kAdoptMax)
constexpr int kAdoptMax = 2048;
// (n: the slice's neurons; a refine or a row >= n exports no rows, the refine flag)
hipError_t launch_slice_seg(const TopCand *cand, const uint64_t *top_cur, const TopState *st,
                            const uint64_t *stats, uint32_t m, uint64_t lo, uint64_t n, uint64_t *seg,
                            hipStream_t s);
// (a flagged segment or a row >= pool: want sentinel rows {~0, 0} and st->refine)
// post (non-null): the top-N post step (k_top_post) for the adopted rows too
hipError_t launch_slice_adopt(const uint64_t *all, uint32_t world, uint64_t stride, uint32_t want,
                              uint64_t pool, TopCand *cand, uint64_t *top_cur, TopState *st,
                              uint64_t *stats, hipStream_t s, const PostArgs *post = nullptr);
hipError_t launch_export(const unsigned long long *set_keys, const uint64_t *set_mask,
                         uint64_t set_alloc, int w128, bool uniq, bool appended,
                         const uint32_t *special, uint32_t n_top, const TopState *st,
                         const uint32_t *post_flags, uint64_t cap_out, uint64_t *dst,
                         unsigned long long *count, hipStream_t s, const MergePrep &mp = MergePrep{});
hipError_t launch_gather(const TopState *st, const uint64_t *stats, const uint64_t *mask,
                         const uint32_t *flags, const uint32_t *flag3, const TopCand *cand,
                         const uint32_t *uniq, uint32_t m, uint8_t *out, uint64_t *done,
                         uint64_t seq, hipStream_t s);
hipError_t launch_set_compact(const unsigned long long *keys, uint64_t cap, const uint32_t *special,
                              uint32_t n_top, const TopCand *top, uint64_t pool,
                              uint64_t *out, unsigned long long *count, hipStream_t s);
hipError_t launch_set_merge(const MergeSrc &m, uint64_t pool, const UniqArgs &u, hipStream_t s);
// [n, min(n, cap) keys of wpk u64 words] from a compacted key list (n on the device)
hipError_t launch_pad_keys(const uint64_t *src, const unsigned long long *n_src, uint64_t cap,
                           int wpk, uint64_t *dst, hipStream_t s);

hipError_t launch_part(const KmerInput &in, int k, int canonical, uint64_t pool,
                       const PartArgs &pa, hipStream_t s);
// key mode km: 0 k <= 32 u64, 1 k > 32 compat, 2 --kmer-width=128
hipError_t launch_part_gen(const KmerInput &in, int k, int canonical, int km, uint64_t pool,
                           const GenPartArgs &ga, int wide, hipStream_t s);
// the same narrow partition (km 0/1, buckets of 2^12..2^15 neurons) also
// writing each kept record's key (the grouped exact table for k > 32)
hipError_t launch_part_gen_keys(const KmerInput &in, int k, int canonical, int km, uint64_t pool,
                                const GenPartArgs &ga, const GenKeyArgs &ka, hipStream_t s);
// uniques rescan over kPartTile tiles for the Gen/Wide count paths; with a
// tile list (tiles, *n_list <= max_list) only those tiles
// the windows of the listed (tile << 9 | lane) entries of lane-tagged records
hipError_t launch_uniq_lanes(const KmerInput &in, int k, int canonical, int km, uint64_t pool,
                             const UniqArgs &u, const uint32_t *list, const uint32_t *n_list,
                             uint32_t max_list, hipStream_t s);
hipError_t launch_uniq_gen(const KmerInput &in, int k, int canonical, int km, uint64_t pool,
                           const UniqArgs &u, hipStream_t s, const uint32_t *tiles = nullptr,
                           const uint32_t *n_list = nullptr, uint32_t max_list = 0);
// the tiles holding the records of the top rows' neurons in the kept Gen/Wide
// records (ga.desc): the top buckets (tbuckets, *n_tb), `slices` workgroups per
// bucket -> tiles[*n_list++] (deduplicated per workgroup); past max_list the
// list is incomplete and flag[0] is set (the caller rescans the input)
hipError_t launch_uniq_tiles(const GenPartArgs &ga, int wide, const UniqArgs &u,
                             const uint32_t *tbuckets, const uint32_t *n_tb, uint32_t max_tb,
                             uint32_t slices, uint32_t *tiles, uint32_t *n_list, uint32_t max_list,
                             uint32_t *flag, uint32_t *mark, uint32_t epoch, uint32_t *lanes,
                             uint32_t hit_queue, hipStream_t s);
// snap_lo / snap_hi (optional): split only the records [snap_lo[b], snap_hi[b])
// of each coarse bucket (one k_part_gen launch's, est_records of them about)
hipError_t launch_split(const GenPartArgs &ga, const PartArgs &fine, hipStream_t s,
                        const unsigned long long *snap_lo = nullptr,
                        const unsigned long long *snap_hi = nullptr, uint64_t est_records = 0);
// the wide count's hash of in's tiles fused with the split of the previous
// launch's records [snap_lo[b], snap_hi[b]) (about split_records of them;
// snap_hi null: no split)
hipError_t launch_gen_split(const KmerInput &in, int k, int canonical, int km, uint64_t pool,
                            const GenPartArgs &ga, const PartArgs &fine,
                            const unsigned long long *snap_lo, const unsigned long long *snap_hi,
                            uint64_t split_records, hipStream_t s);
// snap[b] = min(records reserved in coarse bucket b, cap)
hipError_t launch_fill_snap(const GenPartArgs &ga, unsigned long long *snap, hipStream_t s);
// the exact table's kmer_per_neuron: a key array (wpk u64 words per key, *n_keys
// of them on the device, at most max_n) hashed and partitioned like the count
hipError_t launch_part_keys(const uint64_t *keys, const unsigned long long *n_keys, uint64_t max_n,
                            int wpk, uint64_t pool, const GenPartArgs &ga, int wide, hipStream_t s);
// kpn[i] = cur[i] + sum of `slices` partials (0: none); cur[i] = 0 after
hipError_t launch_kpn_fold(const uint32_t *partials, uint32_t slices, uint64_t pool,
                           unsigned long long *cur, uint32_t *kpn, hipStream_t s);
// K1b of a previous Part count done inside the next count's K1a (k_part_fused):
// its records (off / fill / cap / sub_shift of that count's PartArgs) into
// `slices` partials per bucket, as launch_bucket_hist writes them
constexpr uint32_t kFusePasses = 3;  // a bucket's 32768 bins in thirds (K1a's LDS holds 10923)
struct HistJob {
  const uint16_t *off = nullptr;
  const unsigned long long *fill = nullptr;
  uint64_t cap = 0;
  uint32_t n_buckets = 0, sub_shift = 0, slices = 0;
  uint32_t *partials = nullptr;
  uint64_t pool = 0;
  uint32_t n_items = 0;  // n_buckets * slices * kFusePasses (0: no job)
  uint32_t n_host = 0;   // workgroups [0, n_host) take the items, spread evenly
};
bool part_fused_ok(const PartArgs &pa);  // a count whose K1a has the fused form (and whose K1b it can take)
hipError_t launch_part_fused(const KmerInput &in, int k, int canonical, uint64_t pool,
                             const PartArgs &pa, const HistJob &hj, hipStream_t s);
hipError_t launch_bucket_hist(const PartArgs &pa, uint64_t pool, uint32_t slices,
                              uint32_t *partials, hipStream_t s);
hipError_t launch_partials_add(const uint32_t *partials, uint32_t slices, uint64_t pool,
                               uint64_t *currents, hipStream_t s);
// diagnostic: every kept Part record's key recomputed from its position,
// XOR-folded into *sink (nk_diag_key_gather_ms)
hipError_t launch_diag_key_gather(const KmerInput &in, int k, int canonical, const PartArgs &pa,
                                  unsigned long long *sink, hipStream_t s);
// (also empties the uniques hash set u.set_keys[0 .. *u.set_mask])
hipError_t launch_part_uniques(const KmerInput &in, int k, int canonical, const PartArgs &pa,
                               const UniqArgs &u, const uint32_t *tbuckets, const uint32_t *n_tb,
                               uint32_t max_tb, uint32_t slices, hipStream_t s);

uint64_t top_tbl_size(uint32_t n_top);
uint64_t n_tiles_for(uint64_t n_bases, uint64_t tile);

}  // namespace nk
