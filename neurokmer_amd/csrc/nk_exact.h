// Exact k-mer count table on the device: the reference's
// `counts: DashMap<u64, AtomicU32>` (src/spiking_hash.rs:27,157-165,441-447),
// `get_count` (:675-682) and the full `kmer_per_neuron` (:167-172,467-473).
//
// Built only when nk_opts.exact_counts is set (the reference always builds it;
// it is off the metric's hot path):
//   1. every k-mer key of the input, compacted (one atomic per workgroup);
//   2. radix sort (rocPRIM) over the key's 2k significant bits;
//   3. run-length encode -> sorted unique keys + u32 counts (a count wraps at
//      2^32 like the reference's AtomicU32 / u32 `+=`);
//   4. kmer_per_neuron[H(key) % P] += 1 per unique key.
// get_count = binary search in the sorted keys (+ the process_sequence delta
// table, nk_counter.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "nk_device.h"
#include "nk_kernels.h"

namespace nk {

// ---- table layouts -----------------------------------------------------------
// sorted:  uniq[0, n) ascending (the global radix sort, or nk_exact_adopt)
// grouped: (nk_table.hip) the entries of neuron i at uniq[start, start + len),
//          ent[i] = start | len << 40, in no key order; neurons whose entries
//          went through the side list (ent[i] == kSideEnt) are in the
//          key-sorted part uniq[n[1], n[0])
constexpr unsigned long long kSideEnt = ~0ull;
struct TableView {
  const uint64_t *uniq;
  const uint32_t *cnt;
  const unsigned long long *n;  // device: [0] distinct keys, [1] first index of the sorted part; null: empty
  const uint64_t *ent;          // grouped layout; null: sorted
  FastMod fm;                   // pool (grouped layout)
};

__device__ __forceinline__ bool table_find(const TableView &t, uint64_t key, uint64_t *at) {
  if (!t.n) return false;
  uint64_t lo = 0, hi = t.n[0];
  if (t.ent) {
    const uint64_t e = t.ent[fastmod(sip13_u64(key), t.fm)];
    if (e != kSideEnt) {
      const uint64_t s0 = e & ((1ull << 40) - 1), s1 = s0 + (e >> 40);
      for (uint64_t i = s0; i < s1; ++i)
        if (t.uniq[i] == key) {
          *at = i;
          return true;
        }
      return false;
    }
    lo = t.n[1];
  }
  while (lo < hi) {  // first index with uniq >= key
    const uint64_t mid = (lo + hi) >> 1;
    if (t.uniq[mid] < key) lo = mid + 1;
    else hi = mid;
  }
  *at = lo;
  return lo < t.n[0] && t.uniq[lo] == key;
}

// The grouped build (nk_table.hip) over the bucket regions of a K1a<KEYS>
// partition (one batch, records of 2^bin_bits-neuron buckets with their keys):
// regrouped into groups of 2^ggbits neurons (at most 256 groups per bucket),
// aggregated 2^gbits neurons per LDS pass (one pass when gbits == ggbits).
constexpr int kXGroupBits = 7;     // largest group: 128 neurons (bin2 < 128)
constexpr int kXMaxGroups = 256;   // groups per bucket
constexpr int kXSlice = 16384;     // records per slice of a bucket region
constexpr int kXMinBinBits = 13;   // K1a<KEYS> buckets of at least 8192 neurons (<= 256 of them)
struct XGroupArgs {
  // source partition
  uint32_t n_buckets;
  uint64_t cap;                       // records per bucket region (< 2^32)
  uint32_t bin_bits;                  // neurons per bucket = 2^bin_bits (kXGroupBits..15)
  const uint16_t *off;                // [bucket][cap] neuron within the bucket (0xFFFF: pad)
  const uint64_t *key;                // [bucket][cap]
  const unsigned long long *fill;     // [bucket] records (low 40 bits)
  const uint32_t *overflow;           // [bucket] 1: the bucket goes to the side list
  // 2^ggbits neurons per group (<= 128, n_groups = 2^(bin_bits - ggbits) <= 256
  // per bucket), 2^gbits per LDS pass (<= ggbits), n_slices per bucket
  uint32_t ggbits, gbits, n_groups, n_slices;
  uint32_t *xcnt;                     // [bucket][slice][group] counts -> offsets
  uint32_t *gstart;                   // [bucket][n_groups + 1]
  uint64_t *key2;                     // [bucket][cap] records grouped
  uint8_t *bin2;                      // [bucket][cap] neuron within the group
  // side list (also K1a<KEYS>' spill)
  uint64_t *side;
  unsigned long long *n_side;
  uint64_t side_cap;
  // the table: group g of bucket b owns the entries [bbase[b] + gstart[g],
  // bbase[b] + gstart[g + 1]) (its records: bbase = the records of the
  // buckets before); what its distinct keys leave is (0, count 0): outside
  // every neuron's range, skipped by the multi-GPU partition (skip_zero)
  uint64_t pool;
  uint64_t *uniq;
  uint32_t *cnt;
  unsigned long long *bbase, *bdist;  // [bucket]: table base, distinct keys (zeroed by k_xbase)
  unsigned long long *span;           // grouped part's length (holes included)
  uint64_t *ent;                      // [pool]
  uint32_t *kpn;                      // [pool] kmer_per_neuron (side neurons: 0, added later)
  uint32_t hash_max = 0;              // tests: fewer distinct keys per pass (0: the LDS table's)
  uint32_t hash_bits = 12;            // log2 LDS table slots of k_xgroup (xgroup_hash_bits())
};
// 2^gbits neurons per LDS pass for n_records records over `pool` neurons, and
// whether the expected distinct keys of a pass fit the LDS table; the group
// bits for a bucket of 2^bin_bits neurons
uint32_t xgroup_bits(uint64_t n_records, uint64_t pool);
uint32_t xgroup_hash_bits();
inline uint32_t xgroup_group_bits(uint32_t gbits, uint32_t bin_bits) {
  const uint32_t lo = bin_bits > 8 ? bin_bits - 8 : 0;  // <= 256 groups per bucket
  return gbits > lo ? gbits : lo;
}
bool xgroup_fits(uint64_t n_records, uint64_t pool, uint32_t gbits);
hipError_t xgroup_build(const XGroupArgs &t, hipStream_t s);
// after the side part: n[0] = span + *n_side_uniq (null: 0) (entries),
// n[1] = span (first index of the sorted part), n[5] = distinct + side uniq
hipError_t xgroup_finish(const XGroupArgs &t, unsigned long long *n,
                         const unsigned long long *n_side_uniq, hipStream_t s);

// keys of every valid window of `in` (in.tile_rec for kTile tiles), in any
// order; *n_keys (device) must be 0 on entry
hipError_t exact_keys(const KmerInput &in, int k, int canonical, uint64_t *keys,
                      unsigned long long *n_keys, hipStream_t s);
// scratch bytes for exact_sort_rle over n keys
size_t exact_temp_bytes(size_t n, int end_bit);
// sort keys[0..n) (keys is clobbered) and run-length encode into uniq/cnt;
// *n_uniq (device) receives the number of distinct keys
hipError_t exact_sort_rle(uint64_t *keys, uint64_t *keys_sorted, size_t n, int end_bit,
                          uint64_t *uniq, uint32_t *cnt, unsigned long long *n_uniq, void *tmp,
                          size_t tmp_bytes, hipStream_t s);
// kpn[H(key) % pool] += 1 for every distinct key (kpn zeroed by the caller)
hipError_t exact_kpn(const uint64_t *uniq, const unsigned long long *n_uniq, size_t max_n,
                     uint64_t pool, uint32_t *kpn, hipStream_t s);
// out[i] = count of q[i] in the table (present[i] = 0/1)
hipError_t exact_lookup(const TableView &t, const uint64_t *q, size_t nq, uint32_t *out,
                        uint32_t *present, hipStream_t s);
// ---- process_sequence (src/spiking_hash.rs:203-273) ------------------------
// The k-mers a process_sequence call adds to `counts` go to a device hash
// table ("delta") on top of the sorted table of the last process call.
struct DeltaArgs {
  unsigned long long *keys;   // [cap], kEmpty = free
  uint32_t *vals;             // [cap]
  uint64_t mask;              // cap - 1
  unsigned long long *meta;   // [0] count of key ~0, [1] keys new to counts (distinct)
};
hipError_t delta_clear(const DeltaArgs &d, hipStream_t s);
hipError_t delta_rehash(const DeltaArgs &from, const DeltaArgs &to, hipStream_t s);
// one sequence's keys: currents[H(key) % pool] += 1, touched[idx] = 1, counts[key] += 1
hipError_t seq_accumulate(const uint64_t *keys, const unsigned long long *n_keys, size_t max_n,
                          uint64_t pool, unsigned long long *currents, uint8_t *touched,
                          const DeltaArgs &d, const TableView &t, hipStream_t s);
// kmer_per_neuron += touched; one LifNeuron::update(current as f32) for every
// neuron with current > 0; currents = 0; spike-count histogram + stats
hipError_t seq_lif(uint64_t pool, unsigned long long *currents, uint8_t *touched, uint32_t *kpn,
                   float *v, uint32_t *r, uint64_t *sc, float thr, float leak, uint32_t refr,
                   uint32_t *hist, uint64_t *stats, hipStream_t s);
// get_count over the table (may be empty: t.n null) plus the delta
hipError_t exact_lookup2(const TableView &t, const DeltaArgs &d, const uint64_t *q, size_t nq,
                         uint32_t *out, uint32_t *present, hipStream_t s);

// ---- multi-GPU table (hash partition + all-to-all) --------------------------
// Owner rank of a key: every rank computes the same owner without
// communication, so each distinct key ends up in exactly one rank's table and
// the per-rank kmer_per_neuron contributions add up (all-reduce) to the
// global one.
__host__ __device__ inline uint32_t exact_owner(uint64_t key, uint32_t world) {
  uint64_t x = key + 0x9E3779B97F4A7C15ull;  // splitmix64 finaliser
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  x ^= x >> 31;
  return (uint32_t)(((x >> 32) * (uint64_t)world) >> 32);
}
// per-owner key counts of the table (cnt zeroed by the caller, world <= 4096);
// tcnt non-null: entries whose count is 0 are skipped (the grouped layout's holes)
hipError_t exact_owner_hist(const uint64_t *uniq, const unsigned long long *n_uniq, size_t max_n,
                            uint32_t world, unsigned long long *cnt, hipStream_t s,
                            const uint32_t *tcnt = nullptr);
// (key, count) pairs grouped by owner: cursor[r] = the start of owner r's range
// on entry (advanced by the kernel)
hipError_t exact_owner_scatter(const uint64_t *uniq, const uint32_t *cnt,
                               const unsigned long long *n_uniq, size_t max_n, uint32_t world,
                               unsigned long long *cursor, uint64_t *out_keys, uint32_t *out_cnt,
                               hipStream_t s, bool skip_zero = false);
// scratch bytes for exact_merge_pairs over n pairs
size_t exact_merge_temp_bytes(size_t n, int end_bit);
// sort (key, count) pairs and sum the counts of equal keys (u32, wrapping):
// sorted unique keys + counts, *n_uniq (device)
hipError_t exact_merge_pairs(const uint64_t *keys, const uint32_t *cnt, size_t n, int end_bit,
                             uint64_t *keys_sorted, uint32_t *cnt_sorted, uint64_t *uniq,
                             uint32_t *uniq_cnt, unsigned long long *n_uniq, void *tmp,
                             size_t tmp_bytes, hipStream_t s);

// uniques column of the top rows from kmer_per_neuron
hipError_t exact_top_uniques(const TopCand *cand, uint32_t m, const uint32_t *kpn, uint32_t *uniq,
                             hipStream_t s);

// ---- NK_KMER_128 table (k <= 64; no reference counterpart: the build's true
// k <= 64 mode) -------------------------------------------------
// keys are u128 (lo | hi << 64), 16-byte aligned arrays of 2 u64 words each;
// the same steps as above: extraction, rocPRIM radix sort over 2k bits, RLE,
// kpn[SipHash-1-3(16 LE bytes) % P] += 1 per distinct key, binary-search lookup
hipError_t exact_keys128(const KmerInput &in, int k, int canonical, uint64_t *keys2,
                         unsigned long long *n_keys, hipStream_t s);
size_t exact_temp_bytes128(size_t n, int end_bit);
hipError_t exact_sort_rle128(uint64_t *keys2, uint64_t *sorted2, size_t n, int end_bit,
                             uint64_t *uniq2, uint32_t *cnt, unsigned long long *n_uniq, void *tmp,
                             size_t tmp_bytes, hipStream_t s);
hipError_t exact_kpn128(const uint64_t *uniq2, const unsigned long long *n_uniq, size_t max_n,
                        uint64_t pool, uint32_t *kpn, hipStream_t s);
// q2: nq (lo, hi) pairs
hipError_t exact_lookup128(const uint64_t *uniq2, const uint32_t *cnt,
                           const unsigned long long *n_uniq, const uint64_t *q2, size_t nq,
                           uint32_t *out, uint32_t *present, hipStream_t s);

// ---- top_abundant_neurons(n) for any n (src/spiking_hash.rs:661-673) --------
// The reference's stable sort of (idx, spike_count) by spikes descending over
// the whole pool: a stable rocPRIM radix sort of (max_sc - sc[i], i) pairs, i
// ascending on entry, so ties keep index order.  rows_idx/rows_key receive the
// first `m` rows (key = max_sc - spikes).  Returns the scratch size when tmp is
// null (as rocPRIM does).
size_t rank_rows_temp_bytes(size_t pool);
hipError_t rank_rows(const uint64_t *sc, uint64_t pool, uint64_t max_sc, uint64_t *keys,
                     uint64_t *keys_sorted, uint32_t *idx, uint32_t *idx_sorted, void *tmp,
                     size_t tmp_bytes, hipStream_t s);

}  // namespace nk
