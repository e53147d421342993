// nk_table_host.cpp — the exact k-mer table (the reference's `counts` map and
// kmer_per_neuron, src/spiking_hash.rs:26-27,157-172,675-682), process_sequence
// (:203-273) and top_abundant_neurons past the rows a call selected (:661-673).
#include "nk_handle.h"

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
int table_kpn(nk_counter *c, const uint64_t *uniq, const unsigned long long *n_uniq,
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
TableView table_view(const nk_counter *c) {
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
int build_sorted(nk_counter *c, const KmerInput &in0, hipStream_t s) {
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

// neurons per K1a<KEYS> bucket (log2): kXMinBinBits; NK_XBIN_BITS (A/B,
// 13..15) trades K1a's bucket count against passes per group in k_xgroup
uint32_t xbin_bits() {
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
bool grouped_ok(const nk_counter *c, uint64_t n_bases) {
  // (k > 32: NK_KMER_COMPAT u64 keys, the table's own K1g<KEYS> pass)
  if (c->w128 || c->k > 64 || !c->pool || !n_bases) return false;
  const char *e = getenv("NK_EXACT_SORT");
  if (e && atoi(e)) return false;
  if (((c->pool + kBinsPerBucket - 1) >> kBinBits) > (uint64_t)kMaxBuckets) return false;
  if (n_bases > count_chunk()) return false;
  return xgroup_fits(n_bases, c->pool, xgroup_bits(n_bases, c->pool));
}

// side list capacity: records that leave the grouped path (overflowed K1a
// regions, groups with too many distinct keys); past it the sorted build runs
uint64_t side_cap_for(uint64_t n_bases) {
  const uint64_t e = env_u32("NK_XSIDE_CAP", 0);
  return e ? e : std::max<uint64_t>(n_bases / 8, 1ull << 20);
}

// the K1a<KEYS> arguments whose records feed the grouped table: the key
// array (the count's p_key, or the table's own) and the side list
int keyed_args(nk_counter *c, uint64_t n_bases, PartArgs &pa, bool own, hipStream_t s) {
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
int build_grouped(nk_counter *c, const KmerInput &in0, const PartArgs *keyed, hipStream_t s) {
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
    if (c->k > 32) {  // NK_KMER_COMPAT u64 keys: K1g<KEYS> (k_part counts k <= 32 only)
      GenPartArgs ga{};
      ga.n_buckets = pa.n_buckets;
      ga.bin_bits = (int)pa.bin_bits;
      ga.cap = pa.cap;
      ga.rec = pa.off;
      ga.fill = pa.fill;
      ga.overflow = pa.overflow;
      ga.currents = nullptr;
      const GenKeyArgs ka{pa.key, pa.spill, pa.n_spill, pa.spill_cap};
      HIPCHK(launch_part_gen_keys(in, (int)c->k, c->canonical, 1, P, ga, ka, s));
    } else {
      HIPCHK(launch_part(in, (int)c->k, c->canonical, P, pa, s));
    }
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
    const int end_bit = (int)std::min<uint64_t>(64, 2 * c->k);  // (k > 32: u64 compat keys)
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
int build_exact(nk_counter *c, const KmerInput &in, hipStream_t s,
                       const PartArgs *keyed) {
  if (keyed || grouped_ok(c, in.n_bases)) return build_grouped(c, in, keyed, s);
  return build_sorted(c, in, s);
}

// A process/accumulate call replaces `counts` and `kmer_per_neuron` with its
// input's (src/spiking_hash.rs:157-172,426-427,467-473): built now with
// opts.exact_counts, else marked to be built from that input on demand.
int table_for_input(nk_counter *c, const KmerInput &in, hipStream_t s,
                           const PartArgs *keyed) {
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
int ensure_table(nk_counter *c, hipStream_t s) {
  if (!c->x_lazy) return NK_OK;
  if (!c->input_owned)
    return fail(NK_E_UNSUPPORTED,
                "the last input was device memory of the caller (not kept by the handle): "
                "set nk_opts.exact_counts = 1 for counts / kmer_per_neuron / rows past top_n");
  return build_exact(c, c->last_in, s);
}

// Rows past the ones the last call selected (src/spiking_hash.rs:661-673: the
// stable sort, ties by index), the uniques column from kmer_per_neuron (built
// on demand from the last input without opts.exact_counts).
//   m <= kMaxTopN: the exact threshold by radix passes over the spike counts
//     (as many 8-bit digits as the known largest count has) and the select
//     kernels of the top-N path: O(P / 2048) scratch, no pool-sized sort.
//   more rows: the whole pool ranked by a stable radix sort over the bits of
//     the largest count (24 B of scratch per neuron).
long extended_top(nk_counter *c, size_t m, nk_top_row *out) {
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
extern "C" {

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
}  // extern "C"

DeltaArgs delta_args(nk_counter *c) {
  DeltaArgs d{};
  if (c->d_dirty || !c->d_cap) return d;  // keys == null: no delta
  d.keys = c->d_keys.p;
  d.vals = c->d_vals.p;
  d.mask = c->d_cap - 1;
  d.meta = c->d_meta.p;
  return d;
}

// room in the delta for `add` more distinct keys (load <= 1/2)
int delta_reserve(nk_counter *c, uint64_t add, hipStream_t s) {
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

int need_exact(nk_counter *c) {
  if (!c) return fail(NK_E_INVALID, "null counter");
  if (!c->opts.exact_counts)
    return fail(NK_E_UNSUPPORTED, "the exact k-mer table needs nk_opts.exact_counts = 1");
  return NK_OK;
}
extern "C" {

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
}  // extern "C"

// the table for a query: built now from the last input when it is lazy
int table_ready(nk_counter *c, hipStream_t *s) {
  if (!c) return fail(NK_E_INVALID, "null counter");
  (void)hipSetDevice(c->device);
  *s = pick_stream(c, nullptr);
  return ensure_table(c, *s);
}
extern "C" {

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
    // (on the handle's stream, waited for: the caller may use the pointer on any stream)
    if (c->kpn.ensure(c->pool) || hipMemsetAsync(c->kpn.p, 0, c->pool * 4, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
      return nullptr;
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
}  // extern "C"
