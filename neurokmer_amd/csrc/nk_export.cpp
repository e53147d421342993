// nk_export.cpp — the pieces of the multi-GPU finish a rank runs between
// collectives (nk_dist.cpp drives them): the u32 wire, the export of this
// shard's top k-mers, the merge of the gathered segments, the redo, and the
// pool-sliced finish (each rank the LIF and top rows of its slice).
#include "nk_handle.h"

// uniques column of the top rows from a union of key lists (flat or the
// fixed-stride all-gather form); *complete = 0 if a segment was truncated
// (the top rows are then left as they were)

int merge_keys(nk_counter *c, const MergeSrc &src, uint64_t max_keys, int *complete,
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
uint64_t merge_cap(uint64_t max_keys) {
  uint64_t cap = 64;
  while (cap < 2 * max_keys + 2) cap <<= 1;
  return cap;
}

int enqueue_merge(nk_counter *c, const MergeSrc &src, uint64_t max_keys, uint32_t m,
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
extern "C" {

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
  if (c->pend_slices && (rc = hist_ready(c, s))) return rc;
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
}  // extern "C"

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
int finalize_slice_impl(nk_counter *c, int streaming, const void *d_slice, int slice_bits,
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
extern "C" {

int nk_finalize_slice(nk_counter *c, int streaming, const void *d_slice, int slice_bits,
                      size_t lo, size_t hi, uint64_t *d_seg, size_t seg_rows, void *stream) {
  if (!c || !d_seg) return fail(NK_E_INVALID, "null argument");
  (void)hipSetDevice(c->device);
  return finalize_slice_impl(c, streaming, d_slice, slice_bits, lo, hi, d_seg, seg_rows,
                             pick_stream(c, stream), true);
}
}  // extern "C"

extern "C++" namespace nk {
// the blocking selection of this rank's slice after nk_slice_export (its LIF
// done): a redo of the device-side sliced finish (nk_dist.cpp)
int slice_reselect(nk_counter *c, size_t lo, size_t hi, uint64_t *d_seg, size_t seg_rows,
                   hipStream_t s) {
  (void)hipSetDevice(c->device);
  return finalize_slice_impl(c, 0, nullptr, 32, lo, hi, d_seg, seg_rows, pick_stream(c, s), false);
}
}  // namespace nk

extern "C" {

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
    // the final step writes the slice's segment too (no k_slice_seg launch)
    tf.seg = d_seg;
    tf.seg_lo = lo;
    tf.seg_stats = c->stats.p;
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
  if (!fuse)
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
  // every rank's slice yields min(top_n, its size) rows: together >= min(top_n, pool) = want;
  // the adopt kernel also runs the top-N post step of the uniques pass (no k_top_post)
  const bool uniq = want && c->have_input && c->last_in.n_tiles;
  if ((rc = c->tbuckets.ensure(std::max<uint64_t>(want, 1)))) return rc;
  const PostArgs post = post_args(c, false);
  HIPCHK(launch_slice_adopt(d_all, (uint32_t)world, stride, (uint32_t)want, c->pool, c->cand.p,
                            c->top_cur.p, c->topst.p, c->stats.p, s, uniq ? &post : nullptr));
  if ((rc = c->export_n.ensure(1))) return rc;
  if (!c->export_n_zeroed) {
    HIPCHK(hipMemsetAsync(c->export_n.p, 0, 8, s));
    c->export_n_zeroed = true;
  }
  c->xport_dst = d_keyseg;  // the uniques pass appends each new key to the segment
  c->xport_cap = cap;
  rc = uniq ? enqueue_uniques(c, (uint32_t)want, false, /*post_done=*/true, s) : NK_OK;
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
}  // extern "C"
