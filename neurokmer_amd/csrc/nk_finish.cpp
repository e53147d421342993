// nk_finish.cpp — after a count: the LIF (src/models.rs:34-51,
// src/spiking_hash.rs:186-200), the top-N selection (:661-673), the top rows'
// uniques (:157-172), the readback, and the process_* entry points.
#include "nk_handle.h"

// ---------------------------------------------------------------------------
// exact radix refine of the top-N threshold (spike counts >= 4095; rare)
// ---------------------------------------------------------------------------
// (sc, n): the spike counts ranked — the whole pool, or a rank's slice of it
// (nk_finalize_slice); sc == nullptr means the handle's own pool
int refine_threshold(nk_counter *c, uint64_t want, uint64_t max_sc, TopState &st,
                            hipStream_t s, uint64_t lo, uint64_t n) {
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
LifParams lif_params(const nk_counter *c, int streaming) {
  LifParams lp{};
  lp.steps = c->steps;
  lp.thr = c->thr;
  lp.leak = c->leak;
  lp.refr = c->refr;
  lp.skip_zero = streaming ? 0 : 1;  // process_parallel skips zero currents (:189-191)
  return lp;
}

// closed-form results for fresh neurons with count < 65536, cached per params
int lif_table(nk_counter *c, const LifParams &lp, hipStream_t s) {
  if (!c->lif_valid || c->lif_key.steps != lp.steps || c->lif_key.refr != lp.refr ||
      memcmp(&c->lif_key.thr, &lp.thr, 4) || memcmp(&c->lif_key.leak, &lp.leak, 4)) {
    if (int rc = c->lif_tbl.ensure(kLifTable)) return rc;
    HIPCHK(launch_lif_table(c->lif_tbl.p, kLifTable, lp, s));
    c->lif_key = lp;
    c->lif_valid = true;
  }
  return NK_OK;
}

int lif_prepare(nk_counter *c, int streaming, LifParams &lp, hipStream_t s) {
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
bool k1b_lif_holds(const nk_counter *c, const LifParams &lp, uint32_t fuse_want,
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

int enqueue_lif(nk_counter *c, int streaming, uint32_t fuse_want, bool part,
                       hipStream_t s, const uint32_t *wire) {
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
  if (!wire && c->pend_slices && (rc = hist_ready(c, s))) return rc;
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
int enqueue_select(nk_counter *c, uint64_t want, hipStream_t s, uint64_t lo,
                          uint64_t n) {
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
// the top-N post step's arguments for the uniques pass that follows (the count
// path's buckets: Part, or kept Gen/Wide records; none for a rescan).  The
// caller has sized c->tbuckets for the rows.
PostArgs post_args(nk_counter *c, bool rescan) {
  const bool part = c->part_used && !rescan;
  const bool genk = c->gen_keep && !rescan;
  PostArgs pa{};
  pa.set_alloc = c->set_alloc;
  pa.overflow = part ? c->p_over.p : genk ? c->last_ga.overflow : nullptr;
  pa.part = (part || genk) ? 1 : 0;
  pa.set_mask = c->set_mask_d.p;
  pa.tbuckets = c->tbuckets.p;
  pa.flags = c->post_flags.p;
  pa.uniq = c->uniq.p;
  pa.special = c->special.p;
  pa.n_hits = c->n_hits.p;
  pa.bin_bits = genk ? (uint32_t)c->last_ga.bin_bits : c->last_pa.bin_bits;
  pa.n_over = part ? c->last_pa.n_buckets : genk ? c->last_ga.n_buckets : 0u;
  return pa;
}

int enqueue_uniques(nk_counter *c, uint32_t m, bool rescan, bool post_done,
                           hipStream_t s) {
  const bool part = c->part_used && !rescan;
  const bool genk = c->gen_keep && !rescan;  // kept Gen/Wide records: rescan the hit tiles only
  int rc;
  if ((rc = c->tbuckets.ensure(m))) return rc;
  if (!post_done) {
    const PostArgs pa = post_args(c, rescan);
    HIPCHK(launch_top_post(c->cand.p, c->top_cur.p, m, pa.set_alloc, pa.overflow, pa.part, pa.set_mask,
                           pa.tbuckets, pa.flags, pa.uniq, pa.special, pa.n_hits, pa.bin_bits, s,
                           pa.n_over));
  }
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
    // (whole rounds of the bucket's sub-regions: k_uniq_scan)
    const uint32_t sh = c->last_pa.sub_shift;
    const uint32_t slices = ((std::max<uint32_t>(1, NK_U1_SLICE_BUDGET / m) + (1u << sh) - 1) >> sh) << sh;
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
int enqueue_readback(nk_counter *c, uint32_t m, bool uniq, hipStream_t s,
                            const uint32_t *flag3, const uint32_t *uniq_src) {
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
int wait_readback(nk_counter *c, hipStream_t s) {
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

bool top_fused(const nk_counter *c, uint64_t want) {
  return want && want <= kFuseMaxTopN && lif_blocks(c->pool) <= kFuseMaxBlocks &&
         c->pool <= (1ull << 24);
}

int lif_top_uniques(nk_counter *c, int streaming, bool use_kpn, hipStream_t s,
                           const uint32_t *wire) {
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
int finish_top(nk_counter *c, uint64_t want, bool fused, bool uniq, bool use_kpn,
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
int settle_top(nk_counter *c, uint64_t want, bool uniq, bool use_kpn, bool account,
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
extern "C" {

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
  // the readback was seen and every correction synchronised: nothing of this
  // handle is pending (a stage marker after k_gather touches no buffer), so
  // the next call on another stream starts without a cross-stream wait
  c->quiescent = true;
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
}  // extern "C"

int process_device(nk_counter *c, const uint8_t *d_bases, const uint64_t *d_offs,
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
extern "C" {

int nk_process_parallel_device(nk_counter *c, const uint8_t *d_bases, const uint64_t *d_offs,
                               size_t n_recs, size_t n_bases, void *stream) {
  return process_device(c, d_bases, d_offs, n_recs, n_bases, stream, 0);
}
}  // extern "C"

int check_offsets(const uint64_t *offs, size_t n_recs) {
  if (!offs) return fail(NK_E_INVALID, "null offsets");
  if (offs[0] != 0) return fail(NK_E_INVALID, "rec_offsets[0] must be 0");
  for (size_t i = 0; i < n_recs; ++i)
    if (offs[i + 1] < offs[i]) return fail(NK_E_INVALID, "rec_offsets not monotone at %zu", i);
  return NK_OK;
}

bool any_kmer(const uint64_t *offs, size_t n_recs, size_t k) {
  for (size_t i = 0; i < n_recs; ++i)
    if (offs[i + 1] - offs[i] >= k) return true;
  return false;
}

int process_host(nk_counter *c, const uint8_t *bases, const uint64_t *offs, size_t n_recs,
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
extern "C" {

int nk_process_parallel(nk_counter *c, const uint8_t *bases, const uint64_t *offs, size_t n_recs) {
  return process_host(c, bases, offs, n_recs, 0);
}
}  // extern "C"

// A FASTA/FASTQ file through the GPU ingest (nk_ingest.h), then the LIF rule of
// process_file_streaming (streaming = 1, src/spiking_hash.rs:277-486) or of
// process_parallel over the file's records (streaming = 0, src/main.rs:45-46).
int process_file(nk_counter *c, const char *path, int streaming) {
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
extern "C" {

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
}  // extern "C"
