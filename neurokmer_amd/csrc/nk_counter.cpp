// nk_counter.cpp — the counter handle behind the C ABI (include/neurokmer.h):
// lifecycle, lazy neuron state, accessors, stage timings.  The other paths
// are in the files nk_handle.h lists.
#include "nk_handle.h"

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

const char *kStageNames[kStages] = {"index", "count", "hist", "lif", "topn", "uniques", "total"};
// default (opts.stage_timing == 0): events only around the count kernel and at
// both ends; an event between two kernels idles the GPU for ~6 us on MI355X
const char *kStageNamesLight[kStagesLight] = {"index", "count", "post", "total"};

std::atomic<uint64_t> g_next_uid{1};

// ev[i] for the stage timings; the inner stage boundaries only in full mode
// (stage_timing 0: also around the count kernel; 1: every stage; 2: the ends
// of a call only, so no event sits between two kernels)
bool full_timing(const nk_counter *c) { return c->opts.stage_timing == 1; }

bool count_timing(const nk_counter *c) { return c->opts.stage_timing < 2; }

hipError_t mark(nk_counter *c, int i, hipStream_t s) {
  if (c->opts.stage_timing == 3) return hipSuccess;  // no events at all
  if (full_timing(c) || i == 0 || i == 6 || i == 7 || (count_timing(c) && (i == 1 || i == 2)))
    return hipEventRecord(c->ev[i], s);
  return hipSuccess;
}

uint64_t cost_fixed(double cost) {  // Rust `(cost * 1000.0) as u64`
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
hipStream_t pick_stream(nk_counter *c, void *s) {
  hipStream_t t = s ? (hipStream_t)s : c->own_stream;
  if (c->last_s && c->last_s != t && !c->quiescent && c->order_ev &&
      (c->order_eager || hipEventRecord(c->order_ev, c->last_s) == hipSuccess))
    (void)hipStreamWaitEvent(t, c->order_ev, 0);
  c->quiescent = false;
  c->order_eager = false;
  c->last_s = t;
  return t;
}

// the end of this call's work, for the next call's pick_stream
void record_order(nk_counter *c, hipStream_t s) {
  c->order_eager = c->order_ev && hipEventRecord(c->order_ev, s) == hipSuccess;
}

// Reset is lazy: the neuron state (spikes, v, r) and the currents are only
// marked fresh.  The next LIF takes fresh state as zero without reading it and
// writes every neuron; the next accumulate zeroes the currents in its prep
// kernel; the copy-out / pointer entry points materialise zeros on demand.
int zero_state_on(nk_counter *c, hipStream_t) {
  c->total_spikes = c->total_energy = 0;
  hist_void(c);
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
int settle_state(nk_counter *c, hipStream_t s) {
  if (!c->state_derived) return NK_OK;
  c->state_derived = false;
  HIPCHK(launch_lif_derive(c->cur.p, c->v.p, c->r.p, c->sc.p, c->pool, c->derived_lp, c->lif_tbl.p,
                           kLifTable, s));
  return NK_OK;
}

// spike counts of neurons [lo, ...) as the top-N passes read them
SpikeSrc spike_src(const nk_counter *c, uint64_t lo) {
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
int whole_pool(nk_counter *c) {
  if (c->sliced)
    return fail(NK_E_UNSUPPORTED,
                "the neuron state is sharded across ranks since nk_finalize_slice (this rank "
                "holds its slice only): nk_reset first, or gather the state");
  return NK_OK;
}

// materialise the lazily-zero buffers (what != 0: currents; what == 0: state)
int materialize(nk_counter *c, bool currents, hipStream_t s) {
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
int fold_pending(nk_counter *c, hipStream_t s) {
  if (!c->pend_slices) return NK_OK;
  if (int rc = hist_ready(c, s)) return rc;
  HIPCHK(launch_partials_add(c->partials.p, c->pend_slices, c->pool, c->cur.p, s));
  c->pend_slices = 0;
  return NK_OK;
}

int zero_state(nk_counter *c) {
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
  // (the ordering events keep the system-scope fence: without it the step
  // measured 0.512-0.534 against 0.497-0.508 ms, profiles/r06_ab/order_fence)
  bool ok = hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking) == hipSuccess &&
            hipEventCreateWithFlags(&c->order_ev, hipEventDisableTiming) == hipSuccess &&
            hipEventCreateWithFlags(&c->hist_ev, hipEventDisableTiming) == hipSuccess;
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
  hist_forget(c);
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
  for (PinnedBuf &b : c->ing_he) b.release();
  for (hipEvent_t &e : c->fq_ev)
    if (e) (void)hipEventDestroy(e);
  c->ing_draw.release();
  c->ing_draw2.release(); c->ing_scratch.release(); c->ing_dst.release();
  if (c->ing_cs) (void)hipStreamSynchronize(c->ing_cs);
  for (hipEvent_t &e : c->ing_ev)
    if (e) (void)hipEventDestroy(e);
  if (c->ing_cs) (void)hipStreamDestroy(c->ing_cs);
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
  if (c->hist_ev) (void)hipEventDestroy(c->hist_ev);
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
}  // extern "C"

// The stage markers of the last call may still be pending when it returns
// (the results are awaited on k_gather's completion word, not on the stream):
// the timings are read when asked for.
void collect_timings(nk_counter *c, bool with_count) {
  if (c->opts.stage_timing == 3) {  // nothing was recorded
    c->timing_pending = 0;
    c->n_stage = 0;
    return;
  }
  c->timing_pending = with_count ? 2 : 1;
  c->n_stage = full_timing(c) ? kStages : kStagesLight;
}

void collect_timings_now(nk_counter *c, bool with_count) {
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
extern "C" {

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

int nk_diag_key_gather_ms(nk_counter *c, int reps, float *ms, uint64_t *checksum) {
  if (!c || !ms || reps < 1) return fail(NK_E_INVALID, "nk_diag_key_gather_ms: counter, reps >= 1, ms");
  if (!c->part_used || !c->have_input || !c->last_pa.desc || !c->last_pa.pos || c->last_pa.key ||
      c->k > 32 || c->w128)
    return fail(NK_E_INVALID, "nk_diag_key_gather_ms: the last count kept no Part records (k <= 32, one batch)");
  (void)hipSetDevice(c->device);
  if (hipDeviceSynchronize() != hipSuccess) return fail(NK_E_DEVICE, "device synchronisation failed");
  unsigned long long *sink = nullptr;
  hipStream_t s = nullptr;
  hipEvent_t a = nullptr, b = nullptr;
  int rc = NK_OK;
  float best = 1e30f;
  unsigned long long sum = 0;
  if (hipMalloc(&sink, 8) != hipSuccess) return fail(NK_E_OOM, "hipMalloc");
  if (hipStreamCreate(&s) != hipSuccess || hipEventCreate(&a) != hipSuccess ||
      hipEventCreate(&b) != hipSuccess)
    rc = fail(NK_E_DEVICE, "stream/event creation failed");
  for (int i = 0; rc == NK_OK && i < reps + 1; ++i) {  // + 1 untimed warm-up
    float t = 0.0f;
    if (hipMemsetAsync(sink, 0, 8, s) != hipSuccess || hipEventRecord(a, s) != hipSuccess ||
        launch_diag_key_gather(c->last_in, (int)c->k, c->canonical, c->last_pa, sink, s) != hipSuccess ||
        hipEventRecord(b, s) != hipSuccess || hipEventSynchronize(b) != hipSuccess ||
        hipEventElapsedTime(&t, a, b) != hipSuccess ||
        hipMemcpy(&sum, sink, 8, hipMemcpyDeviceToHost) != hipSuccess)
      rc = fail(NK_E_DEVICE, "diag key gather kernel failed");
    else if (i > 0 && t < best)
      best = t;
  }
  if (a) (void)hipEventDestroy(a);
  if (b) (void)hipEventDestroy(b);
  if (s) (void)hipStreamDestroy(s);
  (void)hipFree(sink);
  if (rc == NK_OK) {
    *ms = best;
    if (checksum) *checksum = sum;
  }
  return rc;
}

int nk_set_stage_timing(nk_counter *c, uint32_t level) {
  if (!c) return fail(NK_E_INVALID, "null counter");
  if (level > 3) return fail(NK_E_INVALID, "stage timing level must be 0, 1, 2 or 3");
  c->opts.stage_timing = level;
  return NK_OK;
}

// The K1a stamp ring to the host (after the handle's stream has drained)
static int read_span_ring(nk_counter *c, std::vector<unsigned long long> &h) {
  h.assign(2 * nk_counter::kCountRing, 0ull);
  if (c->last_s) HIPCHK(hipStreamSynchronize(c->last_s));
  HIPCHK(hipMemcpy(h.data(), c->span.p, h.size() * 8, hipMemcpyDeviceToHost));
  return NK_OK;
}

int nk_count_spans(nk_counter *c, float *ms, int cap) {
  if (!c || (!ms && cap > 0) || cap < 0) return fail(NK_E_INVALID, "null argument");
  (void)hipSetDevice(c->device);
  const uint64_t have = std::min<uint64_t>(c->span_calls, nk_counter::kCountRing);
  const int n = (int)std::min<uint64_t>(have, (uint64_t)cap);
  if (!n) return 0;
  std::vector<unsigned long long> h;
  if (int rc = read_span_ring(c, h)) return rc;
  for (int i = 0; i < n; ++i) {
    const uint64_t call = c->span_calls - (uint64_t)n + (uint64_t)i;
    const unsigned long long *w = &h[2 * (call % nk_counter::kCountRing)];
    ms[i] = w[1] > w[0] ? (float)((double)(w[1] - w[0]) * 1e-5) : -1.0f;  // 10 ns ticks
  }
  return n;
}

int nk_count_stamps(nk_counter *c, unsigned long long *ticks, int cap) {
  if (!c || (!ticks && cap > 0) || cap < 0) return fail(NK_E_INVALID, "null argument");
  (void)hipSetDevice(c->device);
  const int n = (int)std::min<uint64_t>(std::min<uint64_t>(c->span_calls, nk_counter::kCountRing), (uint64_t)cap);
  if (!n) return 0;
  std::vector<unsigned long long> h;
  if (int rc = read_span_ring(c, h)) return rc;
  for (int i = 0; i < n; ++i) {
    const uint64_t call = c->span_calls - (uint64_t)n + (uint64_t)i;
    ticks[2 * i] = h[2 * (call % nk_counter::kCountRing)];
    ticks[2 * i + 1] = h[2 * (call % nk_counter::kCountRing) + 1];
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
