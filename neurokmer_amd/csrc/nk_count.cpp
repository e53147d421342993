// nk_count.cpp — the count: currents = histogram of H(kmer) % pool over an
// input (src/spiking_hash.rs:94-154): the partition plan, the partitioned
// launches (k_part / k_part_gen [+ k_split] + k_bucket_hist), batches.
#include "nk_handle.h"

#include <mutex>
#include <thread>

// How one count batch runs:
//   Part   k <= 32 keys, pool <= 16.7 M: k_part (rolled keys) + k_bucket_hist;
//          the records are kept for the uniques scan
//   Gen    k > 32 compat / 128-bit keys, pool <= 16.7 M: k_part_gen (narrow)
//          + k_bucket_hist
//   Wide   pool <= 2^31, k <= 64: k_part_gen (coarse) + k_split + k_bucket_hist
//   Atomic the direct-atomic kernels (k > 64 compat keys, pool > 2^31)
// (CountPath, CountPlan: nk_handle.h)

// tests: NK_WIDE_BITS=b forces the wide path with coarse buckets of 2^b bins
int wide_bits_forced() {
  const char *e = getenv("NK_WIDE_BITS");
  return e ? atoi(e) : 0;
}

// tests: NK_FORCE_ATOMIC=1 forces the direct-atomic count kernels (k_kmers,
// k_kmers_compat, k_kmers128), which otherwise run only past the partitions
bool atomic_forced() {
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
uint64_t count_chunk(uint64_t n_bases, uint64_t pool, bool wide, uint64_t held) {
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
uint64_t arena_bytes(const nk_counter *c) {
  return c->p_off.n * 2 + c->p_pos.n * 2 + c->p_desc.n * 8 + c->w_rec.n * 4;
}

// Sizes the buffers for a batch of about est_bases bases (slack: extra
// records per bucket region; max_segs: Part's descriptors per bucket) and
// lists the arrays to zero before the first batch.
// part_bits: the narrowest Part buckets to try (the exact table's K1a<KEYS>
// count takes 4096-neuron buckets, up to 512 of them: nk_table.hip)
int plan_count(nk_counter *c, uint64_t est_bases, uint64_t slack, uint64_t max_segs,
                      CountPlan &cp, ZeroList &z, bool keep_gen, int part_bits) {
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
  // Part past 128 buckets (P > 4.2 M) leaves ~13-record segments per (tile,
  // bucket) at config 3's 16 M: K1a wrote 15.2 B per k-mer for 4 (partial
  // lines of scattered 16-B stores) and reserved 489 times per tile.  A count
  // that keeps its records in one launch takes the wide path there instead:
  // <= 128 coarse buckets (long segments of u32 records, the keys rolled in
  // registers as K1a does: gen_rolled64), then the split into the 32768-neuron
  // buckets.  (NK_PART_BIG=1: the Part path as before, A/B.)  Chunked and
  // streamed counts keep Part (they keep every record for the uniques scan).
  const bool big_wide = cp.km == 0 && keep_gen && !part_bits && B > kSubMinBuckets && wide_ok &&
                        c->canonical && !getenv("NK_PART_BIG");
  if ((forced > 0 || big_wide) && wide_ok) cp.path = CountPath::Wide;
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
    // at most 128 coarse buckets (the kernels take 256): ~64 records per
    // (tile, coarse bucket) segment instead of ~33 -- half the pad records and
    // descriptors, a 64-way split.  Config 5 (P = 256 M): 123 buckets of 2^21
    // bins, the count 77.1 ms against 79.7 with 245 of 2^20 and 79.4 with 62 of
    // 2^22 (the uniques scan of a top bucket grows with it, profiles/r05_i)
    // (the Part pools past 4.2 M, big_wide: at most 64 -- config 3's count
    // 23.7 vs 25.2 ms with 62 coarse buckets of 2^18 against 123 of 2^17,
    // the longer segments and fewer split tiles, profiles/r06_c3)
    const uint64_t kCoarse = big_wide ? 64 : 128;
    int bits = kBinBits;
    while (((P + (1ull << bits) - 1) >> bits) > kCoarse) ++bits;
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
  // Part with many buckets (P > 128 x 32768; not the keyed count, whose
  // records the table reads per bucket): a sub-region per XCD in each bucket
  // region (PartArgs::sub_shift).  At 489 buckets (P = 16 M) a tile writes a
  // descriptor and a ~17-record segment per bucket; the descriptors of one
  // bucket, written from all eight XCDs, cost 155 MB of K1a's 926 MB written,
  // 62 MB with a table per XCD (the step 1.4-3 % faster, profiles/r05_o-q;
  // NK_NO_XCD_REGIONS=1: one region per bucket)
  uint32_t sub_shift = 0;
  if (cp.path == CountPath::Part && !part_bits && B > kSubMinBuckets && !getenv("NK_NO_XCD_REGIONS")) {
    sub_shift = kSubShift;
    // records per sub-region (1/8 of the tiles each), with room for the
    // segments' padding to whole 8-record groups (~3.5 per (tile, bucket))
    cap = ((cap + 4 * n_tiles_for(est, kPartTile)) >> sub_shift) + 64;
    max_segs = (max_segs >> sub_shift) + 64;
  }
  cap = (cap + 63) & ~63ull;
  // one round of 1-per-CU workgroups (128 KiB LDS each) on 256 CUs
  cp.slices = (uint32_t)std::max<uint64_t>(1, NK_K1B_WGS / B);
  const uint64_t V = B << sub_shift;  // (virtual) buckets: fill counters, regions
  if ((rc = c->p_off.ensure(V * cap)) || (rc = c->p_fill.ensure(V)) || (rc = c->p_over.ensure(B)) ||
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
  pa.sub_shift = sub_shift;
  if (cp.path == CountPath::Part) {
    if ((rc = c->p_pos.ensure(V * cap)) || (rc = c->p_desc.ensure(V * max_segs))) return rc;
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
  z.ptr[z.n] = c->p_fill.p; z.bytes[z.n++] = V * 8;
  z.ptr[z.n] = c->p_over.p; z.bytes[z.n++] = B * 4;
  return NK_OK;
}

// K1b of a Gen/Wide batch: partials (several slices per bucket) or straight
// into the currents
hipError_t gen_hist(nk_counter *c, const CountPlan &cp, bool defer_partials, hipStream_t s) {
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
constexpr uint64_t kSplitMinTiles = 8192;  // (115 Mbases, 6 launches: +2 % on the count, r05_g)

uint32_t split_launches(uint64_t n_tiles) {
  const char *e = getenv("NK_SPLIT_LAUNCHES");
  uint64_t g = e ? strtoull(e, nullptr, 10) : std::min<uint64_t>(32, n_tiles / kSplitMinTiles);
  g = std::min<uint64_t>(std::min<uint64_t>(g, nk_counter::kSplitMax), n_tiles);
  return (uint32_t)std::max<uint64_t>(g, 1);
}

// The wide count with its split pipelined: k_part_gen is VALU-bound (SipHash)
// and k_split is bound by its bytes, so the input's tiles go in G launches of
// k_gen_split: launch g hashes its tiles and splits the records launch g - 1
// reserved (each coarse bucket's records between the fill snapshots taken
// after launches g - 2 and g - 1), every workgroup doing one of each; a last
// k_split takes launch G - 1's records.
hipError_t split_pipelined(nk_counter *c, const CountPlan &cp, const KmerInput &in, uint32_t G,
                                  hipStream_t s) {
  hipError_t e;
  const uint64_t nb = cp.ga.n_buckets;
  if (c->w_snap.ensure((uint64_t)G * nb)) return hipErrorOutOfMemory;
  const uint64_t per = (in.n_tiles + G - 1) / G;
  const bool defer = getenv("NK_GS_DEFER") != nullptr;  // A/B: every split after the last launch
  uint32_t g = 0;
  uint64_t prev_tiles = 0;
  for (uint64_t t0 = 0; t0 < in.n_tiles; t0 += per, ++g) {
    KmerInput bi = in;
    bi.tile_base = in.tile_base + t0;
    bi.tile_rec = in.tile_rec + t0;
    bi.n_tiles = std::min<uint64_t>(per, in.n_tiles - t0);
    unsigned long long *snap = c->w_snap.p + (uint64_t)g * nb;  // after this launch
    const unsigned long long *hi = g ? snap - nb : nullptr;      // the previous launch's records
    const unsigned long long *lo = g > 1 ? snap - 2 * nb : nullptr;
    if (defer) lo = hi = nullptr;
    if ((e = launch_gen_split(bi, (int)c->k, c->canonical, cp.km, c->pool, cp.ga, cp.pa, lo, hi,
                              prev_tiles * kPartTile * 9 / 8, s)) ||
        (e = launch_fill_snap(cp.ga, snap, s)))
      return e;
    prev_tiles = bi.n_tiles;
  }
  const unsigned long long *last = c->w_snap.p + (uint64_t)(g - 1) * nb;
  if (defer) return launch_split(cp.ga, cp.pa, s);
  return launch_split(cp.ga, cp.pa, s, g > 1 ? last - nb : nullptr, last, prev_tiles * kPartTile);
}

// Gen/Wide count kernels of one batch (before K1b)
hipError_t gen_count(nk_counter *c, const CountPlan &cp, const KmerInput &in, hipStream_t s,
                            bool pipeline) {
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
hipError_t batch_count(nk_counter *c, const CountPlan &cp, const KmerInput &in, hipStream_t s) {
  hipError_t e = cp.path == CountPath::Part
                     ? launch_part(in, (int)c->k, c->canonical, c->pool, cp.pa, s)
                     : gen_count(c, cp, in, s);
  if (e == hipSuccess) e = gen_hist(c, cp, false, s);
  if (e != hipSuccess) return e;
  ZeroList z{};
  z.ptr[z.n] = cp.pa.fill; z.bytes[z.n++] = ((uint64_t)cp.pa.n_buckets << cp.pa.sub_shift) * 8;
  if (cp.path == CountPath::Wide) {
    z.ptr[z.n] = cp.ga.fill; z.bytes[z.n++] = (uint64_t)cp.ga.n_buckets * 8;
  }
  return launch_zero(z, s);
}

// ---------------------------------------------------------------------------
// K1b deferred across handles (opts.defer_hist).  With batches in flight on
// one count stream, K1b of batch i (HBM- and LDS-bound, ~50 us at config 2)
// runs inside K1a of batch i+1 (VALU-bound, HBM ~80 % idle): k_part_fused.
// One slot per device holds the Part count whose K1b has not run; the next
// fusable count on the same stream, from the same host thread and of another
// handle, takes it (its own K1b then waits in the slot in turn).  The owner's
// readers (hist_ready) wait for the fused kernel's end (hist_ev), or run the
// K1b themselves when nothing took it.  hist_state (under g_hist_mu): 0 none,
// 1 in the slot, 2 enqueued (hist_ev recorded after it), 3 being taken (the
// taking thread is between hist_take and hist_taken: a reader on another
// thread waits for 2).
// ---------------------------------------------------------------------------
namespace {
struct HistSlot {
  nk_counter *owner = nullptr;
  hipStream_t s = nullptr;
  std::thread::id tid;
};
std::mutex g_hist_mu;
constexpr int kHistSlots = 64;
HistSlot g_hist_slot[kHistSlots];
HistSlot &slot_of(int dev) { return g_hist_slot[(unsigned)dev % kHistSlots]; }
constexpr uint64_t kFuseMinTiles = 512;  // a count this small runs its own K1b

// K1b of the Part count c as the standalone kernel
hipError_t hist_run(nk_counter *c, hipStream_t s) {
  return launch_bucket_hist(c->last_pa, c->pool, c->hist_slices, c->partials.p, s);
}

// slices of a deferred K1b (partials the LIF folds; NK_FUSE_SLICES: A/B)
uint32_t fuse_slices(uint32_t dflt) {
  const char *e = getenv("NK_FUSE_SLICES");
  const long v = e ? strtol(e, nullptr, 10) : 0;
  return v > 0 && v <= 64 ? (uint32_t)v : dflt;
}

// the workgroups of the taking count that host the items: the first
// NK_FUSE_HOST_PCT percent of its grid (default 75: no item in the tail)
uint32_t fuse_hosts(uint64_t n_tiles) {
  const char *e = getenv("NK_FUSE_HOST_PCT");
  const long v = e ? strtol(e, nullptr, 10) : 0;
  const uint64_t pct = v > 0 && v <= 100 ? (uint64_t)v : 75;
  return (uint32_t)std::max<uint64_t>(1, n_tiles * pct / 100);
}

// another handle's pending K1b that the count of c on stream s can take
nk_counter *hist_take(nk_counter *c, hipStream_t s, uint64_t n_tiles, HistJob &hj) {
  std::lock_guard<std::mutex> g(g_hist_mu);
  HistSlot &h = slot_of(c->device);
  nk_counter *a = h.owner;
  if (!a || a == c || h.s != s || h.tid != std::this_thread::get_id()) return nullptr;
  h.owner = nullptr;
  const PartArgs &pa = a->last_pa;
  hj.off = pa.off;
  hj.fill = pa.fill;
  hj.cap = pa.cap;
  hj.n_buckets = pa.n_buckets;
  hj.sub_shift = pa.sub_shift;
  hj.slices = a->hist_slices;
  hj.partials = a->partials.p;
  hj.pool = a->pool;
  hj.n_items = pa.n_buckets * a->hist_slices * kFusePasses;
  hj.n_host = fuse_hosts(n_tiles);
  a->hist_state = 3;
  return a;
}

// c's own K1b into the slot (false: the slot holds another thread's count)
bool hist_leave(nk_counter *c, hipStream_t s) {
  std::lock_guard<std::mutex> g(g_hist_mu);
  HistSlot &h = slot_of(c->device);
  if (h.owner && h.owner != c) {
    if (h.tid != std::this_thread::get_id()) return false;
    // an older pending K1b of this thread that no count took (another
    // stream): it runs now, on its own stream; its readers wait for hist_ev
    nk_counter *a = h.owner;
    if (hist_run(a, h.s) != hipSuccess || hipEventRecord(a->hist_ev, h.s) != hipSuccess) return false;
    a->hist_state = 2;
  }
  h.owner = c;
  h.s = s;
  h.tid = std::this_thread::get_id();
  c->hist_state = 1;
  return true;
}

// the taking count's fused kernel and hist_ev are enqueued
void hist_taken(nk_counter *a) {
  std::lock_guard<std::mutex> g(g_hist_mu);
  a->hist_state = 2;
}

// c's pending K1b for a reader: 0 none, 1 still in the slot (now out of it),
// 2 enqueued (wait for hist_ev).  keep2: leave state 2 set (the histogram's
// kernel may still be writing c's partials).
int hist_claim(nk_counter *c, bool keep2) {
  for (;;) {
    {
      std::lock_guard<std::mutex> g(g_hist_mu);
      const int st = c->hist_state;
      if (st != 3) {
        if (st == 1) {
          HistSlot &h = slot_of(c->device);
          if (h.owner == c) h.owner = nullptr;
        }
        if (!(keep2 && st == 2)) c->hist_state = 0;
        return st;
      }
    }
    std::this_thread::yield();  // another thread is launching the kernel that took it
  }
}
}  // namespace

int hist_ready(nk_counter *c, hipStream_t s) {
  const int st = hist_claim(c, false);
  if (st == 1) HIPCHK(hist_run(c, s));
  else if (st == 2) HIPCHK(hipStreamWaitEvent(s, c->hist_ev, 0));
  return NK_OK;
}

int hist_arena(nk_counter *c, hipStream_t s) {
  // (state 1: the pending histogram is dropped, the arena is about to be rewritten)
  if (hist_claim(c, false) == 2) HIPCHK(hipStreamWaitEvent(s, c->hist_ev, 0));
  return NK_OK;
}

void hist_void(nk_counter *c) { (void)hist_claim(c, true); }

void hist_forget(nk_counter *c) {
  if (hist_claim(c, false) == 2) (void)hipEventSynchronize(c->hist_ev);
}

// a positive integer from the environment (tests: force the rare branches)
uint32_t env_u32(const char *name, uint32_t dflt) {
  const char *e = getenv(name);
  const unsigned long v = e ? strtoul(e, nullptr, 10) : 0;
  return v ? (uint32_t)v : dflt;
}

// defer_partials: leave K1c (currents += partials) to the LIF kernel of the
// same process call instead of a separate pass

int accumulate(nk_counter *c, const uint8_t *d_bases, const uint64_t *d_offs,
                      size_t n_recs, size_t n_bases, void *stream, bool defer_partials,
                      uint64_t first_pos) {
  if (!c) return fail(NK_E_INVALID, "null counter");
  if (n_bases && ((uintptr_t)d_bases & 15))
    return fail(NK_E_INVALID, "device bases must be 16-byte aligned");
  if (n_bases && !n_recs) return fail(NK_E_INVALID, "bases without records");
  if (c->pool == 0 && n_bases >= c->k)
    return fail(NK_E_INVALID, "pool_size 0 with k-mers present (the reference panics on % 0)");
  (void)hipSetDevice(c->device);
  hipStream_t s = pick_stream(c, stream);
  // a fused count of another handle may still read this handle's records
  if (int rc0 = hist_arena(c, s)) return rc0;
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
  const bool want_keyed = c->opts.exact_counts && c->k <= 32 && grouped_ok(c, n_bases);
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
    // K1a; with another handle's K1b pending on this stream, fused with it
    const bool fusable = !keyed && part_fused_ok(cp.pa) && in.n_tiles >= kFuseMinTiles;
    HistJob hj{};
    nk_counter *taken = fusable ? hist_take(c, s, in.n_tiles, hj) : nullptr;
    if (taken) {
      hipError_t e = launch_part_fused(in, (int)c->k, c->canonical, c->pool, cp.pa, hj, s);
      if (e != hipSuccess) {  // the taken histogram standalone, then this count's K1a
        (void)hipGetLastError();
        if (hist_run(taken, s) == hipSuccess) e = launch_part(in, (int)c->k, c->canonical, c->pool, cp.pa, s);
      }
      const hipError_t r = hipEventRecord(taken->hist_ev, s);
      hist_taken(taken);
      HIPCHK(e);
      HIPCHK(r);
    } else {
      HIPCHK(launch_part(in, (int)c->k, c->canonical, c->pool, cp.pa, s));
    }
    HIPCHK(mark(c, 2, s));
    c->last_pa = cp.pa;
    // this count's K1b: left to the next count on this stream, or now
    const uint32_t fs = fuse_slices(cp.slices);
    bool left = false;
    if (defer_partials && fusable && c->opts.defer_hist) {
      if ((rc = c->partials.ensure((uint64_t)fs * c->pool))) return rc;
      c->hist_slices = fs;
      left = hist_leave(c, s);
    }
    if (left) {
      c->pend_slices = fs;
    } else {
      HIPCHK(launch_bucket_hist(cp.pa, c->pool, cp.slices, c->partials.p, s));
      if (defer_partials)
        c->pend_slices = cp.slices;
      else
        HIPCHK(launch_partials_add(c->partials.p, cp.slices, c->pool, c->cur.p, s));
    }
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
extern "C" {

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
}  // extern "C"
