// nk_ingest_host.cpp — FASTA/FASTQ files counted as they are read
// (src/utils.rs:9-24 stream_sequences, src/spiking_hash.rs:277-486).
#include "nk_handle.h"

#include <unistd.h>

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

size_t ingest_chunk_bytes() {
  const char *e = getenv("NK_INGEST_CHUNK");  // tests: small chunks exercise the carries
  size_t v = e ? (size_t)strtoull(e, nullptr, 10) : 0;
  if (v < 64) v = (size_t)64 << 20;
  return v;
}

// An uncompressed FASTQ file: host threads read it window by window (each its
// slice, pread) and parse it (nk_fqhost.h); only each window's sequence bytes
// and record ends cross PCIe, straight into the resident input (bases,
// offsets), where the count takes them.  Three stages overlap: the read +
// parse of window w + 1, the H2D of window w (copy stream) and its count
// (count stream); the pinned output buffers rotate over three windows.
// Headers and quality lines never leave the host (~52 % of a 150-bp FASTQ's
// bytes: the device FASTQ parse shipped them all, 268 ms for config 3's 10 GB
// file, profiles/r04_s12).  64 MiB windows: config 3's 10 GB file in 164-169
// ms (16 MiB: 205-272, 4 MiB: 440 -- per-window costs, profiles/r05_g).
static size_t fq_window_bytes() {
  const char *e = getenv("NK_FQ_WINDOW");  // tests / A/B
  size_t v = e ? (size_t)strtoull(e, nullptr, 10) : 0;
  if (!v) {
    const char *ic = getenv("NK_INGEST_CHUNK");  // (tests: small windows like small chunks)
    v = ic ? (size_t)strtoull(ic, nullptr, 10) : (size_t)64 << 20;
  }
  return std::max<size_t>(v, 64);
}

// record ends a window's pinned buffer holds: one per 32 bytes (a 150-bp
// FASTQ record is ~330); windows of shorter records are taken in several calls
// (NK_FQ_MAX_REC, tests: a small cap takes every window in several calls)
static uint64_t max_rec_for(size_t w) {
  const char *e = getenv("NK_FQ_MAX_REC");
  const uint64_t forced = e ? strtoull(e, nullptr, 10) : 0ull;
  return forced ? forced : w / 32 + 1024;
}

static int ingest_fastq_host(nk_counter *c, const HostFile &hf, bool *fallback, hipStream_t s) {
  const int fd = hf.fd();
  const uint64_t fsize = hf.size();
  int rc;
  size_t win = fq_window_bytes();
  if ((rc = c->in_bases.ensure(fsize + 80)) || (rc = c->in_offs.ensure(std::max<size_t>(c->in_offs.n, 1025))))
    return rc;
  std::vector<uint8_t> rbuf;  // the window's file bytes (host memory, reused)
  auto buffers = [&](size_t w) -> int {
    rbuf.resize(w + 64);
    for (int i = 0; i < 3; ++i)
      if ((rc = c->ing_hb[i].ensure(w)) || (rc = c->ing_he[i].ensure(max_rec_for(w) * 8))) return rc;
    return NK_OK;
  };
  if ((rc = buffers(win))) return rc;
  if (!c->ing_cs) {
    HIPCHK(hipStreamCreateWithFlags(&c->ing_cs, hipStreamNonBlocking));
    for (hipEvent_t &e : c->ing_ev) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  }
  if (!c->fq_ev[0])
    for (hipEvent_t &e : c->fq_ev) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  hipStream_t cs = c->ing_cs;
  // every exit leaves no copy in flight from the pinned buffers
  struct Drain {
    hipStream_t cs;
    ~Drain() { (void)hipStreamSynchronize(cs); }
  } drain{cs};
  bool used[3] = {false, false, false};  // the buffer has an H2D in flight (its event)
  StreamAcc sa;
  if ((rc = acc_begin(c, fsize / 2, win + 64, sa, s))) return rc;
  HIPCHK(hipMemsetAsync(c->in_offs.p, 0, 8, s));  // offsets[0]
  static const bool prof = getenv("NK_INGEST_PROFILE") != nullptr;
  using clk = std::chrono::steady_clock;
  double t_parse = 0, t_enq = 0;
  uint64_t n_win = 0;
  auto since = [](clk::time_point a) { return std::chrono::duration<double, std::milli>(clk::now() - a).count(); };
  // The host parses window w while the copy engine moves window w - 1 up and
  // the device counts it (the parse waits only for the H2D that last read the
  // pinned buffers it writes, window w - 3's).
  uint64_t pos = 0, data_end = 0, n_rec = 0, counted = 0;
  int b = 0;
  for (;;) {
    const size_t len = (size_t)std::min<uint64_t>(win, fsize - pos);
    const bool eof = pos + len >= fsize;
    const clk::time_point t0 = clk::now();
    if (used[b]) HIPCHK(hipEventSynchronize(c->fq_ev[b]));
    const FqResult r = fq_extract(rbuf.data(), len, eof, c->ing_hb[b].p,
                                  reinterpret_cast<uint64_t *>(c->ing_he[b].p), data_end, shared_host_pool(), fd,
                                  pos, &c->fq_scratch, max_rec_for(len));
    if (prof) t_parse += since(t0);
    ++n_win;
    if (!r.io_error.empty()) return fail(NK_E_IO, "%s: %s", hf.path().c_str(), r.io_error.c_str());
    if (!r.n_rec && !r.stop && !r.blank && !eof) {
      // a record longer than the window: widen it (no copy may read the buffers)
      if (win >= ((size_t)1 << 31)) return fail(NK_E_PARSE, "a FASTQ record longer than 2 GiB");
      HIPCHK(hipStreamSynchronize(cs));
      HIPCHK(hipStreamSynchronize(s));
      win *= 2;
      if ((rc = buffers(win))) return rc;
      used[0] = used[1] = used[2] = false;
      continue;
    }
    if (r.blank) {  // a blank line between records: the host reader takes the file
      *fallback = true;
      return NK_OK;
    }
    const clk::time_point t1 = clk::now();
    const bool last = r.stop || (eof && !r.more);
    if (r.stop)  // (src/utils.rs:17-19: the reference warns and ends the stream there)
      warn_malformed(hf.path().c_str(), n_rec + r.n_rec, "a FASTQ record is malformed or cut off");
    if (n_rec + r.n_rec + 1 > c->in_offs.n) {  // grow the offsets: wait, copy, free
      HIPCHK(hipStreamSynchronize(cs));
      HIPCHK(hipStreamSynchronize(s));
      DevBuf<uint64_t> no;
      if ((rc = no.ensure(std::max<uint64_t>(n_rec + r.n_rec + 1, 2 * c->in_offs.n)))) return rc;
      HIPCHK(hipMemcpy(no.p, c->in_offs.p, (n_rec + 1) * 8, hipMemcpyDeviceToDevice));
      std::swap(no.p, c->in_offs.p);
      std::swap(no.n, c->in_offs.n);
      no.release();
    }
    if (r.n_bases)
      HIPCHK(hipMemcpyAsync(c->in_bases.p + data_end, c->ing_hb[b].p, r.n_bases, hipMemcpyHostToDevice, cs));
    if (r.n_rec)
      HIPCHK(hipMemcpyAsync(c->in_offs.p + 1 + n_rec, c->ing_he[b].p, r.n_rec * 8, hipMemcpyHostToDevice, cs));
    HIPCHK(hipEventRecord(c->fq_ev[b], cs));
    used[b] = true;
    HIPCHK(hipStreamWaitEvent(s, c->fq_ev[b], 0));
    data_end += r.n_bases;
    n_rec += r.n_rec;
    KmerInput whole{};
    whole.bases = c->in_bases.p;
    whole.offsets = c->in_offs.p;
    whole.n_recs = n_rec;
    whole.n_bases = data_end;
    if (n_rec && data_end > counted) {
      if ((rc = acc_batch(c, sa, whole, counted, data_end, s))) return rc;
      counted = data_end;
    }
    if (prof) t_enq += since(t1);
    if (last) {
      if ((rc = acc_end(c, sa, whole, s))) return rc;
      break;
    }
    pos += r.consumed;
    b = (b + 1) % 3;
  }
  if (prof)
    fprintf(stderr, "[nk ingest fastq host] windows %llu  parse %.1f ms  enqueue %.1f ms\n",
            (unsigned long long)n_win, t_parse, t_enq);
  return NK_OK;
}

// Parse a FASTA/FASTQ file on the device in chunks and count it as it arrives
// (src/spiking_hash.rs:277-486 semantics for the records; the caller runs the
// LIF rule).  *fallback: the file needs the host reader (a blank line between
// FASTQ records).
int ingest_file(nk_counter *c, const char *path, bool *fallback) {
  *fallback = false;
  {
    // uncompressed FASTQ: the host extraction (NK_FASTQ_DEVICE=1, tests and
    // A/B: the device parse of every byte, as gzip input still takes)
    HostFile hf;
    std::string ferr;
    uint8_t b0 = 0;
    if (hf.open(path, ferr) == NK_OK && hf.size() && pread(hf.fd(), &b0, 1, 0) == 1 && b0 == '@' &&
        !getenv("NK_FASTQ_DEVICE")) {
      (void)hipSetDevice(c->device);
      return ingest_fastq_host(c, hf, fallback, pick_stream(c, nullptr));
    }
  }
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
  // a chunk is read in pieces (the reader thread) and each piece goes up as
  // soon as it is in (upload_pieces), so a chunk's H2D overlaps its own read:
  // a 117 MB FASTA took 5.3 ms with whole-chunk uploads, the read and the
  // copy of each 64 MiB chunk one after the other
  const size_t piece = std::min<size_t>(chunk, (size_t)16 << 20);
  std::atomic<size_t> ready[3];
  std::future<size_t> next;
  auto prefetch = [&](int b) {
    ready[b].store(0, std::memory_order_relaxed);
    std::atomic<size_t> *rp = &ready[b];
    next = std::async(std::launch::async, [&src, hb, b, chunk, piece, rp] {
      size_t got = 0;
      while (got < chunk) {
        const size_t want = std::min(piece, chunk - got);
        const size_t n = src.read(hb[b].p + got, want);
        got += n;
        rp->store(got, std::memory_order_release);
        if (n < want) break;  // the end of the input (or a failed read: src.failed())
      }
      return got;
    });
  };
  prefetch(0);
  // the format from the first bytes in
  while (!ready[0].load(std::memory_order_acquire) &&
         next.wait_for(std::chrono::microseconds(20)) != std::future_status::ready) {
  }
  if (!ready[0].load(std::memory_order_acquire)) {
    (void)next.get();
    if (src.failed()) return fail(NK_E_IO, "%s: %s", path, src.why().c_str());
    return fail(NK_E_PARSE, "empty file");
  }
  const bool fastq = hb[0].p[0] == '@';
  if (hb[0].p[0] != '>' && !fastq) {
    (void)next.get();
    return fail(NK_E_PARSE, "unknown format: first byte is neither '>' nor '@'");
  }
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
  // the chunk the reader fills into host buffer hb -> draws[b] + room on the
  // copy stream, piece by piece as the reader has them (once the carry out of
  // that buffer and its parse are done); *n = its bytes
  auto upload_pieces = [&](int b, int hbi, size_t *n) -> int {
    if (used[b]) HIPCHK(hipStreamWaitEvent(cs, ev_free[b], 0));
    size_t up = 0;
    for (;;) {
      const bool done = next.wait_for(std::chrono::seconds(0)) == std::future_status::ready;
      const size_t r = ready[hbi].load(std::memory_order_acquire);  // (final once done)
      if (r > up) {
        HIPCHK(hipMemcpyAsync(draws[b]->p + room + up, hb[hbi].p + up, r - up, hipMemcpyHostToDevice, cs));
        up = r;
      }
      if (done) break;
      (void)next.wait_for(std::chrono::microseconds(20));
    }
    *n = next.get();
    HIPCHK(hipEventRecord(ev_copied[b], cs));
    return NK_OK;
  };
  size_t have = 0;
  if ((rc = upload_pieces(0, 0, &have))) return rc;
  if (src.failed()) return fail(NK_E_IO, "%s: %s", path, src.why().c_str());
  bool eof = have < chunk;
  if (!eof) prefetch(1);
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
      if ((rc = upload_pieces(db ^ 1, (int)((ci + 1) % 3), &got))) return rc;
      if (prof) t_read += since(t2);
      if (src.failed()) return fail(NK_E_IO, "%s: %s", path, src.why().c_str());
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
    if (st.stop)  // (src/utils.rs:17-19: the reference warns and ends the stream there)
      warn_malformed(path, st.n_rec, src.damage().empty() ? "a FASTQ record is malformed or cut off"
                                                          : src.damage().c_str());
    else if (eof && !src.damage().empty())  // (a FASTA record cut by a damaged stream)
      warn_malformed(path, st.n_rec ? st.n_rec - 1 : 0, src.damage().c_str());
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
