/*
 * neurokmer.h — C ABI of the MI355X-native NeuroKmer k-mer -> spike hot path.
 *
 * Drop-in boundary for the reference crate's `SpikingKmerCounter`
 * (MrObadiahEJ/NeuroKmer, src/spiking_hash.rs).  Every entry point below names
 * the reference item it replaces.  Plain C types only: pointers + sizes, no
 * torch or HIP types.  Return convention: 0 = OK, negative = NK_E_* code; the
 * message of the last failure on the calling thread is nk_last_error().  No
 * C++ exception crosses this boundary.  One handle is used by one thread at a
 * time (the reference's `&mut self`).
 *
 * Compute runs on one AMD Instinct MI355X (gfx950) per handle.  There is no CPU
 * fallback: nk_new() fails with NK_E_NO_DEVICE when no gfx950 device is
 * present.
 */
#ifndef NEUROKMER_H
#define NEUROKMER_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NK_ABI_VERSION 1

/* error codes */
#define NK_OK 0
#define NK_E_INVALID (-1)     /* bad argument (k == 0, pool == 0 with k-mers, ...) */
#define NK_E_NO_DEVICE (-2)   /* no usable gfx950 device / HIP runtime failure */
#define NK_E_OOM (-3)         /* device or host allocation failed */
#define NK_E_IO (-4)          /* file open/read failure */
#define NK_E_PARSE (-5)       /* FASTA/FASTQ parse failure (empty file, bad first byte) */
#define NK_E_UNSUPPORTED (-6) /* feature not available in this build / for these arguments */
#define NK_E_DEVICE (-7)      /* kernel launch or device-side failure */

typedef struct nk_counter nk_counter;

/* k-mer key width.  NK_KMER_COMPAT reproduces the reference's release-build
 * u64 semantics for every k (k > 32 keeps the last 32 forward bases and the
 * reference's masked-shift reverse strand, src/models.rs:188,192-194,260-266).
 * NK_KMER_128 is the build's true k <= 64 mode (not in the
 * reference): u128 keys (canonical = min(fwd, rev) over 2k bits; non-canonical
 * = pack_kmer in 128 bits), neuron = SipHash-1-3(key 0) over the key's 16 LE
 * bytes % pool.  Its keys cross this ABI as (lo, hi) pairs of u64. */
#define NK_KMER_COMPAT 0
#define NK_KMER_128 1

typedef struct nk_opts {
  int32_t device;        /* HIP device ordinal (default 0) */
  int32_t kmer_width;    /* NK_KMER_COMPAT (default) or NK_KMER_128 */
  uint32_t top_n;        /* neurons whose "unique k-mers colliding" are tracked
                            by every process call (default 20 = src/main.rs:50) */
  uint32_t stage_timing; /* 0 (default): HIP events around the count kernel only
                            (nk_last_timings: index, count, post, total);
                            1: an event between every stage (each costs ~6 us
                            of GPU idle time on MI355X);
                            2: events at both ends of a call only (no event
                            between two kernels; no count-kernel time);
                            3: no events (nk_last_timings reports nothing;
                            nk_count_spans still times the count kernel) */
  uint32_t exact_counts; /* 1: build the exact k-mer count table on the device
                            (the reference's `counts` DashMap and the full
                            `kmer_per_neuron`, src/spiking_hash.rs:27,157-172)
                            in every process/accumulate call.  Default 0: the
                            metric's path (uniques of the top_n rows only); the
                            table of the last input is then built on demand by
                            nk_get_count(s)/nk_get_counts128, nk_distinct_kmers,
                            nk_copy_kmer_per_neuron, nk_top_abundant_neurons
                            past top_n rows and nk_process_sequence — provided
                            the handle holds that input (host-array and file
                            entry points; device input passed by pointer is the
                            caller's: those calls then return NK_E_UNSUPPORTED
                            unless exact_counts = 1).  The multi-GPU exact
                            table (nk_exact_*) needs exact_counts = 1 and
                            NK_KMER_COMPAT keys. */
  uint32_t defer_hist;   /* 1: batches in flight on one stream (several handles
                            counting one after the other, each finish on another
                            stream): a one-level partitioned count (k <= 32,
                            pool <= 4.2 M canonical, <= 8.4 M otherwise)
                            leaves its bucket histogram (K1b) pending and the
                            next such count on the same stream and host thread
                            -- of another handle -- runs it inside its own hash
                            kernel (k_part_fused), where it takes HBM and LDS
                            time the hash leaves idle.  The results are the
                            same; whatever reads this handle's counts first
                            waits for that kernel (or runs the histogram itself
                            when no count took it).  Default 0: each count
                            histograms its own records.  (Measured slower on
                            the bench's three batches in flight: the other
                            batches' finish kernels wait for the longer
                            fused kernel) */
  uint32_t reserved[10];
} nk_opts;

/* Fills *o with the defaults above. */
void nk_opts_default(nk_opts *o);

/* SpikingKmerCounter::new(k, threshold, leak, refractory, spike_cost,
 * pool_size, use_canonical)  — src/spiking_hash.rs:40-77.
 * opts may be NULL.  Returns NULL on failure (see nk_last_error()). */
nk_counter *nk_new(size_t k, float threshold, float leak, uint32_t refractory,
                   double spike_cost, size_t pool_size, int use_canonical,
                   const nk_opts *opts);
void nk_free(nk_counter *c);

/* SpikingKmerCounter::process_parallel(&mut self, seqs: &[Vec<u8>])
 * — src/spiking_hash.rs:84-201.  Host records: record i is
 * bases[rec_offsets[i] .. rec_offsets[i+1]), rec_offsets has n_recs+1 entries,
 * rec_offsets[0] == 0.  Borrowed for the duration of the call. */
int nk_process_parallel(nk_counter *c, const uint8_t *bases,
                        const uint64_t *rec_offsets, size_t n_recs);

/* Same, with bases and rec_offsets already resident in device memory of the
 * handle's device (16-byte aligned `d_bases`).  `stream` is a hipStream_t or
 * NULL for the handle's own stream.  n_bases == rec_offsets[n_recs]. */
int nk_process_parallel_device(nk_counter *c, const uint8_t *d_bases,
                               const uint64_t *d_rec_offsets, size_t n_recs,
                               size_t n_bases, void *stream);

/* SpikingKmerCounter::process_file_streaming(&mut self, path)
 * — src/spiking_hash.rs:277-486 (FASTA/FASTQ, format from the first byte;
 * gzip read transparently).  The file is parsed on the device in chunks that
 * are counted as they arrive (GPU FASTX ingest, needletail's rules as the host
 * reader restates them); a FASTQ file with blank lines between records goes
 * through the host reader instead. */
int nk_process_file_streaming(nk_counter *c, const char *path);
/* The CLI's in-memory mode from a file: stream_sequences(path).collect() then
 * process_parallel (src/main.rs:40-46), through the same GPU ingest. */
int nk_process_file_parallel(nk_counter *c, const char *path);

/* Split-phase form of the two calls above, for multi-GPU use (one process per
 * GPU; the caller all-reduces the u64 currents between the phases):
 *   nk_accumulate_device   — zero + accumulate this shard's currents
 *   <caller: allreduce(nk_device_currents(c), pool_size u64, sum)>
 *   nk_finalize            — LIF + top-N (+ uniques of this shard's k-mers)
 * `streaming_semantics` = 1 applies process_file_streaming's LIF rule (zero
 * current neurons also step, src/spiking_hash.rs:544-659), 0 process_parallel's
 * (they are skipped, :189-191).
 * Calls of one handle stay ordered across streams: a call on another stream
 * than the handle's previous one first waits for that call's work (after
 * nk_accumulate_device: for exactly its work, recorded when it returns, so
 * another handle's batch queued behind it is not waited for). */
int nk_accumulate_device(nk_counter *c, const uint8_t *d_bases,
                         const uint64_t *d_rec_offsets, size_t n_recs,
                         size_t n_bases, void *stream);
int nk_finalize(nk_counter *c, int streaming_semantics, void *stream);
/* The same split-phase step with ONE host synchronisation (what
 * neurokmer_amd/dist.py::finalize_step runs; the caller's collectives go on
 * `stream` between the calls):
 *   nk_accumulate_device
 *   nk_wire32            — this shard's currents as u32 into d_wire[pool_size]
 *                          (valid while all ranks' k-mers together < 2^31;
 *                          else all-reduce nk_device_currents as u64 and pass
 *                          d_wire = NULL below)
 *   <caller: allreduce(d_wire, pool_size u32, sum)>
 *   nk_finalize_export   — LIF from the reduced wire vector, top-N, this
 *                          shard's distinct top k-mers into d_seg[1 + w*cap]
 *                          ([n | flags << 56, keys...], w = 1, or 2 for 128-bit
 *                          keys as (lo, hi)); enqueued, no wait
 *   <caller: allgather(d_seg) -> d_buf[world * stride]>
 *   nk_merge_export      — union of the segments -> uniques column, results
 *                          read back (one wait); *redo = 1 when any rank could
 *                          not export exactly (a full set, an overflowed top
 *                          bucket, a top-N past the histogram, more than cap
 *                          keys): every rank then sees the same *redo and
 *                          calls nk_finalize_redo and the blocking exchange
 *                          (nk_top_kmers_padded / nk_merge_top_kmers_padded).
 * Not with opts.exact_counts (NK_E_UNSUPPORTED: use nk_finalize). */
int nk_wire32(nk_counter *c, uint32_t *d_wire, void *stream);
int nk_finalize_export(nk_counter *c, int streaming_semantics, const uint32_t *d_wire,
                       uint64_t *d_seg, size_t cap, void *stream);
int nk_merge_export(nk_counter *c, const uint64_t *d_buf, size_t world, size_t stride,
                    size_t cap, int *redo, void *stream);
int nk_finalize_redo(nk_counter *c, void *stream);
/* Pool-sliced finish for very large pools (config 5: P up to 2^31 over W ranks;
 * neurokmer_amd/dist.py::finalize_step_sliced).  Rank r owns the neurons
 * [lo, hi) = [r*S, min(P, (r+1)*S)), S = ceil(P / W):
 *   nk_accumulate_device (+ nk_wire32 into a W*S-entry wire, zero-padded, or the
 *                          u64 currents copied into a W*S-entry buffer)
 *   <caller: reduce_scatter(wire) -> this rank's S summed entries d_slice>
 *   nk_finalize_slice   — LIF of [lo, hi) only from d_slice (u32 or u64 per
 *                         slice_bits), the slice's top rows into d_seg:
 *                         [rows, new spikes, max spike count, (idx, spikes,
 *                         current) x rows], seg_rows >= min(top_n, pool);
 *                         one host synchronisation
 *   <caller: all-gather(d_seg) -> d_all[world * stride], stride >= 3 + 3*seg_rows>
 *   nk_adopt_slices     — the global top rows (every global top row is among
 *                         its slice's), total spikes and energy, this shard's
 *                         uniques pass for those rows
 *   <caller: the union of the shards' keys — nk_top_kmers_padded /
 *                         nk_merge_top_kmers_padded, as after nk_finalize>
 * Afterwards v / refractory / spike counts / currents are authoritative on
 * [lo, hi) only (the other ranks own the rest): until nk_reset, the calls that
 * run the LIF or read the whole pool (nk_finalize, nk_finalize_export, the
 * process calls, nk_process_sequence, nk_simulate_spikes_auto and rows past
 * top_n in nk_top_abundant_neurons) return NK_E_UNSUPPORTED; further
 * accumulate + nk_finalize_slice steps are allowed.  Replaces the reference's
 * single-process pool (src/spiking_hash.rs:49-53,97,186-200). */
int nk_finalize_slice(nk_counter *c, int streaming_semantics, const void *d_slice, int slice_bits,
                      size_t lo, size_t hi, uint64_t *d_seg, size_t seg_rows, void *stream);
int nk_adopt_slices(nk_counter *c, const uint64_t *d_all, size_t world, size_t stride,
                    void *stream);
/* The same pool-sliced finish with no host wait until nk_merge_export (u32
 * slices; world * top_n <= 2048):
 *   nk_slice_export  LIF of [lo, hi) from the reduce-scattered u32 slice and
 *                    the slice's top rows into d_seg (3 + 3*seg_rows words),
 *                    by kernels;
 *   <all-gather of the d_seg segments>
 *   nk_adopt_export  the global rows picked on the device from the gathered
 *                    segments, this shard's uniques pass for them, its new
 *                    keys appended to d_keyseg (1 + key_words*cap words, the
 *                    layout of nk_finalize_export);
 *   <all-gather of the key segments>
 *   nk_merge_export  as after nk_finalize_export; on *redo = 1 the blocking
 *                    path follows (a slice's spike counts past 4095 need the
 *                    exact refine; the set or a bucket overflowed; a segment
 *                    was truncated).  nk_finalize_sliced_dist runs all of it. */
int nk_slice_export(nk_counter *c, int streaming_semantics, const uint32_t *d_slice, size_t lo,
                    size_t hi, uint64_t *d_seg, size_t seg_rows, void *stream);
int nk_adopt_export(nk_counter *c, const uint64_t *d_all, size_t world, size_t stride,
                    uint64_t *d_keyseg, size_t cap, void *stream);
/* ---- multi-GPU step with the collectives inside the library ---------------
 * One communicator per rank (RCCL over xGMI; one process per GPU): rank 0
 * makes an id, the caller broadcasts it (e.g. torch.distributed), every rank
 * builds its communicator from it.  Replaces the reference's single-process
 * rayon reduce of the currents (src/spiking_hash.rs:145-154) across GPUs. */
#define NK_COMM_ID_BYTES 128
typedef struct nk_comm nk_comm;
int nk_comm_unique_id(uint8_t id[NK_COMM_ID_BYTES]);
nk_comm *nk_comm_new(const uint8_t id[NK_COMM_ID_BYTES], int world, int rank, int device);
void nk_comm_free(nk_comm *m);
/* Drop the device buffers m holds for handle c (wire, export and all-gather
 * segments); call before nk_free(c) when m outlives c.  nk_comm_free drops
 * every handle's. */
void nk_comm_forget(nk_comm *m, const nk_counter *c);
/* Loopback transport (tests and one-GPU rehearsals; not an RCCL replacement):
 * `world` ranks as host threads of ONE process on one device, each with its
 * own nk_comm_new_loopback communicator, every collective done by device
 * copies and a sum kernel between host barriers (a rank that does not arrive
 * within 120 s fails every rank's call).  RCCL refuses two ranks on one
 * device, so this is how nk_finalize_dist / nk_finalize_sliced_dist run at
 * world > 1 on a one-GPU box.  world: 1 .. 16.  Each rank joins once (a second
 * communicator for a live rank fails; nk_comm_free leaves the group).  A
 * group that broke (a rank failed or timed out) stays broken: every later
 * collective fails, so free it and make a new one. */
typedef struct nk_loop_group nk_loop_group;
nk_loop_group *nk_loop_group_new(int world);
void nk_loop_group_free(nk_loop_group *g);  /* after every member's nk_comm_free */
nk_comm *nk_comm_new_loopback(nk_loop_group *g, int rank, int device);
/* After nk_accumulate_device(_from) on every rank: the whole multi-GPU finish
 * enqueued on `stream` with no host code between the steps (the same protocol
 * as nk_wire32 .. nk_merge_export above, the all-reduce and all-gather issued
 * by the library):
 *   u32 wire + all-reduce (u64 currents when total_kmers >= 2^31), LIF + top-N
 *   + this shard's top k-mers into a segment of `cap` keys, all-gather of the
 *   segments, their union -> uniques column, one host wait; a redo (full set,
 *   overflowed bucket, truncated segment: every rank sees the same headers)
 *   takes the blocking exchange, still inside.
 * total_kmers: an upper bound of all ranks' k-mers together (the same on
 * every rank).  With an adopted multi-GPU exact table (nk_exact_adopt) the
 * currents are all-reduced as u64 and the uniques come from kmer_per_neuron. */
int nk_finalize_dist(nk_counter *c, nk_comm *m, int streaming_semantics, uint64_t total_kmers,
                     size_t cap, void *stream);
/* The pool-sliced finish (nk_finalize_slice / nk_adopt_slices) with its
 * reduce-scatter, all-gather and the top k-mer union inside the library. */
int nk_finalize_sliced_dist(nk_counter *c, nk_comm *m, int streaming_semantics,
                            uint64_t total_kmers, size_t cap, void *stream);

/* nk_accumulate_device counting only the windows that start at or after
 * first_pos (bases before it are context: a shard cut inside a record of a
 * k > 32 NK_KMER_COMPAT input keeps a 32-base warm-up, after which the
 * reference's rolling reverse strand no longer depends on the record start,
 * src/models.rs:260-266). */
int nk_accumulate_device_from(nk_counter *c, const uint8_t *d_bases,
                              const uint64_t *d_rec_offsets, size_t n_recs, size_t n_bases,
                              size_t first_pos, void *stream);
/* After nk_finalize on a shard: the distinct k-mer keys of this shard that map
 * to the current top-N neurons (device buffer owned by the handle, valid until
 * the next call).  The caller gathers every shard's list and hands the union
 * to nk_merge_top_kmers(), which recomputes the uniques column exactly.
 * NK_KMER_128: the buffer holds n_keys (lo, hi) pairs (2 * n_keys u64). */
int nk_top_kmers(nk_counter *c, const uint64_t **d_keys, size_t *n_keys);
int nk_merge_top_kmers(nk_counter *c, const uint64_t *d_keys, size_t n_keys, void *stream);
/* The same exchange with one fixed-size all-gather and no host round trip:
 * nk_top_kmers_padded writes [n, key 0 .. key min(n, cap)-1] (n = this
 * shard's key count; NK_KMER_128 keys take two words) to d_out on `stream`;
 * the caller all-gathers world such segments of `stride` u64 words (stride
 * >= 1 + cap, or 1 + 2 cap for NK_KMER_128) and nk_merge_top_kmers_padded
 * recomputes the uniques column from them.  *complete = 0 when a segment held
 * more than cap keys (every rank sees the same headers): the top rows are left
 * unchanged and the caller falls back to nk_top_kmers + nk_merge_top_kmers. */
int nk_top_kmers_padded(nk_counter *c, uint64_t *d_out, size_t cap, void *stream);
int nk_merge_top_kmers_padded(nk_counter *c, const uint64_t *d_buf, size_t world,
                              size_t stride, size_t cap, int *complete, void *stream);

/* SpikingKmerCounter::top_abundant_neurons(&self, n) — src/spiking_hash.rs:661-673.
 * Writes min(n, pool_size) rows into out (caller-allocated), returns the count
 * written, or a negative error.  Rows are ordered by spikes descending, ties
 * by ascending neuron index (the reference's stable sort).  `uniques` is the
 * neuron's kmer_per_neuron: the distinct k-mers of the last process call
 * mapped to it (+1 per process_sequence record touching it).  Any n: the
 * opts.top_n rows come with every process call; more rows rank the whole pool
 * on the device and take the uniques from the exact table (see exact_counts
 * for when that table can be built on demand). */
typedef struct nk_top_row {
  uint64_t idx;
  uint64_t spikes;
  uint32_t uniques;
  uint32_t _pad;
} nk_top_row;
long nk_top_abundant_neurons(nk_counter *c, size_t n, nk_top_row *out);

/* SpikingKmerCounter::get_count(&self, kmer) — src/spiking_hash.rs:675-682:
 * *present = 1 and *out = the k-mer's count (u32, wrapping like AtomicU32), or
 * *present = 0.  The table: see nk_opts.exact_counts.  NK_KMER_COMPAT keys
 * (NK_KMER_128 handles: nk_get_counts128). */
int nk_get_count(nk_counter *c, uint64_t kmer, uint32_t *out, int *present);
/* SpikingKmerCounter::process_sequence(&mut self, seq) — src/spiking_hash.rs:
 * 203-273: one record; counts[key] += 1 per k-mer, currents[H(key) % P] += 1
 * on top of the currents already held, kmer_per_neuron[idx] += 1 per neuron
 * the record touches, then ONE LifNeuron::update(current as f32) for every
 * neuron with current > 0 and currents = 0.  len < k: no-op.  The uniques
 * column is kmer_per_neuron, so the table of the previous process call is
 * built first when it is still pending (see exact_counts).  NK_KMER_COMPAT
 * keys (the reference's u64 map); NK_E_UNSUPPORTED for NK_KMER_128. */
int nk_process_sequence(nk_counter *c, const uint8_t *seq, size_t len);
/* Batched get_count over host arrays (out[i], present[i] per key). */
int nk_get_counts(nk_counter *c, const uint64_t *kmers, size_t n, uint32_t *out,
                  uint8_t *present);
/* NK_KMER_128 handles: get_count of n u128 keys given as (lo, hi) pairs
 * (kmers2[2i], kmers2[2i+1]).  (No reference counterpart: the reference keys
 * are u64; the table's counts wrap at 2^32 like the u64 table's.) */
int nk_get_counts128(nk_counter *c, const uint64_t *kmers2, size_t n, uint32_t *out,
                     uint8_t *present);
/* Number of distinct k-mers in the table (the reference's counts.len()). */
long nk_distinct_kmers(nk_counter *c);
/* The full `kmer_per_neuron` (src/spiking_hash.rs:28,167-172,262-267): out[i]
 * for every neuron i < pool (n must equal pool_size).  The table: see
 * nk_opts.exact_counts (built with every call, or on demand from the last
 * input the handle holds). */
int nk_copy_kmer_per_neuron(nk_counter *c, uint32_t *out, size_t n);

/* SpikingKmerCounter::simulate_spikes_auto(&mut self) — src/spiking_hash.rs:
 * 697-714.  On x86-64 with AVX2 (the reference's target and an MI355X node's
 * host) that is simulate_spikes_simd (:544-659): `steps` LifNeuron updates of
 * EVERY neuron (zero currents included) from the currents the counter holds
 * (the last process call's; zero after process_sequence), spikes added to the
 * neurons' counts and the energy tracker; steps == 0 does nothing.  The top
 * rows are re-selected; their uniques column is kmer_per_neuron when the handle
 * holds the table, else the distinct k-mers of the last input (device input
 * passed by pointer must still be resident, as for nk_finalize).
 * NK_E_UNSUPPORTED after nk_finalize_slice (sharded state) until nk_reset. */
int nk_simulate_spikes_auto(nk_counter *c);

/* Multi-GPU exact table (hash partition + all-to-all), after
 * an accumulate/process call with exact_counts on every rank (one process per
 * GPU; replaces the reference's single DashMap, src/spiking_hash.rs:27,
 * 157-165):
 *   nk_exact_partition  — this rank's (key, count) pairs grouped by owner rank
 *                         (device buffers owned by the handle, valid until the
 *                         next call; send_counts[r] = pairs for rank r, host)
 *   <caller: all-to-all of the keys (u64) and counts (u32) with those splits>
 *   nk_exact_adopt      — the received pairs become this rank's table (sorted,
 *                         counts of equal keys summed, u32 wrapping) and
 *                         kmer_per_neuron = the owned keys' contribution
 *   <caller: allreduce(nk_device_kmer_per_neuron(c), pool_size u32, sum)>
 *   nk_finalize         — the uniques column comes from kmer_per_neuron
 * Afterwards nk_get_count(s) answers for the keys this rank owns
 * (nk_exact_owner(key, world) == rank) and nk_distinct_kmers counts them; the
 * caller routes queries (neurokmer_amd/dist.py).  COMPAT keys only. */
uint32_t nk_exact_owner(uint64_t kmer, uint32_t world);
int nk_exact_partition(nk_counter *c, uint32_t world, uint64_t *send_counts,
                       const uint64_t **d_keys, const uint32_t **d_counts, void *stream);
int nk_exact_adopt(nk_counter *c, const uint64_t *d_keys, const uint32_t *d_counts,
                   size_t n, void *stream);
/* Device pointer of kmer_per_neuron (u32, pool_size entries; exact_counts). */
uint32_t *nk_device_kmer_per_neuron(nk_counter *c);

/* EnergyTracker / accessors — src/models.rs:145-173, src/spiking_hash.rs:684-695 */
uint64_t nk_total_spikes(const nk_counter *c);        /* energy.total_spikes() */
double nk_energy_used(const nk_counter *c);           /* energy_used() */
void nk_set_steps(nk_counter *c, uint64_t steps);     /* set_steps */
uint64_t nk_get_steps(const nk_counter *c);           /* get_steps */
size_t nk_pool_size(const nk_counter *c);
size_t nk_k(const nk_counter *c);
int nk_use_canonical(const nk_counter *c);

/* Parity views (device -> host copies of per-neuron state; n = pool_size). */
int nk_copy_currents(nk_counter *c, uint64_t *out, size_t n);
int nk_copy_spike_counts(nk_counter *c, uint64_t *out, size_t n);
int nk_copy_voltages(nk_counter *c, float *out, size_t n);
int nk_copy_refractory(nk_counter *c, uint32_t *out, size_t n);
/* Device pointer of the u64 currents vector (pool_size entries).  Pending
 * partial sums are folded first.  The vector is complete on the stream of the
 * last call that passed one; after a call on the handle's own stream (NULL)
 * this waits for that stream, so any stream may read it.  NULL on error. */
uint64_t *nk_device_currents(nk_counter *c);
/* Write out the per-neuron state (voltages, refractory counters, spike counts)
 * that the last finish left derived.  A finish from the reset state leaves
 * them as a function of the currents (nothing reads them in a typical step);
 * every reader (nk_copy_*, a further process call) writes them out first, so
 * results never differ.  The reference writes them in every call
 * (src/spiking_hash.rs:186-200): bench.py times a step plus this call to show
 * what that costs.  Enqueued on `stream` (NULL: the handle's stream). */
int nk_settle(nk_counter *c, void *stream);
/* Resets neurons, currents and energy to the state nk_new() left them in. */
int nk_reset(nk_counter *c);
/* Same, enqueued on `stream` (hipStream_t or NULL for the handle's stream)
 * without waiting for it. */
int nk_reset_async(nk_counter *c, void *stream);

/* Per-stage device timings of the last process/finalize call, milliseconds
 * (hipEvents on the stream the kernels ran on).  Returns the number of stages
 * written (<= cap); names are static strings. */
int nk_last_timings(const nk_counter *c, const char **names, float *ms, int cap);
/* Device time of the count kernel (K1: hash + partition/count) of each of the
 * last min(cap, 256) accumulate/process calls, oldest first, milliseconds
 * (hipEvents around the launch on its stream).  Lets a benchmark read every
 * timed step's K1 duration after its timed loop.  Returns the number written.
 * (No reference counterpart: measurement only.) */
int nk_count_history(const nk_counter *c, float *ms, int cap);
/* Sets nk_opts.stage_timing (0 .. 3) for later calls on this handle, e.g. 3
 * for timed benchmark steps and 0 for a separate count-kernel measurement.
 * (No reference counterpart: measurement only.) */
int nk_set_stage_timing(nk_counter *c, uint32_t level);
/* Duration in ms of the partitioned count kernel (K1a) of each of the last
 * min(cap, 256) accumulate/process calls that ran it, oldest first, from
 * in-kernel s_memrealtime stamps (earliest workgroup start to latest
 * workgroup end): no event sits in the stream, so it is also valid with
 * stage_timing 2.  Synchronises the handle's stream.  -> count, or < 0.
 * (No reference counterpart: measurement only.) */
int nk_count_spans(nk_counter *c, float *ms, int cap);
/* The same launches' raw [start, end] stamps (s_memrealtime, 10 ns ticks of the
 * device's constant clock, one clock for every handle on the device), two words
 * per launch, oldest first: the gap between one handle's K1a end and another's
 * next K1a start, with nothing in the stream.  -> launches, or < 0.
 * (No reference counterpart: measurement only.) */
int nk_count_stamps(nk_counter *c, unsigned long long *ticks, int cap);
/* Diagnostic: the best of `reps` device times (ms) of a kernel that computes
 * SipHash-1-3 (key 0) of n_keys u64 keys generated in registers plus the exact
 * `% pool` (nk_device.h: sip13_u64 + fastmod32, the count kernel's per-k-mer
 * hash work with no memory traffic).  Measures the VALU floor of the count
 * kernel live on the device.  (No reference counterpart.) */
int nk_diag_hash_ms(int device, uint64_t n_keys, uint64_t pool, int reps, float *ms);
/* The same for width 128: SipHash-1-3 over 16-byte keys (NK_KMER_128, the
 * config-5 count kernel's hash), or 64.  (No reference counterpart.) */
int nk_diag_hash_ms_w(int device, uint64_t n_keys, uint64_t pool, int width, int reps, float *ms);
/* Diagnostic: the best of `reps` device times (ms) of a kernel that recomputes
 * the key of every record the handle's last count kept (the one-level
 * partitioned count: k <= 32, pool <= 4.2 M -- larger pools count through the
 * wide two-level path, which keeps no such records -- one batch, no exact
 * table; otherwise NK_E_INVALID) from its position in the input -- the
 * tile from the segment descriptors, the k bases from the resident input --
 * and XOR-folds the keys into *checksum (may be NULL): what an exact-table pass
 * that reads positions instead of K1a-written keys would pay for its keys.
 * (The checksum covers the kept records: the excess of an overflowed region,
 * counted directly, is not among them.)  Synchronises the device.  The last
 * count's input must still be resident: when it was the caller's device
 * memory (nk_accumulate_device*), the caller keeps it allocated until this
 * returns -- the kernel reads those bases (the handle's own copies, from the
 * host-array and file entry points, are always resident).  (No reference
 * counterpart: measurement only.) */
int nk_diag_key_gather_ms(nk_counter *c, int reps, float *ms, uint64_t *checksum);

/* ---- associative memory (src/associative.rs) -------------
 * WillshawNetwork — :12-62.  Binary weights of pattern_size^2 bits on the
 * device (bit-packed rows).  store: every pair of set bits of the pattern gets
 * weight 1 (a pattern of another size: NK_E_INVALID "Pattern size mismatch");
 * recall: up to `steps` synchronous updates state' = (W state > 0), stopping
 * when the state repeats; out[i] = 255 or 0. */
typedef struct nk_willshaw nk_willshaw;
nk_willshaw *nk_willshaw_new(size_t pattern_size, int device);
void nk_willshaw_free(nk_willshaw *w);
int nk_willshaw_store(nk_willshaw *w, const uint8_t *pattern, size_t len);
int nk_willshaw_recall(nk_willshaw *w, const uint8_t *noisy, size_t len, size_t steps,
                       uint8_t *out);
uint64_t nk_willshaw_stored(const nk_willshaw *w);  /* stored_count */
/* KmerAssociativeMemory — :64-139.  pattern_size = 2^k for k <= 10, else 1024;
 * a k-mer's pattern sets bit (byte i % 32 of BLAKE3(kmer as 8 LE bytes)) %
 * pattern_size for i < pattern_size / 100, computed on the device.
 * nk_assoc_store_kmers = store_kmer over a batch (counts may be NULL: the
 * reference does not use them).  nk_assoc_find_similar = find_similar: the
 * query's pattern recalled over 10 steps, then every distinct stored k-mer
 * whose pattern is within max_distance bits (Hamming) of it, with similarity
 * 1 - d / pattern_size (f32), by similarity descending (equal similarities by
 * k-mer ascending: the reference's order there is HashMap iteration order).
 * Writes min(count, cap) results, returns count (or < 0). */
typedef struct nk_assoc nk_assoc;
nk_assoc *nk_assoc_new(size_t k, int device);
void nk_assoc_free(nk_assoc *a);
size_t nk_assoc_pattern_size(const nk_assoc *a);
int nk_assoc_store_kmers(nk_assoc *a, const uint64_t *kmers, const uint32_t *counts, size_t n);
long nk_assoc_find_similar(nk_assoc *a, uint64_t query, size_t max_distance, uint64_t *kmers,
                           float *sim, size_t cap);

const char *nk_last_error(void);
const char *nk_version(void);

#ifdef __cplusplus
}
#endif
#endif /* NEUROKMER_H */
