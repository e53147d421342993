/*
 * nk_oracle.h — CPU restatement of NeuroKmer's k-mer -> spike hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (neurokmer_amd/, include/,
 * the C ABI, the CLI) may link, load or call this code.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg use it, and only as
 * the checker / the timed CPU baseline, never as the thing measured.
 *
 * It restates, line by line, the reference Rust crate (MrObadiahEJ/NeuroKmer):
 *   src/models.rs:9-51      LifNeuron::update
 *   src/models.rs:145-173   EnergyTracker
 *   src/models.rs:175-299   RollingKmerHash (release-mode u64 semantics, k>32 too)
 *   src/utils.rs:26-39      pack_kmer
 *   src/spiking_hash.rs:78-82     map_kmer_to_neuron (SipHash-1-3, key 0, % pool)
 *   src/spiking_hash.rs:84-201    process_parallel
 *   src/spiking_hash.rs:277-486   process_file_streaming (+ :544-659 AVX2 LIF)
 *   src/spiking_hash.rs:661-673   top_abundant_neurons
 *   src/spiking_hash.rs:675-682   get_count
 *
 * Parity pinning: the reference is Rust and no Rust toolchain exists in this
 * image, and the reference ships no fixtures or asserting tests.  The SipHash
 * core is pinned against published vectors (SipHash paper, key 00..0f) and
 * against CPython 3.10's hash(bytes) (SipHash-2-4, key 0 under
 * PYTHONHASHSEED=0); everything else is a restatement cross-checked against an
 * independent pure-Python restatement (oracle/nk_oracle.py).  See DESIGN.md §3.
 */
#ifndef NK_ORACLE_H
#define NK_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- primitives ---------------------------------------------------------- */
/* Generic SipHash-c-d over a byte string (siphasher 1.0.2 semantics). */
uint64_t nko_siphash(int c_rounds, int d_rounds, uint64_t k0, uint64_t k1,
                     const uint8_t *msg, size_t len);
/* SipHasher13::new_with_keys(0,0); u64::hash -> write_u64 (8 LE bytes); finish(). */
uint64_t nko_sip13_u64(uint64_t m);
/* --kmer-width=128 (the build's own mode, see nk_oracle.c):
 * SipHash-1-3 (key 0) over the 16 LE bytes of a u128 (lo word first). */
uint64_t nko_sip13_u128(uint64_t lo, uint64_t hi);
/* 128-bit keys of one record, as (lo, hi) pairs; returns the key count. */
size_t nko_kmer_keys128(const uint8_t *seq, size_t len, size_t k, int canonical,
                        uint64_t *out);
/* map_kmer_to_neuron: src/spiking_hash.rs:78-82 */
uint64_t nko_map_kmer(uint64_t kmer, uint64_t pool);
/* pack_kmer: src/utils.rs:26-39 */
uint64_t nko_pack_kmer(const uint8_t *w, size_t k);
/* The k-mer keys the reference derives from one record, in order
 * (src/spiking_hash.rs:102-138).  Returns the count written (len-k+1 or 0). */
size_t nko_kmer_keys(const uint8_t *seq, size_t len, size_t k, int canonical,
                     uint64_t *out);
/* One neuron, `steps` calls of LifNeuron::update with c = (count/steps) as f32.
 * skip_zero = 1 reproduces process_parallel's `if total_current == 0 continue`. */
void nko_lif(uint64_t count, uint64_t steps, float thr, float leak, uint32_t refr,
             int skip_zero, float *v, uint32_t *r, uint64_t *spikes);

/* ---- counter ------------------------------------------------------------- */
typedef struct nko_counter nko_counter;

nko_counter *nko_new(size_t k, float threshold, float leak, uint32_t refractory,
                     double spike_cost, size_t pool_size, int use_canonical);
/* width 64 (= nko_new) or 128 (k <= 64); NULL on a bad width/k */
nko_counter *nko_new_w(size_t k, float threshold, float leak, uint32_t refractory,
                       double spike_cost, size_t pool_size, int use_canonical, int width);
void nko_free(nko_counter *c);
/* records = bases[offsets[i] .. offsets[i+1]), i < n_recs.  n_threads >= 1:
 * records are distributed over threads like rayon's par_iter (work unit = one
 * record). Returns 0, or -1 on error (pool 0 with k-mers present). */
int nko_process_parallel(nko_counter *c, const uint8_t *bases,
                         const uint64_t *offsets, size_t n_recs, int n_threads);
int nko_process_streaming(nko_counter *c, const uint8_t *bases,
                          const uint64_t *offsets, size_t n_recs, int n_threads);
/* simulate_spikes_auto (src/spiking_hash.rs:697-714 -> simulate_spikes_simd,
 * :544-659): the streaming LIF rule over the held currents */
void nko_simulate_spikes_auto(nko_counter *c);

/* A lean CPU baseline, NOT the reference's structure ("an
 * honest stronger baseline, clearly labelled not-the-reference"): the
 * currents of one in-memory call without the exact k-mer map, over n_threads
 * chunks of the windows (each record's k-mers split by position; k <= 32, where
 * the canonical key is a function of its window alone, models.rs:254-286),
 * per-thread u64 currents summed, then the 1000-step LIF of every neuron from
 * the fresh state in parallel over neurons (nko_lif: the reference's update
 * loop, bit-identical, with threshold thr, leak and refractory period refr;
 * spikes memoised by count, which the fresh state makes exact).  Writes
 * currents[pool], spikes[pool], *total_spikes.  A thread that cannot be
 * created runs its share on the calling thread. */
int nko_lean_currents_lif(const uint8_t *bases, const uint64_t *offsets, size_t n_recs, size_t k,
                          int canonical, uint64_t pool, uint64_t steps, float thr, float leak,
                          uint32_t refr, int n_threads,
                          uint64_t *currents, uint64_t *spikes, uint64_t *total_spikes);
/* process_sequence (src/spiking_hash.rs:203-273): per-record single-step form */
int nko_process_sequence(nko_counter *c, const uint8_t *seq, size_t len);

const uint64_t *nko_currents(const nko_counter *c);
const float *nko_voltages(const nko_counter *c);
const uint32_t *nko_refractory(const nko_counter *c);
const uint64_t *nko_spike_counts(const nko_counter *c);
const uint32_t *nko_kmer_per_neuron(const nko_counter *c);
uint64_t nko_total_spikes(const nko_counter *c);
uint64_t nko_total_energy_fixed(const nko_counter *c);
double nko_energy_used(const nko_counter *c);
size_t nko_distinct_kmers(const nko_counter *c);
void nko_set_steps(nko_counter *c, uint64_t steps);
uint64_t nko_get_steps(const nko_counter *c);
size_t nko_top_abundant(const nko_counter *c, size_t n, uint64_t *idx,
                        uint64_t *spikes, uint32_t *uniques);
/* 1 and *out set if present, 0 if absent */
int nko_get_count(const nko_counter *c, uint64_t kmer, uint32_t *out);
int nko_get_count128(const nko_counter *c, uint64_t lo, uint64_t hi, uint32_t *out);

#ifdef __cplusplus
}
#endif
#endif
