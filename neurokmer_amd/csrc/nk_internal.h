// nk_internal.h — what other translation units of libneurokmer.so read of a
// counter handle (internal; not ABI).  Implemented in nk_counter.cpp.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "neurokmer.h"

// nk_last_error() text for this thread; returns code
int nk_fail_msg(int code, const char *msg);

namespace nk {
// min(opts.top_n, pool_size): the rows every finish selects
uint64_t counter_rows(const nk_counter *c);
// u64 words per k-mer key (2 for NK_KMER_128)
int counter_key_words(const nk_counter *c);
// the uniques column comes from an adopted global kmer_per_neuron (multi-GPU
// exact table): the finish is a plain nk_finalize after the currents' all-reduce
bool counter_kpn_global(const nk_counter *c);
// the u64 currents complete on stream s (lazily-zero currents materialised,
// pending K1b partials folded, no host wait); null on error
// the world size of the merge after the next nk_finalize_export (its set is
// then emptied by the export's header kernel)
void counter_merge_hint(nk_counter *c, uint32_t world);
uint64_t *counter_currents_on(nk_counter *c, hipStream_t s);
// after nk_slice_export + nk_merge_export asked for a redo: the blocking,
// exact selection of this rank's slice [lo, hi) into d_seg (its LIF not rerun)
int slice_reselect(nk_counter *c, size_t lo, size_t hi, uint64_t *d_seg, size_t seg_rows,
                   hipStream_t s);
// a per-process id of the handle, never reused after nk_free
uint64_t counter_uid(const nk_counter *c);
// the loopback transport (nk_loop.hip)
int loop_join(nk_loop_group *g, int rank, int device);  // (a rank joins once)
void loop_leave(nk_loop_group *g, int rank);            // (nk_comm_free)
// a rank that failed between collectives releases the others (they fail too)
void loop_break(nk_loop_group *g);
int loop_world(const nk_loop_group *g);
// kind 0 all-reduce (sum, n elements), 1 all-gather (n per rank), 2
// reduce-scatter (sum, n per rank); elem 4 or 8 bytes; blocks until done
int loop_collective(nk_loop_group *g, int rank, int kind, const void *send, void *recv, size_t n,
                    int elem, hipStream_t s);
}  // namespace nk
