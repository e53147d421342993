"""`SpikingKmerCounter` — Python mirror of the reference's public API, backed by
the MI355X C ABI (include/neurokmer.h).  Same names, argument meaning and
results as src/spiking_hash.rs; errors raise NeuroKmerError (the reference
panics or returns Err).

    c = SpikingKmerCounter(31, 1.0, 0.95, 2, 1.0, 2_000_000, True)
    c.process_parallel(seqs)              # src/spiking_hash.rs:84
    c.process_file_streaming(path)        # :277
    c.top_abundant_neurons(20)            # :661  -> [(idx, spikes, uniques)]
    c.energy.total_spikes(); c.energy_used()   # src/models.rs:166, :684
"""
from __future__ import annotations

import ctypes as C
from typing import Iterable, Optional, Sequence

import numpy as np

from . import _lib
from ._lib import NkOpts, NkTopRow, check


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data if a.size else 0


def records_to_arrays(seqs: Iterable[bytes]):
    """list of record byte strings -> (bases uint8, offsets uint64[n+1])."""
    seqs = [bytes(s) for s in seqs]
    offs = np.zeros(len(seqs) + 1, np.uint64)
    if seqs:
        np.cumsum(np.fromiter((len(s) for s in seqs), np.uint64, len(seqs)), out=offs[1:])
    bases = np.frombuffer(b"".join(seqs), np.uint8) if seqs else np.zeros(0, np.uint8)
    return bases, offs


class EnergyTracker:
    """src/models.rs:145-173 view (spike totals live in the native handle)."""

    def __init__(self, owner: "SpikingKmerCounter"):
        self._o = owner

    def total_spikes(self) -> int:
        return int(self._o._L.nk_total_spikes(self._o._h))

    def total_energy(self) -> float:
        return float(self._o._L.nk_energy_used(self._o._h))


class SpikingKmerCounter:
    def __init__(self, k: int, threshold: float, leak: float, refractory: int,
                 spike_cost: float, pool_size: int, use_canonical: bool, *,
                 device: int = 0, top_n: int = 20, stage_timing: bool = False,
                 kmer_width: int = 64, exact_counts: bool = False,
                 defer_hist: bool = False):
        """defer_hist: batches in flight on one count stream across handles --
        this handle's bucket histogram runs inside the next handle's count
        kernel (nk_opts.defer_hist); same results."""
        self._L = _lib.load()
        o = NkOpts()
        self._L.nk_opts_default(C.byref(o))
        o.device = device
        o.top_n = top_n
        o.stage_timing = 1 if stage_timing else 0
        if kmer_width not in (64, 128):
            raise ValueError("kmer_width must be 64 (the reference's u64 keys) or 128")
        o.kmer_width = _lib.NK_KMER_128 if kmer_width == 128 else _lib.NK_KMER_COMPAT
        o.exact_counts = 1 if exact_counts else 0
        o.defer_hist = 1 if defer_hist else 0
        self.kmer_width = kmer_width
        self.exact_counts = bool(exact_counts)
        self._h = None
        h = self._L.nk_new(k, threshold, leak, refractory, spike_cost, pool_size,
                           1 if use_canonical else 0, C.byref(o))
        if not h:
            raise _lib.NeuroKmerError(_lib.NK_E_NO_DEVICE, _lib.last_error())
        self._h = h
        self.k = k
        self.pool_size = pool_size
        self.use_canonical = bool(use_canonical)
        self.top_n = top_n
        self.energy = EnergyTracker(self)

    def close(self):
        if self._h:
            self._L.nk_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- processing --------------------------------------------------------
    def process_parallel(self, seqs: Sequence[bytes]) -> None:
        """src/spiking_hash.rs:84-201 (records in host memory)."""
        self.process_parallel_arrays(*records_to_arrays(seqs))

    def process_parallel_arrays(self, bases: np.ndarray, offsets: np.ndarray) -> None:
        bases = np.ascontiguousarray(bases, np.uint8)
        offsets = np.ascontiguousarray(offsets, np.uint64)
        check(self._L.nk_process_parallel(self._h, _ptr(bases), _ptr(offsets), offsets.size - 1))

    def process_parallel_device(self, d_bases: int, d_offsets: int, n_recs: int, n_bases: int,
                                stream: int = 0) -> None:
        """Input already in HBM (raw device pointers, e.g. torch tensor.data_ptr())."""
        check(self._L.nk_process_parallel_device(self._h, d_bases, d_offsets, n_recs, n_bases,
                                                 stream or None))

    def process_file_streaming(self, path: str) -> None:
        """src/spiking_hash.rs:277-486 (GPU FASTX ingest)."""
        check(self._L.nk_process_file_streaming(self._h, str(path).encode()))

    def process_file_parallel(self, path: str) -> None:
        """stream_sequences(path).collect() + process_parallel (src/main.rs:40-46)."""
        check(self._L.nk_process_file_parallel(self._h, str(path).encode()))

    # split phase (multi-GPU: allreduce currents between the two)
    def accumulate_device(self, d_bases: int, d_offsets: int, n_recs: int, n_bases: int,
                          stream: int = 0) -> None:
        check(self._L.nk_accumulate_device(self._h, d_bases, d_offsets, n_recs, n_bases,
                                           stream or None))

    def accumulate_device_from(self, d_bases: int, d_offsets: int, n_recs: int, n_bases: int,
                               first_pos: int, stream: int = 0) -> None:
        """accumulate_device counting only windows that start at >= first_pos."""
        check(self._L.nk_accumulate_device_from(self._h, d_bases, d_offsets, n_recs,
                                                n_bases, first_pos, stream or None))

    def finalize_slice(self, d_slice: int, slice_bits: int, lo: int, hi: int, d_seg: int,
                       seg_rows: int, streaming: bool = False, stream: int = 0) -> None:
        """Pool-sliced finish, step 1 (include/neurokmer.h nk_finalize_slice)."""
        check(self._L.nk_finalize_slice(self._h, 1 if streaming else 0, d_slice or None,
                                        slice_bits, lo, hi, d_seg, seg_rows, stream or None))

    def adopt_slices(self, d_all: int, world: int, stride: int, stream: int = 0) -> None:
        """Pool-sliced finish, step 2 (nk_adopt_slices)."""
        check(self._L.nk_adopt_slices(self._h, d_all, world, stride, stream or None))

    def finalize(self, streaming: bool = False, stream: int = 0) -> None:
        check(self._L.nk_finalize(self._h, 1 if streaming else 0, stream or None))

    def top_kmers_device(self):
        """-> (device pointer, count) of this shard's distinct top-N k-mer keys
        (kmer_width 128: count (lo, hi) u64 pairs)."""
        p = C.c_void_p()
        n = C.c_size_t()
        check(self._L.nk_top_kmers(self._h, C.byref(p), C.byref(n)))
        return (p.value or 0), n.value

    def merge_top_kmers(self, d_keys: int, n_keys: int, stream: int = 0) -> None:
        check(self._L.nk_merge_top_kmers(self._h, d_keys, n_keys, stream or None))

    # multi-GPU exact table (include/neurokmer.h: nk_exact_partition / _adopt)
    def exact_partition(self, world: int, stream: int = 0):
        """-> (send_counts per rank, device ptr of the u64 keys, device ptr of
        the u32 counts): this rank's table grouped by owner rank."""
        cnt = (C.c_uint64 * world)()
        kp, cp = C.c_void_p(), C.c_void_p()
        check(self._L.nk_exact_partition(self._h, world, cnt, C.byref(kp), C.byref(cp),
                                         stream or None))
        return [int(x) for x in cnt], (kp.value or 0), (cp.value or 0)

    def exact_adopt(self, d_keys: int, d_counts: int, n: int, stream: int = 0) -> None:
        check(self._L.nk_exact_adopt(self._h, d_keys or None, d_counts or None, n, stream or None))

    def device_kmer_per_neuron_ptr(self) -> int:
        return self._L.nk_device_kmer_per_neuron(self._h) or 0

    def top_kmers_padded(self, d_out: int, cap: int, stream: int = 0) -> None:
        """[n, keys...] (at most cap keys) of this shard into d_out, no host sync."""
        check(self._L.nk_top_kmers_padded(self._h, d_out, cap, stream or None))

    def merge_top_kmers_padded(self, d_buf: int, world: int, stride: int, cap: int,
                               stream: int = 0) -> bool:
        """Uniques from an all-gather of world padded segments; False: a segment
        was truncated (fall back to top_kmers_device + merge_top_kmers)."""
        ok = C.c_int(0)
        check(self._L.nk_merge_top_kmers_padded(self._h, d_buf, world, stride, cap,
                                                C.byref(ok), stream or None))
        return bool(ok.value)

    # --- multi-GPU step with one host synchronisation (dist.finalize_step) ---
    def wire32(self, d_wire: int, stream: int = 0) -> None:
        check(self._L.nk_wire32(self._h, d_wire, stream or None))

    def finalize_export(self, d_wire: int, d_seg: int, cap: int, streaming: bool = False,
                        stream: int = 0) -> None:
        check(self._L.nk_finalize_export(self._h, 1 if streaming else 0, d_wire or None, d_seg,
                                         cap, stream or None))

    def merge_export(self, d_buf: int, world: int, stride: int, cap: int, stream: int = 0) -> bool:
        """-> True when a redo is needed (the same answer on every rank)."""
        redo = C.c_int(0)
        check(self._L.nk_merge_export(self._h, d_buf, world, stride, cap, C.byref(redo),
                                      stream or None))
        return bool(redo.value)

    def finalize_redo(self, stream: int = 0) -> None:
        check(self._L.nk_finalize_redo(self._h, stream or None))

    def settle(self, stream: int = 0) -> None:
        """Write out the derived per-neuron state (nk_settle)."""
        check(self._L.nk_settle(self._h, stream))

    def device_currents_ptr(self) -> int:
        return self._L.nk_device_currents(self._h) or 0

    def reset(self, stream: int = 0, blocking: bool = True) -> None:
        """Fresh neuron pool (the state new() leaves).  blocking=False enqueues
        the reset on `stream` and returns at once."""
        if blocking:
            check(self._L.nk_reset(self._h))
        else:
            check(self._L.nk_reset_async(self._h, stream or None))

    # ---- results -----------------------------------------------------------
    def top_abundant_neurons(self, n: int):
        """src/spiking_hash.rs:661-673 -> [(neuron_idx, spikes, unique_kmers)]"""
        rows = (NkTopRow * max(n, 1))()
        m = check(self._L.nk_top_abundant_neurons(self._h, n, rows))
        return [(int(rows[i].idx), int(rows[i].spikes), int(rows[i].uniques)) for i in range(m)]

    def get_count(self, kmer: int) -> Optional[int]:
        """src/spiking_hash.rs:675-682.  The table is built with every process call
        (exact_counts=True) or on demand from the last input the handle holds."""
        out = C.c_uint32()
        present = C.c_int()
        check(self._L.nk_get_count(self._h, kmer, C.byref(out), C.byref(present)))
        return int(out.value) if present.value else None

    def process_sequence(self, seq: bytes) -> None:
        """src/spiking_hash.rs:203-273 (u64 keys; the previous call's table first)."""
        buf = np.frombuffer(bytes(seq), dtype=np.uint8)
        check(self._L.nk_process_sequence(self._h, buf.ctypes.data if buf.size else None,
                                          buf.size))

    def simulate_spikes_auto(self) -> None:
        """src/spiking_hash.rs:697-714 (AVX2 branch, :544-659): `steps` LIF
        updates of every neuron from the held currents; spikes and energy add
        to the totals."""
        check(self._L.nk_simulate_spikes_auto(self._h))

    def get_counts(self, kmers) -> tuple:
        """Batched get_count: -> (counts u32[n], present bool[n])."""
        q = np.ascontiguousarray(kmers, dtype=np.uint64)
        out = np.zeros(max(q.size, 1), np.uint32)
        pres = np.zeros(max(q.size, 1), np.uint8)
        check(self._L.nk_get_counts(self._h, q.ctypes.data if q.size else None, q.size,
                                    out.ctypes.data, pres.ctypes.data))
        return out[:q.size], pres[:q.size].astype(bool)

    def get_counts128(self, kmers) -> tuple:
        """kmer_width=128 handles: get_count of u128 keys (python ints) -> (counts, present)."""
        ks = [int(x) for x in kmers]
        q = np.zeros(max(2 * len(ks), 2), np.uint64)
        for i, x in enumerate(ks):
            q[2 * i] = x & 0xFFFFFFFFFFFFFFFF
            q[2 * i + 1] = x >> 64
        out = np.zeros(max(len(ks), 1), np.uint32)
        pres = np.zeros(max(len(ks), 1), np.uint8)
        check(self._L.nk_get_counts128(self._h, q.ctypes.data if ks else None, len(ks),
                                       out.ctypes.data, pres.ctypes.data))
        return out[:len(ks)], pres[:len(ks)].astype(bool)

    def distinct_kmers(self) -> int:
        """counts.len()."""
        n = int(self._L.nk_distinct_kmers(self._h))
        if n < 0:
            check(n)
        return n

    def kmer_per_neuron(self) -> np.ndarray:
        """The full kmer_per_neuron map as a dense u32 array."""
        return self._copy("nk_copy_kmer_per_neuron", np.uint32)

    def energy_used(self) -> float:
        return float(self._L.nk_energy_used(self._h))

    def set_steps(self, steps: int) -> None:
        self._L.nk_set_steps(self._h, steps)

    def get_steps(self) -> int:
        return int(self._L.nk_get_steps(self._h))

    def _copy(self, fn, dtype):
        out = np.zeros(self.pool_size, dtype)
        check(getattr(self._L, fn)(self._h, _ptr(out), out.size))
        return out

    def currents(self) -> np.ndarray:
        return self._copy("nk_copy_currents", np.uint64)

    def spike_counts(self) -> np.ndarray:
        return self._copy("nk_copy_spike_counts", np.uint64)

    def voltages(self) -> np.ndarray:
        return self._copy("nk_copy_voltages", np.float32)

    def refractory(self) -> np.ndarray:
        return self._copy("nk_copy_refractory", np.uint32)

    def last_timings(self) -> dict:
        names = (C.c_char_p * 8)()
        ms = (C.c_float * 8)()
        n = self._L.nk_last_timings(self._h, names, ms, 8)
        return {names[i].decode(): float(ms[i]) for i in range(n)}

    def set_stage_timing(self, level: int) -> None:
        """0: events around the count kernel (default); 1: every stage; 2: only
        at both ends of a call (no event between kernels, no K1 time); 3: none."""
        _lib.check(self._L.nk_set_stage_timing(self._h, level))

    def count_history(self, n: int) -> list:
        """K1 (count kernel) device time in ms of each of the last min(n, 256)
        accumulate/process calls, oldest first (hipEvents around the launch)."""
        buf = (C.c_float * max(n, 1))()
        m = self._L.nk_count_history(self._h, buf, n)
        return [float(buf[i]) for i in range(m)]

    def diag_key_gather(self, reps: int = 5) -> tuple:
        """(best ms, XOR of the keys) of recomputing the key of every record
        the last count kept from its input position (nk_diag_key_gather_ms):
        the key cost of an exact table built from positions, measured."""
        ms, cs = C.c_float(0.0), C.c_uint64(0)
        _lib.check(self._L.nk_diag_key_gather_ms(self._h, reps, C.byref(ms), C.byref(cs)))
        return float(ms.value), int(cs.value)

    def count_spans(self, n: int) -> list:
        """K1a (partitioned count kernel) duration in ms of each of the last
        min(n, 256) calls that ran it, oldest first, from in-kernel
        s_memrealtime stamps (no event in the stream; valid at stage_timing 2)."""
        buf = (C.c_float * max(n, 1))()
        m = _lib.check(self._L.nk_count_spans(self._h, buf, n))
        return [float(buf[i]) for i in range(m)]

    def count_stamps(self, n: int) -> list:
        """[(start, end)] s_memrealtime ticks (10 ns, one device clock) of the
        same K1a launches as count_spans, oldest first."""
        buf = (C.c_ulonglong * max(2 * n, 2))()
        m = _lib.check(self._L.nk_count_stamps(self._h, buf, n))
        return [(int(buf[2 * i]), int(buf[2 * i + 1])) for i in range(m)]


def diag_hash_ms(n_keys: int, pool: int, device: int = 0, reps: int = 5, width: int = 64) -> float:
    """Best device time (ms) of SipHash-1-3 + exact % pool over n_keys keys
    generated in registers (width 128: 16-byte keys): the count kernel's hash
    floor (nk_diag_hash_ms_w)."""
    ms = C.c_float(0.0)
    _lib.check(_lib.load().nk_diag_hash_ms_w(device, n_keys, pool, width, reps, C.byref(ms)))
    return float(ms.value)
