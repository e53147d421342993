"""ctypes binding of the C restatement (oracle/nk_oracle.c) -- TEST INFRASTRUCTURE ONLY.

Importable only from tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg.  The product (neurokmer_amd) never loads this library.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "libnk_oracle.so")
_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = C.CDLL(_LIB_PATH)
        u8p, u64p, f32p, u32p = (C.POINTER(C.c_uint8), C.POINTER(C.c_uint64),
                                 C.POINTER(C.c_float), C.POINTER(C.c_uint32))
        L.nko_siphash.restype = C.c_uint64
        L.nko_siphash.argtypes = [C.c_int, C.c_int, C.c_uint64, C.c_uint64, u8p, C.c_size_t]
        L.nko_sip13_u64.restype = C.c_uint64
        L.nko_sip13_u64.argtypes = [C.c_uint64]
        L.nko_map_kmer.restype = C.c_uint64
        L.nko_map_kmer.argtypes = [C.c_uint64, C.c_uint64]
        L.nko_pack_kmer.restype = C.c_uint64
        L.nko_pack_kmer.argtypes = [u8p, C.c_size_t]
        L.nko_kmer_keys.restype = C.c_size_t
        L.nko_kmer_keys.argtypes = [u8p, C.c_size_t, C.c_size_t, C.c_int, u64p]
        L.nko_lif.restype = None
        L.nko_lif.argtypes = [C.c_uint64, C.c_uint64, C.c_float, C.c_float, C.c_uint32, C.c_int,
                              f32p, u32p, u64p]
        L.nko_new.restype = C.c_void_p
        L.nko_new.argtypes = [C.c_size_t, C.c_float, C.c_float, C.c_uint32, C.c_double,
                              C.c_size_t, C.c_int]
        L.nko_free.argtypes = [C.c_void_p]
        for fn in ("nko_process_parallel", "nko_process_streaming"):
            f = getattr(L, fn)
            f.restype = C.c_int
            f.argtypes = [C.c_void_p, u8p, u64p, C.c_size_t, C.c_int]
        L.nko_process_sequence.restype = C.c_int
        L.nko_process_sequence.argtypes = [C.c_void_p, u8p, C.c_size_t]
        L.nko_lean_currents_lif.restype = C.c_int
        L.nko_lean_currents_lif.argtypes = [u8p, u64p, C.c_size_t, C.c_size_t, C.c_int, C.c_uint64,
                                            C.c_uint64, C.c_float, C.c_float, C.c_uint32, C.c_int,
                                            u64p, u64p, u64p]
        L.nko_simulate_spikes_auto.restype = None
        L.nko_simulate_spikes_auto.argtypes = [C.c_void_p]
        for fn, rt in (("nko_currents", u64p), ("nko_voltages", f32p), ("nko_refractory", u32p),
                       ("nko_spike_counts", u64p), ("nko_kmer_per_neuron", u32p)):
            f = getattr(L, fn)
            f.restype = rt
            f.argtypes = [C.c_void_p]
        for fn, rt in (("nko_total_spikes", C.c_uint64), ("nko_total_energy_fixed", C.c_uint64),
                       ("nko_energy_used", C.c_double), ("nko_distinct_kmers", C.c_size_t),
                       ("nko_get_steps", C.c_uint64)):
            f = getattr(L, fn)
            f.restype = rt
            f.argtypes = [C.c_void_p]
        L.nko_set_steps.argtypes = [C.c_void_p, C.c_uint64]
        L.nko_top_abundant.restype = C.c_size_t
        L.nko_top_abundant.argtypes = [C.c_void_p, C.c_size_t, u64p, u64p, u32p]
        L.nko_get_count.restype = C.c_int
        L.nko_get_count.argtypes = [C.c_void_p, C.c_uint64, u32p]
        # --kmer-width=128
        L.nko_sip13_u128.restype = C.c_uint64
        L.nko_sip13_u128.argtypes = [C.c_uint64, C.c_uint64]
        L.nko_kmer_keys128.restype = C.c_size_t
        L.nko_kmer_keys128.argtypes = [u8p, C.c_size_t, C.c_size_t, C.c_int, u64p]
        L.nko_new_w.restype = C.c_void_p
        L.nko_new_w.argtypes = [C.c_size_t, C.c_float, C.c_float, C.c_uint32, C.c_double,
                                C.c_size_t, C.c_int, C.c_int]
        L.nko_get_count128.restype = C.c_int
        L.nko_get_count128.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64, u32p]
        _lib = L
    return _lib


def _ptr(a: np.ndarray, ct):
    return a.ctypes.data_as(C.POINTER(ct))


def siphash(c, d, k0, k1, msg: bytes) -> int:
    buf = np.frombuffer(msg, dtype=np.uint8) if msg else np.zeros(1, np.uint8)
    return int(lib().nko_siphash(c, d, k0, k1, _ptr(buf, C.c_uint8), len(msg)))


def sip13_u64(m: int) -> int:
    return int(lib().nko_sip13_u64(m))


def kmer_keys(seq: bytes, k: int, canonical: bool) -> np.ndarray:
    n = max(0, len(seq) - k + 1)
    out = np.zeros(max(n, 1), np.uint64)
    buf = np.frombuffer(seq, dtype=np.uint8) if seq else np.zeros(1, np.uint8)
    m = lib().nko_kmer_keys(_ptr(buf, C.c_uint8), len(seq), k, int(canonical),
                            _ptr(out, C.c_uint64))
    return out[:m]


def sip13_u128(key: int) -> int:
    return int(lib().nko_sip13_u128(key & (2**64 - 1), key >> 64))


def kmer_keys128(seq: bytes, k: int, canonical: bool) -> list:
    """--kmer-width=128 keys of one record as Python ints."""
    n = max(0, len(seq) - k + 1)
    out = np.zeros(2 * max(n, 1), np.uint64)
    buf = np.frombuffer(seq, dtype=np.uint8) if seq else np.zeros(1, np.uint8)
    m = lib().nko_kmer_keys128(_ptr(buf, C.c_uint8), len(seq), k, int(canonical),
                               _ptr(out, C.c_uint64))
    return [int(out[2 * i]) | (int(out[2 * i + 1]) << 64) for i in range(m)]


def lif(count, steps, thr, leak, refr, skip_zero, v=0.0, r=0, spikes=0):
    cv, cr, cs = C.c_float(v), C.c_uint32(r), C.c_uint64(spikes)
    lib().nko_lif(count, steps, thr, leak, refr, int(skip_zero), C.byref(cv), C.byref(cr),
                  C.byref(cs))
    return cv.value, cr.value, cs.value


def records_to_arrays(seqs):
    """list[bytes] -> (bases u8, offsets u64[n+1])."""
    offs = np.zeros(len(seqs) + 1, np.uint64)
    np.cumsum([len(s) for s in seqs], out=offs[1:]) if seqs else None
    bases = np.frombuffer(b"".join(seqs), dtype=np.uint8) if seqs else np.zeros(0, np.uint8)
    return bases, offs


class OracleCounter:
    """SpikingKmerCounter restated in C (see oracle/nk_oracle.h)."""

    def __init__(self, k, threshold, leak, refractory, spike_cost, pool_size, use_canonical,
                 width=64):
        self._L = lib()
        self.pool = pool_size
        self.width = width
        self._h = self._L.nko_new_w(k, threshold, leak, refractory, spike_cost, pool_size,
                                    int(use_canonical), width)
        if not self._h:
            raise ValueError("bad width/k")

    def __del__(self):
        if getattr(self, "_h", None):
            self._L.nko_free(self._h)
            self._h = None

    def _run(self, fn, bases, offsets, n_threads):
        bases = np.ascontiguousarray(bases, np.uint8)
        offsets = np.ascontiguousarray(offsets, np.uint64)
        b = bases if bases.size else np.zeros(1, np.uint8)
        rc = fn(self._h, _ptr(b, C.c_uint8), _ptr(offsets, C.c_uint64), offsets.size - 1,
                n_threads)
        if rc != 0:
            raise RuntimeError("oracle rejected the input (k == 0 or pool == 0)")

    def process_parallel_arrays(self, bases, offsets, n_threads=1):
        self._run(self._L.nko_process_parallel, bases, offsets, n_threads)

    def process_streaming_arrays(self, bases, offsets, n_threads=1):
        self._run(self._L.nko_process_streaming, bases, offsets, n_threads)

    def process_parallel(self, seqs, n_threads=1):
        self.process_parallel_arrays(*records_to_arrays(seqs), n_threads)

    def process_streaming(self, seqs, n_threads=1):
        self.process_streaming_arrays(*records_to_arrays(seqs), n_threads)

    def process_sequence(self, seq: bytes):
        buf = np.frombuffer(seq, dtype=np.uint8) if seq else np.zeros(1, np.uint8)
        if self._L.nko_process_sequence(self._h, _ptr(buf, C.c_uint8), len(seq)) != 0:
            raise RuntimeError("oracle rejected the input")

    def simulate_spikes_auto(self):
        self._L.nko_simulate_spikes_auto(self._h)

    def _arr(self, fn, dt):
        p = getattr(self._L, fn)(self._h)
        return np.ctypeslib.as_array(p, shape=(self.pool,)).astype(dt, copy=True) if self.pool \
            else np.zeros(0, dt)

    def currents(self):
        return self._arr("nko_currents", np.uint64)

    def voltages(self):
        return self._arr("nko_voltages", np.float32)

    def refractory(self):
        return self._arr("nko_refractory", np.uint32)

    def spike_counts(self):
        return self._arr("nko_spike_counts", np.uint64)

    def kmer_per_neuron(self):
        return self._arr("nko_kmer_per_neuron", np.uint32)

    @property
    def total_spikes(self):
        return int(self._L.nko_total_spikes(self._h))

    @property
    def total_energy_fixed(self):
        return int(self._L.nko_total_energy_fixed(self._h))

    def energy_used(self):
        return float(self._L.nko_energy_used(self._h))

    def distinct_kmers(self):
        return int(self._L.nko_distinct_kmers(self._h))

    def set_steps(self, s):
        self._L.nko_set_steps(self._h, s)

    def get_steps(self):
        return int(self._L.nko_get_steps(self._h))

    def top_abundant_neurons(self, n):
        idx = np.zeros(max(n, 1), np.uint64)
        sp = np.zeros(max(n, 1), np.uint64)
        un = np.zeros(max(n, 1), np.uint32)
        m = self._L.nko_top_abundant(self._h, n, _ptr(idx, C.c_uint64), _ptr(sp, C.c_uint64),
                                     _ptr(un, C.c_uint32))
        return [(int(idx[i]), int(sp[i]), int(un[i])) for i in range(m)]

    def get_count(self, kmer):
        out = C.c_uint32(0)
        if self.width == 128:
            ok = self._L.nko_get_count128(self._h, kmer & (2**64 - 1), kmer >> 64, C.byref(out))
        else:
            ok = self._L.nko_get_count(self._h, kmer, C.byref(out))
        return int(out.value) if ok else None


# ---- associative memory (oracle/nk_assoc_oracle.c; src/associative.rs) -------
def _assoc_sigs(L):
    if getattr(L, "_assoc_ready", False):
        return L
    vp, sz, u64 = C.c_void_p, C.c_size_t, C.c_uint64
    for name, rt, args in (
            ("nko_blake3", C.c_int, [vp, sz, vp]),
            ("nko_willshaw_new", vp, [sz]), ("nko_willshaw_free", None, [vp]),
            ("nko_willshaw_store", C.c_int, [vp, vp, sz]),
            ("nko_willshaw_recall", C.c_int, [vp, vp, sz, sz, vp]),
            ("nko_willshaw_stored", u64, [vp]),
            ("nko_assoc_new", vp, [sz]), ("nko_assoc_free", None, [vp]),
            ("nko_assoc_pattern_size", sz, [sz]),
            ("nko_assoc_kmer_pattern", None, [sz, u64, vp]),
            ("nko_assoc_store", C.c_int, [vp, u64, C.c_uint32]),
            ("nko_assoc_find_similar", sz, [vp, u64, sz, vp, vp, sz])):
        f = getattr(L, name)
        f.restype, f.argtypes = rt, args
    L._assoc_ready = True
    return L


def blake3(data: bytes) -> bytes:
    """BLAKE3 digest of <= 1024 bytes (the oracle's one-chunk restatement)."""
    L = _assoc_sigs(lib())
    buf = np.frombuffer(bytes(data), np.uint8) if data else np.zeros(1, np.uint8)
    out = np.zeros(32, np.uint8)
    if L.nko_blake3(buf.ctypes.data, len(data), out.ctypes.data) != 0:
        raise ValueError("input longer than one chunk")
    return out.tobytes()


class OracleWillshaw:
    def __init__(self, n):
        self._L = _assoc_sigs(lib())
        self.n = n
        self._h = self._L.nko_willshaw_new(n)

    def __del__(self):
        if getattr(self, "_h", None):
            self._L.nko_willshaw_free(self._h)
            self._h = None

    def store(self, pattern):
        p = np.frombuffer(bytes(pattern), np.uint8) if len(pattern) else np.zeros(1, np.uint8)
        if self._L.nko_willshaw_store(self._h, p.ctypes.data, len(pattern)) != 0:
            raise ValueError("Pattern size mismatch")

    def recall(self, noisy, steps):
        p = np.frombuffer(bytes(noisy), np.uint8) if len(noisy) else np.zeros(1, np.uint8)
        out = np.zeros(max(len(noisy), 1), np.uint8)
        if self._L.nko_willshaw_recall(self._h, p.ctypes.data, len(noisy), steps,
                                       out.ctypes.data) != 0:
            raise ValueError("Noisy pattern size mismatch")
        return out[:len(noisy)].tobytes()

    @property
    def stored_count(self):
        return int(self._L.nko_willshaw_stored(self._h))


class OracleAssoc:
    def __init__(self, k):
        self._L = _assoc_sigs(lib())
        self._h = self._L.nko_assoc_new(k)
        self.pattern_size = int(self._L.nko_assoc_pattern_size(k))

    def __del__(self):
        if getattr(self, "_h", None):
            self._L.nko_assoc_free(self._h)
            self._h = None

    def kmer_pattern(self, kmer):
        out = np.zeros(self.pattern_size, np.uint8)
        self._L.nko_assoc_kmer_pattern(self.pattern_size, kmer, out.ctypes.data)
        return out.tobytes()

    def store_kmer(self, kmer, count=0):
        self._L.nko_assoc_store(self._h, kmer, count)

    def find_similar(self, query, max_distance):
        n = self._L.nko_assoc_find_similar(self._h, query, max_distance, None, None, 0)
        km = np.zeros(max(n, 1), np.uint64)
        sim = np.zeros(max(n, 1), np.float32)
        self._L.nko_assoc_find_similar(self._h, query, max_distance, km.ctypes.data,
                                       sim.ctypes.data, n)
        return [(int(km[i]), float(sim[i])) for i in range(n)]


def lean_currents_lif(bases, offsets, k, pool, canonical=True, steps=1000, n_threads=1,
                      threshold=1.0, leak=0.95, refractory=2):
    """The lean CPU baseline (nko_lean_currents_lif; not the reference's
    structure): (currents, spike counts, total spikes) of one in-memory call
    from the reset state (the LIF memoised by count)."""
    bases = np.ascontiguousarray(bases, np.uint8)
    offsets = np.ascontiguousarray(offsets, np.uint64)
    cur = np.zeros(pool, np.uint64)
    sp = np.zeros(pool, np.uint64)
    tot = np.zeros(1, np.uint64)
    rc = lib().nko_lean_currents_lif(_ptr(bases, C.c_uint8), _ptr(offsets, C.c_uint64),
                                     offsets.size - 1, k, int(canonical), pool, steps,
                                     float(threshold), float(leak), int(refractory), n_threads,
                                     _ptr(cur, C.c_uint64), _ptr(sp, C.c_uint64), _ptr(tot, C.c_uint64))
    if rc:
        raise ValueError("nko_lean_currents_lif failed (k <= 32, pool >= 1)")
    return cur, sp, int(tot[0])
