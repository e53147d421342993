"""Associative memory over the C ABI (include/neurokmer.h, nk_assoc.hip):
the reference's WillshawNetwork and KmerAssociativeMemory
(src/associative.rs:12-139), with the weights, BLAKE3 patterns, recall and the
similarity scan on the device.  No CPU fallback.

    net = WillshawNetwork(64)            # :20 new(pattern_size)
    net.store(pattern_bytes)             # :29 store
    net.recall(noisy_bytes, steps)       # :45 recall -> bytes of 255 / 0
    mem = KmerAssociativeMemory(k)       # :72 new(k)
    mem.store_kmer(kmer, count)          # :99 (or store_kmers for a batch)
    mem.find_similar(kmer, max_distance) # :113 -> [(kmer, similarity f32)]
"""
from __future__ import annotations

import ctypes as C
from typing import List, Tuple

import numpy as np

from . import _lib


class WillshawNetwork:
    def __init__(self, pattern_size: int, device: int = 0):
        self._L = _lib.load()
        self._h = self._L.nk_willshaw_new(pattern_size, device)
        if not self._h:
            raise _lib.NeuroKmerError(_lib.NK_E_NO_DEVICE, _lib.last_error())
        self.pattern_size = pattern_size

    def close(self):
        if self._h:
            self._L.nk_willshaw_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def store(self, pattern) -> None:
        p = np.ascontiguousarray(np.frombuffer(bytes(pattern), np.uint8))
        _lib.check(self._L.nk_willshaw_store(self._h, p.ctypes.data if p.size else None, p.size))

    def recall(self, noisy, steps: int) -> bytes:
        p = np.ascontiguousarray(np.frombuffer(bytes(noisy), np.uint8))
        out = np.zeros(max(p.size, 1), np.uint8)
        _lib.check(self._L.nk_willshaw_recall(self._h, p.ctypes.data if p.size else None, p.size,
                                              steps, out.ctypes.data))
        return out[:p.size].tobytes()

    @property
    def stored_count(self) -> int:
        return int(self._L.nk_willshaw_stored(self._h))


class KmerAssociativeMemory:
    def __init__(self, k: int, device: int = 0):
        self._L = _lib.load()
        self._h = self._L.nk_assoc_new(k, device)
        if not self._h:
            raise _lib.NeuroKmerError(_lib.NK_E_NO_DEVICE, _lib.last_error())
        self.pattern_size = int(self._L.nk_assoc_pattern_size(self._h))

    def close(self):
        if self._h:
            self._L.nk_assoc_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def store_kmer(self, kmer: int, count: int = 0) -> None:
        self.store_kmers([kmer], [count])

    def store_kmers(self, kmers, counts=None) -> None:
        k = np.ascontiguousarray(kmers, dtype=np.uint64)
        c = None if counts is None else np.ascontiguousarray(counts, dtype=np.uint32)
        _lib.check(self._L.nk_assoc_store_kmers(self._h, k.ctypes.data if k.size else None,
                                                c.ctypes.data if c is not None and c.size else None,
                                                k.size))

    def find_similar(self, query_kmer: int, max_distance: int) -> List[Tuple[int, float]]:
        n = int(_lib.check(self._L.nk_assoc_find_similar(self._h, query_kmer, max_distance,
                                                         None, None, 0)))
        km = np.zeros(max(n, 1), np.uint64)
        sim = np.zeros(max(n, 1), np.float32)
        m = int(_lib.check(self._L.nk_assoc_find_similar(self._h, query_kmer, max_distance,
                                                         km.ctypes.data, sim.ctypes.data, n)))
        return [(int(km[i]), float(sim[i])) for i in range(min(m, n))]
