"""Loader for the in-tree HIP library (neurokmer_amd/lib/libneurokmer.so).

There is no CPU fallback: if the library is missing, or no gfx950 device is
present, every entry point raises.  The library is loaded from the package
directory (never from site-packages) so a GPU run visibly uses the in-tree
native code.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libneurokmer.so")
# A/B experiments only (tools/ab_build.sh): another build of the same library
if os.environ.get("NK_AB_LIB"):
    LIB_PATH = os.path.abspath(os.environ["NK_AB_LIB"])
CLI_PATH = os.path.join(_HERE, "bin", "neurokmer")

NK_OK = 0
NK_E_INVALID = -1
NK_E_NO_DEVICE = -2
NK_E_OOM = -3
NK_E_IO = -4
NK_E_PARSE = -5
NK_E_UNSUPPORTED = -6
NK_E_DEVICE = -7
NK_KMER_COMPAT = 0
NK_KMER_128 = 1

# every symbol include/neurokmer.h declares
EXPORTS = (
    "nk_opts_default", "nk_new", "nk_free", "nk_process_parallel", "nk_process_parallel_device",
    "nk_process_file_streaming", "nk_process_file_parallel", "nk_accumulate_device", "nk_finalize", "nk_top_kmers",
    "nk_merge_top_kmers", "nk_top_abundant_neurons", "nk_get_count", "nk_get_counts",
    "nk_get_counts128",
    "nk_distinct_kmers", "nk_copy_kmer_per_neuron", "nk_process_sequence", "nk_total_spikes",
    "nk_energy_used", "nk_set_steps", "nk_get_steps", "nk_pool_size", "nk_k",
    "nk_use_canonical", "nk_copy_currents", "nk_copy_spike_counts", "nk_copy_voltages",
    "nk_copy_refractory", "nk_device_currents", "nk_reset", "nk_reset_async", "nk_last_timings",
    "nk_count_history", "nk_wire32", "nk_finalize_export", "nk_merge_export", "nk_finalize_redo",
    "nk_top_kmers_padded", "nk_merge_top_kmers_padded",
    "nk_finalize_slice", "nk_adopt_slices", "nk_slice_export", "nk_adopt_export", "nk_accumulate_device_from",
    "nk_willshaw_new", "nk_willshaw_free", "nk_willshaw_store", "nk_willshaw_recall",
    "nk_willshaw_stored", "nk_assoc_new", "nk_assoc_free", "nk_assoc_pattern_size",
    "nk_assoc_store_kmers", "nk_assoc_find_similar",
    "nk_exact_owner", "nk_exact_partition", "nk_exact_adopt", "nk_device_kmer_per_neuron",
    "nk_set_stage_timing", "nk_diag_hash_ms", "nk_diag_hash_ms_w", "nk_diag_key_gather_ms", "nk_count_spans", "nk_count_stamps", "nk_simulate_spikes_auto",
    "nk_comm_unique_id", "nk_comm_new", "nk_comm_free", "nk_finalize_dist", "nk_finalize_sliced_dist",
    "nk_settle", "nk_comm_forget", "nk_loop_group_new", "nk_loop_group_free", "nk_comm_new_loopback",
    "nk_last_error",
    "nk_version",
)


class NkOpts(C.Structure):
    _fields_ = [("device", C.c_int32), ("kmer_width", C.c_int32), ("top_n", C.c_uint32),
                ("stage_timing", C.c_uint32), ("exact_counts", C.c_uint32),
                ("defer_hist", C.c_uint32), ("reserved", C.c_uint32 * 10)]


class NkTopRow(C.Structure):
    _fields_ = [("idx", C.c_uint64), ("spikes", C.c_uint64), ("uniques", C.c_uint32),
                ("_pad", C.c_uint32)]


class NeuroKmerError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"[{code}] {msg}")
        self.code = code


_lib = None


def _share_torch_runtime() -> None:
    # torch ships its own libamdhip64 (same SONAME as /opt/rocm's).  Loading
    # torch first makes this library bind to that one runtime, so device
    # pointers and streams are shared with torch in one process.
    try:
        import torch  # noqa: F401
    except Exception:
        pass


def load(share_torch: bool = True):
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise NeuroKmerError(NK_E_NO_DEVICE,
                             f"HIP library not built: {LIB_PATH} missing "
                             "(run `python -c 'import __graft_entry__ as g; g.build()'`)")
    if share_torch:
        _share_torch_runtime()
    L = C.CDLL(LIB_PATH, mode=C.RTLD_GLOBAL)
    vp, sz, u64, u32 = C.c_void_p, C.c_size_t, C.c_uint64, C.c_uint32
    P = C.POINTER
    sig = {
        "nk_opts_default": (None, [P(NkOpts)]),
        "nk_new": (vp, [sz, C.c_float, C.c_float, u32, C.c_double, sz, C.c_int, P(NkOpts)]),
        "nk_free": (None, [vp]),
        "nk_process_parallel": (C.c_int, [vp, vp, vp, sz]),
        "nk_process_parallel_device": (C.c_int, [vp, vp, vp, sz, sz, vp]),
        "nk_process_file_streaming": (C.c_int, [vp, C.c_char_p]),
        "nk_process_file_parallel": (C.c_int, [vp, C.c_char_p]),
        "nk_accumulate_device": (C.c_int, [vp, vp, vp, sz, sz, vp]),
        "nk_finalize": (C.c_int, [vp, C.c_int, vp]),
        "nk_willshaw_new": (vp, [sz, C.c_int]),
        "nk_willshaw_free": (None, [vp]),
        "nk_willshaw_store": (C.c_int, [vp, vp, sz]),
        "nk_willshaw_recall": (C.c_int, [vp, vp, sz, sz, vp]),
        "nk_willshaw_stored": (u64, [vp]),
        "nk_assoc_new": (vp, [sz, C.c_int]),
        "nk_assoc_free": (None, [vp]),
        "nk_assoc_pattern_size": (sz, [vp]),
        "nk_assoc_store_kmers": (C.c_int, [vp, vp, vp, sz]),
        "nk_assoc_find_similar": (C.c_long, [vp, u64, sz, vp, vp, sz]),
        "nk_finalize_slice": (C.c_int, [vp, C.c_int, vp, C.c_int, sz, sz, vp, sz, vp]),
        "nk_adopt_slices": (C.c_int, [vp, vp, sz, sz, vp]),
        "nk_slice_export": (C.c_int, [vp, C.c_int, vp, sz, sz, vp, sz, vp]),
        "nk_adopt_export": (C.c_int, [vp, vp, sz, sz, vp, sz, vp]),
        "nk_accumulate_device_from": (C.c_int, [vp, vp, vp, sz, sz, sz, vp]),
        "nk_top_kmers": (C.c_int, [vp, P(vp), P(sz)]),
        "nk_merge_top_kmers": (C.c_int, [vp, vp, sz, vp]),
        "nk_top_kmers_padded": (C.c_int, [vp, vp, sz, vp]),
        "nk_merge_top_kmers_padded": (C.c_int, [vp, vp, sz, sz, sz, P(C.c_int), vp]),
        "nk_top_abundant_neurons": (C.c_long, [vp, sz, P(NkTopRow)]),
        "nk_get_count": (C.c_int, [vp, u64, P(u32), P(C.c_int)]),
        "nk_get_counts": (C.c_int, [vp, vp, sz, vp, vp]),
        "nk_get_counts128": (C.c_int, [vp, vp, sz, vp, vp]),
        "nk_distinct_kmers": (C.c_long, [vp]),
        "nk_copy_kmer_per_neuron": (C.c_int, [vp, vp, sz]),
        "nk_process_sequence": (C.c_int, [vp, vp, sz]),
        "nk_total_spikes": (u64, [vp]),
        "nk_energy_used": (C.c_double, [vp]),
        "nk_set_steps": (None, [vp, u64]),
        "nk_get_steps": (u64, [vp]),
        "nk_pool_size": (sz, [vp]),
        "nk_k": (sz, [vp]),
        "nk_use_canonical": (C.c_int, [vp]),
        "nk_copy_currents": (C.c_int, [vp, vp, sz]),
        "nk_copy_spike_counts": (C.c_int, [vp, vp, sz]),
        "nk_copy_voltages": (C.c_int, [vp, vp, sz]),
        "nk_copy_refractory": (C.c_int, [vp, vp, sz]),
        "nk_device_currents": (vp, [vp]),
        "nk_settle": (C.c_int, [vp, vp]),
        "nk_exact_owner": (u32, [u64, u32]),
        "nk_exact_partition": (C.c_int, [vp, u32, P(u64), P(vp), P(vp), vp]),
        "nk_exact_adopt": (C.c_int, [vp, vp, vp, sz, vp]),
        "nk_device_kmer_per_neuron": (vp, [vp]),
        "nk_reset": (C.c_int, [vp]),
        "nk_reset_async": (C.c_int, [vp, vp]),
        "nk_last_timings": (C.c_int, [vp, P(C.c_char_p), P(C.c_float), C.c_int]),
        "nk_count_history": (C.c_int, [vp, P(C.c_float), C.c_int]),
        "nk_count_spans": (C.c_int, [vp, P(C.c_float), C.c_int]),
        "nk_count_stamps": (C.c_int, [vp, P(C.c_ulonglong), C.c_int]),
        "nk_set_stage_timing": (C.c_int, [vp, C.c_uint32]),
        "nk_diag_hash_ms": (C.c_int, [C.c_int, u64, u64, C.c_int, P(C.c_float)]),
        "nk_diag_hash_ms_w": (C.c_int, [C.c_int, u64, u64, C.c_int, C.c_int, P(C.c_float)]),
        "nk_diag_key_gather_ms": (C.c_int, [vp, C.c_int, P(C.c_float), P(u64)]),
        "nk_wire32": (C.c_int, [vp, vp, vp]),
        "nk_finalize_export": (C.c_int, [vp, C.c_int, vp, vp, sz, vp]),
        "nk_merge_export": (C.c_int, [vp, vp, sz, sz, sz, P(C.c_int), vp]),
        "nk_finalize_redo": (C.c_int, [vp, vp]),
        "nk_simulate_spikes_auto": (C.c_int, [vp]),
        "nk_comm_unique_id": (C.c_int, [vp]),
        "nk_comm_new": (vp, [vp, C.c_int, C.c_int, C.c_int]),
        "nk_comm_free": (None, [vp]),
        "nk_comm_forget": (None, [vp, vp]),
        "nk_loop_group_new": (vp, [C.c_int]),
        "nk_loop_group_free": (None, [vp]),
        "nk_comm_new_loopback": (vp, [vp, C.c_int, C.c_int]),
        "nk_finalize_dist": (C.c_int, [vp, vp, C.c_int, u64, sz, vp]),
        "nk_finalize_sliced_dist": (C.c_int, [vp, vp, C.c_int, u64, sz, vp]),
        "nk_last_error": (C.c_char_p, []),
        "nk_version": (C.c_char_p, []),
    }
    for name, (rt, args) in sig.items():
        f = getattr(L, name)
        f.restype = rt
        f.argtypes = args
    _lib = L
    return L


def last_error() -> str:
    return load().nk_last_error().decode(errors="replace")


def check(rc: int) -> int:
    if rc < 0:
        raise NeuroKmerError(rc, last_error())
    return rc
