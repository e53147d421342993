"""neurokmer_amd — MI355X-native NeuroKmer k-mer -> spike counting hot path.

Host mirror of the reference crate's public API (MrObadiahEJ/NeuroKmer,
src/lib.rs re-exports) over the C ABI in include/neurokmer.h.  Compute runs in
hand-written gfx950 kernels (neurokmer_amd/csrc/nk_kernels.hip); there is no
CPU fallback.
"""
from ._lib import NeuroKmerError, CLI_PATH, LIB_PATH  # noqa: F401

__all__ = ["SpikingKmerCounter", "NeuroKmerError", "stream_sequences", "records_to_arrays",
           "version"]


def __getattr__(name):
    # lazy: importing the package (e.g. for neurokmer_amd.synth) must not load HIP
    if name in ("SpikingKmerCounter", "EnergyTracker", "records_to_arrays"):
        from . import counter
        return getattr(counter, name)
    if name == "stream_sequences":
        from .fastx import stream_sequences
        return stream_sequences
    raise AttributeError(name)


def version() -> str:
    from . import _lib
    return _lib.load().nk_version().decode()
