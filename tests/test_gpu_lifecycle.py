"""Handle lifetime on the device: nk_free returns every buffer a handle
allocated.  Until round 4 it released 79 of the handle's 100 device buffers,
so a process that made many wide-pool handles (the config-5 path: wide-count
arena, split records, uniques tile lists, the u8 spike mirror) kept their
memory.  Each case builds and frees a handle several times and checks that
the device's free memory comes back.

Reference: src/spiking_hash.rs:40-48 (SpikingKmerCounter::new; Rust drops the
state with the value).
"""
import gc

import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("no GPU", allow_module_level=True)

from neurokmer_amd import SpikingKmerCounter, synth  # noqa: E402


@pytest.mark.parametrize("k,pool,width", [(63, 1 << 26, 128), (31, 20_000_000, 64), (31, 2_000_000, 64)])
def test_free_returns_device_memory(k, pool, width):
    bases, offs = synth.make_records(2_000_000, 5, seed=91, repeats_per_mb=2000, motif_len=120)

    def one_round():
        c = SpikingKmerCounter(k, 1.0, 0.95, 2, 1.0, pool, True, kmer_width=width)
        c.process_parallel_arrays(bases, offs)
        c.top_abundant_neurons(20)
        c.close()

    one_round()  # first use: the runtime's own allocations
    torch.cuda.synchronize()
    gc.collect()
    free0, _ = torch.cuda.mem_get_info()
    for _ in range(4):
        one_round()
    torch.cuda.synchronize()
    gc.collect()
    free1, _ = torch.cuda.mem_get_info()
    # a pool of 2^26 neurons alone holds > 1 GB of state per handle: a leak of
    # it (or of the count arena) over four handles is far past this slack
    assert free0 - free1 < 256 << 20, (free0, free1)
