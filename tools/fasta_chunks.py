"""The FASTA file path (nk_process_file_parallel: device FASTA parse, the
bench's end_to_end.fasta_file) at several ingest chunk sizes (NK_INGEST_CHUNK,
read per call): median of 5 calls each from the reset state, results checked
equal.  NK_AB_LIB selects another build for an A/B.
Usage: python tools/fasta_chunks.py [MiB ...]"""
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from neurokmer_amd import SpikingKmerCounter as Counter, synth  # noqa: E402

sizes = [int(a) for a in sys.argv[1:]] or [64, 32, 16, 8]
bases, offs = synth.make_records(115_000_000, 7, seed=synth.SEED, repeats_per_mb=64, motif_len=200)
path = "/dev/shm/nk_fasta_chunks.fa"
synth.write_fasta(path, bases, offs)
fsize = os.path.getsize(path)
g = Counter(31, 1.0, 0.95, 2, 1.0, 2_000_000, True)
ref = None
try:
    for rnd in range(2):
        for mib in sizes:
            os.environ["NK_INGEST_CHUNK"] = str(mib << 20)
            g.reset()
            g.process_file_parallel(path)  # warm (buffers sized for this chunk)
            ts = []
            for _ in range(5):
                g.reset()  # (each call from the reset state: results comparable)
                t = time.perf_counter()
                g.process_file_parallel(path)
                ts.append(time.perf_counter() - t)
            res = (g.energy.total_spikes(), g.top_abundant_neurons(20))
            ref = ref or res
            print(f"round {rnd} chunk {mib} MiB: median {statistics.median(ts) * 1e3:.2f} ms, best "
                  f"{min(ts) * 1e3:.2f} ms ({fsize / min(ts) / 1e9:.1f} GB/s), same {res == ref}", flush=True)
finally:
    os.environ.pop("NK_INGEST_CHUNK", None)
    g.close()
    os.unlink(path)
