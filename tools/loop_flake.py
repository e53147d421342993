"""Diagnostic: the loopback sliced finish's refine case (world 3, pool 2 M,
20000 LIF steps; tests/test_gpu_loopback.py), repeated in one process; each
rank's slice of the currents against the restatement, and on a mismatch the
neuron, the ranks' values, one handle's count of every record, and the
rank-local counts before the finish.  Usage: python tools/loop_flake.py [reps]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
from neurokmer_amd import SpikingKmerCounter, synth  # noqa: E402
from neurokmer_amd import dist as nkdist  # noqa: E402
from oracle import cbind  # noqa: E402
import test_gpu_loopback as T  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
world, width, pool, steps, cap = 3, 64, 2_000_000, int(os.environ.get("LF_STEPS", "20000")), 4096
k = 31
bases, offs = T._input(900_000, 81 + world, 7)
shards = T._shards(bases, offs, world)
ref = cbind.OracleCounter(k, 1.0, 0.95, 2, 1.0, pool, True, width=width)
ref.set_steps(steps)
ref.process_parallel_arrays(bases, offs, 4)
want = ref.currents()
local = []
for r in range(world):  # each rank's own count (no finish), for the diagnosis
    b, o = shards[r]
    g = SpikingKmerCounter(k, 1.0, 0.95, 2, 1.0, pool, True)
    g.process_parallel_arrays(b, o)
    local.append(g.currents())
    g.close()
print("rank-local sums == want:", bool(np.array_equal(sum(local), want)), flush=True)
bad = 0
for it in range(reps):
    def body(r, comm):
        b, o = shards[r]
        d_b, d_o = T._dev(b, o)
        c = SpikingKmerCounter(k, 1.0, 0.95, 2, 1.0, pool, True, kmer_width=width)
        c.set_steps(steps)
        c.accumulate_device(d_b.data_ptr(), d_o.data_ptr(), o.size - 1, b.size)
        nkdist.finalize_step_sliced(c, total_kmers=int(offs[-1]), cap=cap, comm=comm)
        torch.cuda.current_stream().synchronize()
        cur = c.currents()
        comm.forget(c)
        c.close()
        return cur
    got = T._run_ranks(world, body)
    for r in range(world):
        lo, hi, _ = nkdist.slice_bounds(pool, world, r)
        d = np.nonzero(got[r][lo:hi] != want[lo:hi])[0]
        if d.size:
            bad += 1
            i = int(d[0]) + lo
            print(f"rep {it} rank {r}: {d.size} mismatches, first neuron {i}: got {int(got[r][i])} "
                  f"want {int(want[i])} local {[int(x[i]) for x in local]}", flush=True)
print(f"reps {reps}, mismatching rank slices {bad}", flush=True)
