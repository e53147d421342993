import os, sys
sys.path.insert(0, os.getcwd())
import numpy as np
import torch
import torch.distributed as dist
os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT="29533")
dist.init_process_group("gloo", rank=0, world_size=1)
from neurokmer_amd import SpikingKmerCounter, synth
from neurokmer_amd import dist as nkdist
from oracle import cbind
bases, offs = synth.make_records(400_000, 5, seed=44, repeats_per_mb=20000, motif_len=80, n_rate=0.002)
K, POOL = 25, 7001
d_b = torch.from_numpy(np.concatenate([bases, np.zeros(16, np.uint8)])).cuda()
d_o = torch.from_numpy(offs.astype(np.uint64).view(np.int64)).cuda()
torch.cuda.synchronize()
ref = cbind.OracleCounter(K, 1.0, 0.95, 2, 1.0, POOL, True)
ref.process_parallel_arrays(bases, offs)
print("ref", ref.top_abundant_neurons(5))
s = torch.cuda.current_stream().cuda_stream
c = SpikingKmerCounter(K, 1.0, 0.95, 2, 1.0, POOL, True)
c.process_parallel_device(d_b.data_ptr(), d_o.data_ptr(), offs.size - 1, int(offs[-1]), s)
print("process", c.top_abundant_neurons(5))
c.reset()
c.accumulate_device(d_b.data_ptr(), d_o.data_ptr(), offs.size - 1, int(offs[-1]), s)
wire = torch.empty(POOL, dtype=torch.int32, device="cuda")
c.wire32(wire.data_ptr(), s)
cap = 4096
seg = torch.zeros(1 + cap, dtype=torch.int64, device="cuda")
c.finalize_export(wire.data_ptr(), seg.data_ptr(), cap, False, s)
torch.cuda.synchronize()
h = int(seg[0].item())
print("hdr n", h & ((1 << 56) - 1), "flags", h >> 56, "first keys", seg[1:4].tolist())
redo = c.merge_export(seg.data_ptr(), 1, 1 + cap, cap, s)
print("redo", redo, c.top_abundant_neurons(5))
c.reset()
c.accumulate_device(d_b.data_ptr(), d_o.data_ptr(), offs.size - 1, int(offs[-1]), s)
c.finalize(False, s)
print("finalize", c.top_abundant_neurons(5))
pk = torch.zeros(1 + cap, dtype=torch.int64, device="cuda")
c.top_kmers_padded(pk.data_ptr(), cap, s)
torch.cuda.synchronize()
print("padded n", int(pk[0].item()))
dist.destroy_process_group()
