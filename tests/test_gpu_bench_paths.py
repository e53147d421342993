"""bench.py's N > 1 code path, end to end on one GPU, before the driver's
8-GPU run takes it: the shard setup, the in-library sliced finish with two
batches in flight, the max-over-ranks timing, `parity_ranks` (rank 0 counts
every rank's input in one handle and compares the N-rank step's final state,
N > 1) and the JSON line -- with the ranks as loopback threads (`--loopback
2`) and as a one-rank RCCL group (`--force-dist`: the communicator the 8-GPU
run builds, every collective an identity).  At a reduced input size: the line is
a rehearsal, not a measurement.
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("no GPU", allow_module_level=True)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*args):
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "3", "--warmup", "1",
           "--no-cpu-baseline", "--no-extras", "--bases", "20000000", "--settle", "0", *args]
    out = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    line = [ln for ln in out.stdout.strip().splitlines() if ln.startswith("{")][-1]
    return json.loads(line)


@pytest.mark.parametrize("args,world", [(("--loopback", "2"), 2), (("--force-dist",), 1)],
                         ids=["loopback2", "rccl1"])
def test_bench_multi_rank_path(args, world):
    d = _bench(*args)
    assert d["n_gpus"] == world
    assert d["config"]["finish"] == "sliced"
    assert d["inflight"] == 2
    assert d["value"] > 0 and d["ms_per_step"] > 0
    if world > 1:  # (one rank: nothing to compare across ranks)
        assert d["parity_ranks"]["all_equal"] is True, d["parity_ranks"]
        assert d["rehearsal"] is True
